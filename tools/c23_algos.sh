#!/bin/bash
# configs 2 / 3: one bench line per (config, algo), per-kernel times
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
OUT=gpurun_out/${TAG:-c23a}
mkdir -p $OUT
for c in ${CFGS:-2 3}; do
  for al in ${ALGOS:-0 3}; do
    timeout -k 10 200 python bench.py --config $c --algo $al --steps 10 --warmup 2 --no-cpu-baseline > $OUT/c${c}_a${al}.log 2>&1 || exit $?
    python - $OUT/c${c}_a${al}.log "c=$c algo=$al" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["roofline"]["kernels_ms"]
print(f"{sys.argv[2]:12s} ms={d['ms_per_step']:.4f} frac={d['roofline']['frac']:.3f} " + " ".join(f"{n}={v*1e3:.1f}us" for n, v in k.items()))
PY
  done
done

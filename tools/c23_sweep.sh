#!/bin/bash
# configs 2 / 3 chunk-length sweep (EKS_CHUNK_LEN), one bench line per point
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
OUT=gpurun_out/c23sweep
mkdir -p $OUT
for c in ${CFGS:-2 3}; do
  for L in ${LENS:-0}; do
    if [ "$L" = 0 ]; then unset EKS_CHUNK_LEN; else export EKS_CHUNK_LEN=$L; fi
    timeout -k 10 200 python bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline > $OUT/c${c}_L${L}.log 2>&1 || exit $?
    python - $OUT/c${c}_L${L}.log "c=$c L=$L" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["roofline"]["kernels_ms"]
print(f"{sys.argv[2]:12s} ms={d['ms_per_step']:.4f} frac={d['roofline']['frac']:.3f} " + " ".join(f"{n}={v*1e3:.1f}us" for n, v in k.items()))
PY
  done
done

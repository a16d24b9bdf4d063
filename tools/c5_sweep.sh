#!/bin/bash
# config-5 tuning sweep: k_c1_elem waves per SIMD (EKS_C1_WPE) x chunk length
# (EKS_CHUNK_LEN); one bench line per point under gpurun_out/c5sweep/
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
OUT=gpurun_out/c5sweep
mkdir -p $OUT
for w in ${WPES:-0 2 3}; do
  for L in ${LENS:-0}; do
    if [ "$L" = 0 ]; then unset EKS_CHUNK_LEN; else export EKS_CHUNK_LEN=$L; fi
    EKS_C1_WPE=$w timeout -k 10 200 python bench.py --config 5 --steps 5 --warmup 1 --no-cpu-baseline > $OUT/w${w}_L${L}.log 2>&1 || exit $?
    python - $OUT/w${w}_L${L}.log "w=$w L=$L" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["roofline"]["kernels_ms"]
print(f"{sys.argv[2]:14s} ms={d['ms_per_step']:.3f} " + " ".join(f"{n}={v:.3f}" for n, v in k.items()))
PY
  done
done

#!/bin/bash
# configs x forced chunk length (EKS_CHUNK_LEN; 0 = the default rule)
set -o pipefail
mkdir -p gpurun_out
for L in ${LENS:-0 16 32 64}; do
  if [ $L = 0 ]; then unset EKS_CHUNK_LEN; else export EKS_CHUNK_LEN=$L; fi
  for c in ${CONFIGS:-3 5 2}; do
    timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/c${c}_L$L.log 2>&1 || exit $?
    python - gpurun_out/c${c}_L$L.log $c $L <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["roofline"]["kernels_ms"]
print(f"config {sys.argv[2]} L={sys.argv[3]:3s} ms={d['ms_per_step']:.3f} " + " ".join(f"{n}={v:.3f}" for n, v in k.items()))
PY
  done
done

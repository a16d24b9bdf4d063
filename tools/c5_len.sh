#!/bin/bash
# config 5 at forced chunk lengths (EKS_CHUNK_LEN: tuning only)
set -o pipefail
for L in ${LENS:-0 112 224 448}; do
  if [ "$L" = 0 ]; then unset EKS_CHUNK_LEN; else export EKS_CHUNK_LEN=$L; fi
  timeout -k 10 200 python bench.py --config 5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/c5_L$L.log 2>&1 || exit $?
  python - gpurun_out/c5_L$L.log $L <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("L", sys.argv[2], "ms", round(d["ms_per_step"], 4), {n: round(v, 4) for n, v in d["roofline"]["kernels_ms"].items()})
PY
done

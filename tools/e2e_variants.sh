#!/bin/bash
# Config-4 end-to-end (device fit + smooth) kernel times of each library
# variant (default + exp/*), alternated ROUNDS times on one box.
set -o pipefail
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
for r in $(seq ${ROUNDS:-2}); do
for v in default ${VARIANTS:-$(ls exp)}; do
  if [ "$v" = default ]; then unset EKS_LIB; else export EKS_LIB=exp/$v/libeks_hip.so; fi
  timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline > gpurun_out/e2e_$v.log 2>&1 || exit $?
  python - gpurun_out/e2e_$v.log $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
e = d["end_to_end"]
print(f"{sys.argv[2]:10s} e2e_ms={e['ms_per_step']:.3f} " + " ".join(f"{n}={v:.3f}" for n, v in e["kernels_ms"].items()))
PY
done
done

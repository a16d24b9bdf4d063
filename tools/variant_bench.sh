#!/bin/bash
# Bench config 4 (or $CONFIG) with each library variant: default + exp/*/
set -o pipefail
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
for v in default ${VARIANTS:-$(ls exp)}; do
  if [ "$v" = default ]; then unset EKS_LIB; else export EKS_LIB=exp/$v/libeks_hip.so; fi
  timeout -k 10 300 python bench.py --config ${CONFIG:-4} --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline > gpurun_out/vb_$v.log 2>&1 || exit $?
  python - gpurun_out/vb_$v.log $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["roofline"]["kernels_ms"]
print(f"{sys.argv[2]:10s} ms={d['ms_per_step']:.3f} frac={d['roofline']['frac']:.3f} " + " ".join(f"{n}={v:.3f}" for n, v in k.items()))
PY
done

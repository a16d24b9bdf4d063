#!/bin/bash
# Config-4 shard sizes (VIDEOS, default 128 256 1024) with each library
# variant (default + exp/*): step time and the algo-3 kernel times.
set -o pipefail
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
for nv in ${VIDEOS:-128 256 1024}; do
for v in default ${VARIANTS:-$(ls exp)}; do
  if [ "$v" = default ]; then unset EKS_LIB; else export EKS_LIB=exp/$v/libeks_hip.so; fi
  timeout -k 10 300 python bench.py --videos $nv --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/sv_${nv}_$v.log 2>&1 || exit $?
  python - gpurun_out/sv_${nv}_$v.log $nv $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"{sys.argv[2]:>5s} {sys.argv[3]:10s} ms={d['ms_per_step']:.3f} " + " ".join(f"{n}={v:.3f}" for n, v in d["roofline"]["kernels_ms"].items()))
PY
done; done

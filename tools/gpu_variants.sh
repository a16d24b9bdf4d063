#!/bin/bash
# config-4 timings (full batch and one 8-GPU shard) for the default library and exp/* variants
set -o pipefail
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
for v in default ${VARIANTS:-$(ls exp)}; do
  if [ "$v" = default ]; then unset EKS_LIB; else export EKS_LIB=exp/$v/libeks_hip.so; fi
  for nv in ${VIDEOS:-1024 128}; do
  args="--videos $nv"
    tag=$(echo $args | tr -d ' -')
    timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline $args > gpurun_out/v_${v}_$tag.log 2>&1 || exit $?
    python - gpurun_out/v_${v}_$tag.log "$v $args" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["roofline"]["kernels_ms"]
print(f"{sys.argv[2]:24s} ms={d['ms_per_step']:.3f} frac={d['roofline']['frac']:.3f} " + " ".join(f"{n}={v:.3f}" for n, v in k.items()))
PY
  done
done

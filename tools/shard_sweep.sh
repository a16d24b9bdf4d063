#!/bin/bash
# config 4 full batch and one 8-GPU shard (128 videos) x forced chunk length
set -o pipefail
mkdir -p gpurun_out
for V in ${VIDEOS:-1024 128}; do
for L in ${LENS:-0 96 128 192 256}; do
  if [ $L = 0 ]; then unset EKS_CHUNK_LEN; else export EKS_CHUNK_LEN=$L; fi
  timeout -k 10 300 python bench.py --videos $V --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/v${V}_L$L.log 2>&1 || exit $?
  python - gpurun_out/v${V}_L$L.log $V $L <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["roofline"]["kernels_ms"]
print(f"videos={sys.argv[2]} L={sys.argv[3]:3s} ms={d['ms_per_step']:.3f} value={d['value']:.3e} " + " ".join(f"{n}={v:.3f}" for n, v in k.items()))
PY
done
done

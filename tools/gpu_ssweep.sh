#!/bin/bash
# k3_coarse sub-part sweep (EKS_K3_S) at one 8-GPU shard (128 videos) and 512 videos
set -o pipefail
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
for nv in ${SS_VIDEOS:-128 512}; do
  for s in ${SS_S:-1 2 4 8}; do
    EKS_K3_S=$s timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --videos $nv > gpurun_out/s_${nv}_$s.log 2>&1 || exit $?
    python - gpurun_out/s_${nv}_$s.log "v=$nv S=$s" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["roofline"]["kernels_ms"]
print(f"{sys.argv[2]:12s} ms={d['ms_per_step']:.3f} " + " ".join(f"{n}={v:.3f}" for n, v in k.items()))
PY
  done
done

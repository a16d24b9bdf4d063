#!/bin/bash
# sequential vs wave-parallel chunk scans on the 1024- and 128-video workloads
mkdir -p gpurun_out
for V in 1024 128; do for W in 100000 0; do
  EKS_WAVE_SCAN_CHUNKS=$W timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --videos $V > gpurun_out/scan_${V}_$W.log 2>&1 || exit $?
  python -c "
import json
l=[x for x in open('gpurun_out/scan_${V}_$W.log') if x.startswith('{')][-1]; d=json.loads(l)
print('videos=$V wave_threshold=$W', 'ms=%.3f'%d['ms_per_step'], 'frac=%.3f'%d['roofline']['frac'], d['roofline']['kernels_ms'])"
done; done

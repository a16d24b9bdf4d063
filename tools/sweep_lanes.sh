#!/bin/bash
# chunk-count sweep of the time-parallel smoother on the bench workload
mkdir -p gpurun_out
for L in 262144 524288 1048576 2097152; do
  EKS_TARGET_LANES=$L timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline ${EXTRA} > gpurun_out/sweep_$L.log 2>&1 || exit $?
  python -c "
import json
l=[x for x in open('gpurun_out/sweep_$L.log') if x.startswith('{')][-1]; d=json.loads(l)
print($L, 'ms=%.3f'%d['ms_per_step'], 'frac=%.3f'%d['roofline']['frac'], d['roofline']['kernels_ms'])"
done

#!/bin/bash
# algo-3 two-stream split: its GPU test, then config 4 with EKS_A3_SPLIT =
# 0 (one stream) / 1 (B's chain on the side stream) / 2 (A's scans + final
# on the high-priority side stream), and a kernel trace of mode 2
# (results: profiles/r02/split/)
set -o pipefail
OUT=gpurun_out/${1:-split}
mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread \
  -k "split_streams or batch_slices or coarse_subparts" > $OUT/pytest_split.log 2>&1 || exit $?
tail -1 $OUT/pytest_split.log
for m in 0 1 2; do
  EKS_A3_SPLIT=$m timeout -k 10 300 python bench.py > $OUT/bench_m$m.log 2>&1 || exit $?
  python -c "
import json
d=json.loads([x for x in open('$OUT/bench_m$m.log') if x.startswith('{')][-1])
print('mode $m', d['ms_per_step'], d['roofline']['frac'], d['roofline']['kernels_ms'])"
done
EKS_A3_SPLIT=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python bench.py --steps 3 --warmup 1 > $OUT/prof.log 2>&1 || exit $?
find $OUT/prof -name '*kernel_trace.csv' | head -1

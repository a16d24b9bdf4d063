#!/bin/bash
# One GPU session of a round: GPU tests, smoke, the bench lines of configs
# 4/2/3/5 and the rocprofv3 passes (trace + FETCH/WRITE counters) of the
# default workload.  Every GPU step has its own time limit and the chain
# stops at the first failure.  Usage: tools/gpu_round.sh TAG [skip-tests]
set -o pipefail
TAG=${1:-r02}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit $?
  tail -1 $OUT/pytest_gpu.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
fi
timeout -k 10 400 python bench.py > $OUT/bench.log 2>&1 || exit $?
tail -c 600 $OUT/bench.log
for c in 2 3 5; do
  timeout -k 10 400 python bench.py --config $c --steps 5 --warmup 1 > $OUT/bench_c$c.log 2>&1 || exit $?
done
bash tools/gpu_profile.sh $TAG || exit $?

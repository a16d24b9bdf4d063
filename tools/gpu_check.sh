#!/bin/bash
# One GPU session: parity tests, smoke, benches.  Every GPU step has its own
# time limit and the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 900 python -m pytest tests -m gpu -q --maxfail=30 > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1 || exit $?
for c in 2 3 5; do
  timeout -k 10 400 python bench.py --config $c --steps 5 --warmup 1 > gpurun_out/bench_c$c.log 2>&1 || exit $?
done
timeout -k 10 600 python bench.py --steps 5 --warmup 1 --algo 1 --no-cpu-baseline > gpurun_out/bench_algo1.log 2>&1 || exit $?

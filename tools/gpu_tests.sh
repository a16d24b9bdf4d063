#!/bin/bash
# the whole -m gpu suite in one process (per-test time limit), then smoke
set -o pipefail
OUT=gpurun_out/${TAG:-tests}
mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -2 $OUT/smoke.log

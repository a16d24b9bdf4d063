#!/bin/bash
# algo 3 check: targeted parity tests, then config-4 variants (tools/variant_bench.sh)
set -o pipefail
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "${PYTEST_K:-fused or long or edge or yev}" > gpurun_out/a3_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/a3_pytest.log; tail -1 gpurun_out/a3_pytest.log; [ $rc -eq 0 ] || exit $rc
STEPS=5 bash tools/variant_bench.sh

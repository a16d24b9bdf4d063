set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out/sel
EKS_LIB=exp/s6/libeks_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_fit_mask.py tests/test_gpu_parity.py -k "fit or mask or select" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/sel/pytest_s6.log 2>&1 || { tail -20 gpurun_out/sel/pytest_s6.log; exit 1; }
tail -2 gpurun_out/sel/pytest_s6.log
EKS_LIB=exp/s8/libeks_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_fit_mask.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/sel/pytest_s8.log 2>&1 || { tail -20 gpurun_out/sel/pytest_s8.log; exit 1; }
tail -2 gpurun_out/sel/pytest_s8.log
VARIANTS="s6 s8" ROUNDS=2 bash tools/e2e_variants.sh 2>&1 | tee gpurun_out/sel/e2e.txt

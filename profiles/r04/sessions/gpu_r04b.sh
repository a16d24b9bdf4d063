#!/bin/bash
# round-4 session b: runtime-n / wide-fit tests, then the look-back A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_rt.py tests/test_gpu_fit_mask.py tests/test_gpu_parity.py \
  -k "rt or runtime or multicam or mask or wide" -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/rt.log 2>&1
rc=$?; tail -3 gpurun_out/rt.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python bench.py --config 3 --cameras 6 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c3v6.log 2>&1 || exit $?
tail -c 600 gpurun_out/bench_c3v6.log
TAG=lb0 TESTS=tests/test_gpu_chain.py LIBS="default exp/r03/libeks_hip.so" VIDEOS="1024 512 256 128" bash tools/gpu_ab.sh || exit $?
TAG=lb1 BENCH_ARGS="--a3-lb 1" VIDEOS="512 256 128" bash tools/gpu_ab.sh || exit $?
TAG=lb2 BENCH_ARGS="--a3-lb 2" VIDEOS="1024 512 256" bash tools/gpu_ab.sh

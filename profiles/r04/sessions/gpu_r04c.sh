#!/bin/bash
# round-4 session c: runtime-n fixes, config 3 at 6 cameras, k3_bwd variants, PMC passes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_rt.py tests/test_gpu_fit_mask.py -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/rt.log 2>&1
rc=$?; tail -n 3 gpurun_out/rt.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for V in 6 4; do
  timeout -k 10 200 python bench.py --config 3 --cameras $V --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c3v$V.log 2>&1 || exit $?
  python - gpurun_out/bench_c3v$V.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(d["config"].get("cameras"), "smooth ms", round(d["ms_per_step"], 4), d["roofline"]["kernels_ms"])
print("   e2e", round(d["end_to_end"]["ms_per_step"], 4), d["end_to_end"]["kernels_ms"])
PY
done
TAG=var LIBS="default exp/r03/libeks_hip.so exp/varA/libeks_hip.so exp/varB/libeks_hip.so" VIDEOS="1024 128" bash tools/gpu_ab.sh || exit $?
TAG=r04 bash tools/gpu_pmc.sh

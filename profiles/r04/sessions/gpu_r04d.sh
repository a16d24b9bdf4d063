#!/bin/bash
# round-4 session d: fit / runtime-n tests, configs 2/3 (V = 4, 6), prefetch-depth variants
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_rt.py tests/test_gpu_fit_mask.py tests/test_gpu_parity.py -k "rt or runtime or fit or mask or wide" -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/fit.log 2>&1
rc=$?; tail -n 3 gpurun_out/fit.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for c in "2" "3 --cameras 4" "3 --cameras 6"; do
  timeout -k 10 200 python bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench.log 2>&1 || exit $?
  python - gpurun_out/bench.log "$c" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = lambda k: {n: round(v, 4) for n, v in k.items()}
print("c", sys.argv[2], "smooth ms", round(d["ms_per_step"], 4), r(d["roofline"]["kernels_ms"]))
print("   e2e", round(d["end_to_end"]["ms_per_step"], 4), r(d["end_to_end"]["kernels_ms"]))
PY
done
TAG=vard LIBS="default exp/r03/libeks_hip.so exp/varD3/libeks_hip.so" VIDEOS="1024 256 128" bash tools/gpu_ab.sh

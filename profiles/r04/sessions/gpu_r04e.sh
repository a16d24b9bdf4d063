#!/bin/bash
# round-4 session e: fit / runtime-n tests, configs 2 / 3 (4 and 6 cameras) / 4 / 5
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_rt.py tests/test_gpu_fit_mask.py tests/test_gpu_parity.py -k "rt or runtime or fit or mask or wide" -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/fit.log 2>&1
rc=$?; tail -n 3 gpurun_out/fit.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for c in "2" "3 --cameras 4" "3 --cameras 6" "3 --cameras 8" "5" "4 --videos 128" "4"; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench.log 2>&1 || exit $?
  python - gpurun_out/bench.log "$c" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = lambda k: {n: round(v, 4) for n, v in k.items()}
print("c", sys.argv[2], "ms", round(d["ms_per_step"], 4), "frac", d["roofline"].get("frac"), r(d["roofline"]["kernels_ms"]))
if d.get("end_to_end"): print("   e2e", round(d["end_to_end"]["ms_per_step"], 4), r(d["end_to_end"]["kernels_ms"]))
PY
done

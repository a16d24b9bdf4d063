#!/bin/bash
# Round-end evidence of the shipped build: the whole -m gpu suite, smoke, and
# bench lines (default config 4 with its CPU baseline; the 8-GPU shard size;
# configs 2, 3 (4 / 6 / 8 cameras) and 5).  Every GPU step has its own limit.
set -o pipefail
OUT=gpurun_out/${TAG:-final}
mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -n 3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -n 2 $OUT/smoke.log
timeout -k 10 400 python bench.py > $OUT/bench_default.log 2>&1 || exit $?
tail -c 400 $OUT/bench_default.log; echo
for c in "4 --videos 128" "4 --videos 256" "2" "3" "3 --cameras 6" "3 --cameras 8" "5"; do
  name=$(echo "c$c" | tr -d ' -' )
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_$name.log 2>&1 || exit $?
  python - $OUT/bench_$name.log "$c" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = lambda k: {n: round(v, 4) for n, v in k.items()}
print("c", sys.argv[2], "ms", round(d["ms_per_step"], 4), "frac", d["roofline"].get("frac"), r(d["roofline"]["kernels_ms"]))
if d.get("end_to_end"): print("   e2e", round(d["end_to_end"]["ms_per_step"], 4), r(d["end_to_end"]["kernels_ms"]))
PY
done

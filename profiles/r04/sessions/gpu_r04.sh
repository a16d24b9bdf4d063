#!/bin/bash
# Round-4 GPU iteration: chosen tests first (TESTS, default the chain tests),
# then the whole -m gpu suite (FULL=1), then config-4 bench lines at the
# given video counts (VIDEOS, default "1024 128").  Every GPU step has its
# own time limit; the chain stops at the first failure.
set -o pipefail
TAG=${TAG:-r04}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
if [ -n "${TESTS-tests/test_gpu_chain.py}" ]; then
  timeout -k 10 400 python -u -m pytest ${TESTS-tests/test_gpu_chain.py} -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_sel.log 2>&1
  rc=$?; tail -3 $OUT/pytest_sel.log; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$FULL" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
  rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
  tail -2 $OUT/smoke.log
fi
for mode in ${MODES-0}; do
for nv in ${VIDEOS-1024 128}; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --videos $nv --a3-mode $mode > $OUT/bench_v${nv}_m$mode.log 2>&1 || exit $?
  python - $OUT/bench_v${nv}_m$mode.log $nv $mode <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["roofline"]["kernels_ms"]
print(f"v{sys.argv[2]:5s} m{sys.argv[3]} ms={d['ms_per_step']:.3f} frac={d['roofline']['frac']:.3f} " + " ".join(f"{n}={v:.3f}" for n, v in k.items())
      + f" e2e={d['end_to_end']['ms_per_step']:.3f}")
PY
done
done
for c in ${CONFIGS-}; do
  timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline > $OUT/bench_c$c.log 2>&1 || exit $?
  python - $OUT/bench_c$c.log $c <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
e = d.get("end_to_end") or {}
print(f"c{sys.argv[2]} ms={d['ms_per_step']:.4f} " + " ".join(f"{n}={v:.4f}" for n, v in d["roofline"]["kernels_ms"].items()))
if e: print(f"   e2e={e['ms_per_step']:.4f} " + " ".join(f"{n}={v:.4f}" for n, v in e["kernels_ms"].items()))
PY
done

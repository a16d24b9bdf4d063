#!/bin/bash
# A/B of library variants on config 4 (bench lines, kernel times):
#   LIBS="default exp/r03/libeks_hip.so ..." VIDEOS="1024 128" bash tools/gpu_ab.sh
set -o pipefail
OUT=gpurun_out/${TAG:-ab}
mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
  rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
i=0
for lib in ${LIBS:-default}; do
  i=$((i+1))
  for nv in ${VIDEOS:-1024 128}; do
    if [ "$lib" = "default" ]; then unset EKS_LIB; else export EKS_LIB=$lib; fi
    timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --videos $nv $BENCH_ARGS > $OUT/b${i}_v$nv.log 2>&1 || exit $?
    python - $OUT/b${i}_v$nv.log "$lib" $nv <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["roofline"]["kernels_ms"]
print(f"{sys.argv[2][-30:]:30s} v{sys.argv[3]:5s} ms={d['ms_per_step']:.3f} frac={d['roofline']['frac']:.3f} " + " ".join(f"{n}={v:.3f}" for n, v in k.items()) + f" e2e={d['end_to_end']['ms_per_step']:.3f}")
PY
  done
done
unset EKS_LIB
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

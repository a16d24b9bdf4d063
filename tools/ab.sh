#!/bin/bash
# A/B on one box: optional GPU tests, then config-4 bench lines of each
# library variant (default = eks_amd/lib; NAME = exp/NAME/libeks_hip.so),
# alternated REPS times per video count.
#   PYTEST="tests/test_gpu_chain.py" PYTEST_LIB=NAME VARIANTS="r05 default" VIDEOS="1024 128" REPS=2 bash tools/ab.sh
set -o pipefail
mkdir -p gpurun_out/ab
export PYTHONDONTWRITEBYTECODE=1
if [ -n "$PYTEST" ]; then
  # PYTEST_LIB=NAME: the tests against exp/NAME/libeks_hip.so
  [ -n "$PYTEST_LIB" ] && export EKS_LIB=exp/$PYTEST_LIB/libeks_hip.so
  timeout -k 10 900 python -u -m pytest $PYTEST -m gpu -x -q --timeout 300 --timeout-method thread \
      ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/ab/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/ab/pytest.log; [ $rc -eq 0 ] || exit $rc
  unset EKS_LIB
fi
for rep in $(seq ${REPS:-1}); do
  for nv in ${VIDEOS:-1024 128}; do
    for v in ${VARIANTS:-default}; do
      if [ "$v" = default ]; then unset EKS_LIB; else export EKS_LIB=exp/$v/libeks_hip.so; fi
      log=gpurun_out/ab/${v}_v${nv}_r${rep}.log
      timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline \
          --videos $nv ${BENCH_ARGS} > $log 2>&1 || { echo "bench failed: $log"; tail -5 $log; exit 1; }
      python - $log "$v v$nv r$rep" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["roofline"]["kernels_ms"]
e = d.get("end_to_end") or {}
print(f"{sys.argv[2]:22s} ms={d['ms_per_step']:.4f} frac={d['roofline']['frac']:.4f} "
      + " ".join(f"{n}={v:.4f}" for n, v in k.items())
      + (f" e2e={e['ms_per_step']:.3f}" if e else ""))
PY
    done
  done
done

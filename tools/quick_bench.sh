#!/bin/bash
# quick GPU check: fit tests + configs 4/3/2 without CPU baseline; one summary line each
set -o pipefail
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
if [ "${PYTEST_K:-fit}" != none ]; then
  timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -m gpu -q -k "${PYTEST_K:-fit}" > gpurun_out/pytest_q.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_q.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
for c in ${CONFIGS:-4 3 2}; do
  timeout -k 10 400 python bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/qb$c.log 2>&1 || exit $?
  python - gpurun_out/qb$c.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
e = d.get("end_to_end") or {}
print(sys.argv[1], f"value={d['value']:.3e} ms={d['ms_per_step']:.3f} frac={d['roofline']['frac']:.3f}",
      f"e2e={e.get('value', 0):.3e} e2e_ms={e.get('ms_per_step', 0):.3f}", e.get("kernels_ms"))
PY
done

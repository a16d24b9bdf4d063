#!/bin/bash
# config 5: two chunks per K1 lane (k_c1_elem2, default) vs one (EKS_C1_PAIR=0)
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out/pair
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pair/pytest.log 2>&1 || { tail -30 gpurun_out/pair/pytest.log; exit 1; }
tail -1 gpurun_out/pair/pytest.log
for i in 1 2; do for pr in 1 0; do
  EKS_C1_PAIR=$pr timeout -k 10 300 python bench.py --config 5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/pair/c5_$pr.log 2>&1 || exit $?
  python - gpurun_out/pair/c5_$pr.log "pair=$pr" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], f"ms={d['ms_per_step']:.4f} maxd={d.get('max_abs_diff_vs_cpu')}", d["roofline"]["kernels_ms"])
PY
done; done

#!/bin/bash
# algo 3 (chained two-pass) check: its GPU tests, then config-4 timings (full
# batch and one 8-GPU shard).  Every GPU step has its own time limit.
set -o pipefail
OUT=gpurun_out/${TAG:-a3}
mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "${PYTEST_K:-algo3 or fused_batch or time_parallel_long or yev_handoff or fused_edge}" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for nv in ${VIDEOS:-1024 128}; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --videos $nv > $OUT/bench_v$nv.log 2>&1 || exit $?
  python - $OUT/bench_v$nv.log $nv <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["roofline"]["kernels_ms"]
print(f"videos {sys.argv[2]:5s} ms={d['ms_per_step']:.3f} frac={d['roofline']['frac']:.3f} e2e={d['end_to_end']['ms_per_step']:.3f} " + " ".join(f"{n}={v:.3f}" for n, v in k.items()))
PY
done

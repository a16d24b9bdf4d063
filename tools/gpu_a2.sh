#!/bin/bash
# algo 2 (few long trajectories) check: its GPU tests, then configs 2 / 3 / 5
# bench lines (optionally a chunk-length sweep: LENS="8 16 ...").
set -o pipefail
OUT=gpurun_out/${TAG:-a2}
mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1
if [ -z "$NOTEST" ]; then
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_timeshard.py tests/test_gpu_configs.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "${PYTEST_K:-time_parallel or filter_only or algo2 or fused_batch or pupil or multicam or fit_then or segments or configs or config}" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
for c in ${CFGS:-2 3 5}; do
  for L in ${LENS:-0}; do
    if [ "$L" = 0 ]; then unset EKS_CHUNK_LEN; else export EKS_CHUNK_LEN=$L; fi
    timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline > $OUT/c${c}_L$L.log 2>&1 || exit $?
    python - $OUT/c${c}_L$L.log "c=$c L=$L" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["roofline"]["kernels_ms"]
print(f"{sys.argv[2]:12s} ms={d['ms_per_step']:.4f} frac={d['roofline']['frac']:.3f} " + " ".join(f"{n}={v*1e3:.1f}us" for n, v in k.items()))
PY
  done
done

#!/bin/bash
# quick config-4 timings: full batch and one 8-GPU shard (128 videos), algo auto
set -o pipefail
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
if [ -n "$PYTEST_K" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "$PYTEST_K" > gpurun_out/q_pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/q_pytest.log; [ $rc -eq 0 ] || exit $rc
fi
for nv in ${VIDEOS:-1024 128}; do
  args="--videos $nv"
  tag=$(echo $args | tr -d ' -')
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline $args > gpurun_out/q_$tag.log 2>&1 || exit $?
  python - gpurun_out/q_$tag.log "$args" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["roofline"]["kernels_ms"]
print(f"{sys.argv[2]:16s} ms={d['ms_per_step']:.3f} frac={d['roofline']['frac']:.3f} " + " ".join(f"{n}={v:.3f}" for n, v in k.items()))
PY
done

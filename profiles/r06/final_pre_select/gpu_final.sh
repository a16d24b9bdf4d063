#!/bin/bash
# Round-end evidence of the shipped build (TAG=r06 by default):
# -m gpu suite, smoke, the default bench line (CPU baseline), configs 2 / 3
# (4, 6, 8 cameras) / 5, the 4- / 8-GPU shard sizes, T = 4 000, rocprofv3
# kernel traces + FETCH / WRITE passes of config 4 and its 8-GPU shard, and
# the SQ / VALU passes of algo 3.
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
TAG=${TAG:-r06}
O=gpurun_out/final_$TAG; mkdir -p $O
PART=${PART:-all}  # bench | prof | all (each part stays under gpurun's 64 MiB copy-back)
summ() { python - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["roofline"]["kernels_ms"]
e = d.get("end_to_end") or {}
print(f"{sys.argv[2]:12s} ms={d['ms_per_step']:.4f} frac={d['roofline']['frac']:.3f} " + " ".join(f"{n}={v:.4f}" for n, v in k.items()), flush=True)
if e: print(f"{'':12s} e2e={e['ms_per_step']:.4f} " + " ".join(f"{n}={v:.4f}" for n, v in e["kernels_ms"].items()), flush=True)
PY
}
if [ "$PART" != prof ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import time, ctypes; t = time.time(); ctypes.CDLL('eks_amd/lib/libeks_hip.so'); print('dlopen s', round(time.time() - t, 3))" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -2 $O/smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench_default.log 2>&1 || exit $?
tail -c 300 $O/bench_default.log; echo
summ $O/bench_default.log default
for c in "4 --videos 128" "4 --videos 256" "2" "3" "3 --cameras 6" "3 --cameras 8" "5"; do
  name=$(echo "c$c" | tr -d ' -')
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_$name.log 2>&1 || exit $?
  summ $O/bench_$name.log $name
done
for lib in default; do
  if [ $lib = default ]; then unset EKS_LIB; else export EKS_LIB=exp/$lib/libeks_hip.so; fi
  timeout -k 10 300 python bench.py --frames 4000 --steps 20 --warmup 5 --no-cpu-baseline > $O/t4000_$lib.log 2>&1 || exit $?
  summ $O/t4000_$lib.log t4000_$lib
done
unset EKS_LIB
fi
if [ "$PART" != bench ]; then
bash tools/gpu_profile.sh ${TAG}c4 > $O/profile_c4.log 2>&1 || exit $?
BENCH_ARGS="--videos 128" bash tools/gpu_profile.sh ${TAG}v128 > $O/profile_v128.log 2>&1 || exit $?
TAG=$TAG bash tools/gpu_pmc.sh > $O/pmc.log 2>&1 || exit $?
BENCH_ARGS="--config 5" bash tools/gpu_profile.sh ${TAG}c5 > $O/profile_c5.log 2>&1 || exit $?
BENCH_ARGS="--config 3 --cameras 6" bash tools/gpu_profile.sh ${TAG}c3v6 > $O/profile_c3v6.log 2>&1 || exit $?
fi
echo done

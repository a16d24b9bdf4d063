# A/B: k3_fwd member ring depth 3 / 4 (k3fd3 / k3fd4) and one algo-3 block per
# CU (bpc + EKS_A3_BLOCKS_PER_CU=1) against the default; the default's
# trajectory-fastest accumulation from 64 trajectories on (fit tests, v128 /
# v256 / config 4 end to end).
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/g9; mkdir -p $O
summ() { python - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["roofline"]["kernels_ms"]
e = d.get("end_to_end") or {}
print(f"{sys.argv[2]:16s} ms={d['ms_per_step']:.4f} " + " ".join(f"{n}={v:.4f}" for n, v in k.items()), flush=True)
if e: print(f"{'':16s} e2e={e['ms_per_step']:.4f} " + " ".join(f"{n}={v:.4f}" for n, v in e["kernels_ms"].items()), flush=True)
PY
}
timeout -k 10 300 python -u -m pytest tests/test_gpu_fit_mask.py tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() {  # name, lib, env..., -- bench args
  local name=$1 lib=$2; shift 2
  if [ $lib = default ]; then unset EKS_LIB; else export EKS_LIB=exp/$lib/libeks_hip.so; fi
  timeout -k 10 300 env "$@" > $O/$name.log 2>&1 || exit $?
  summ $O/$name.log $name
}
for rep in 1 2; do
  run def_v1024 default python bench.py --steps 20 --warmup 3 --no-cpu-baseline
  run fd3_v1024 k3fd3 python bench.py --steps 20 --warmup 3 --no-cpu-baseline
  run fd4_v1024 k3fd4 python bench.py --steps 20 --warmup 3 --no-cpu-baseline
  run def_v128 default python bench.py --videos 128 --steps 20 --warmup 3 --no-cpu-baseline
  run fd3_v128 k3fd3 python bench.py --videos 128 --steps 20 --warmup 3 --no-cpu-baseline
  run bpc1_v128 bpc EKS_A3_BLOCKS_PER_CU=1 python bench.py --videos 128 --steps 20 --warmup 3 --no-cpu-baseline
  run def_v256 default python bench.py --videos 256 --steps 20 --warmup 3 --no-cpu-baseline
  run bpc1_v256 bpc EKS_A3_BLOCKS_PER_CU=1 python bench.py --videos 256 --steps 20 --warmup 3 --no-cpu-baseline
done
echo done

set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
for nv in 8 16 32 64 1024; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --videos $nv --algo 3 > gpurun_out/mall_$nv.log 2>&1 || exit $?
  python - gpurun_out/mall_$nv.log $nv <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["roofline"]["kernels_ms"]; u = d["roofline"]["units_per_launch"]
print(sys.argv[2], f"ms={d['ms_per_step']:.3f}", " ".join(f"{n}={v:.4f}({v*1e-3/u*1e12:.2f}ps)" for n, v in k.items()))
PY
done

set -o pipefail
mkdir -p gpurun_out
for L in 0 48 64 128 160; do
  if [ $L = 0 ]; then unset EKS_CHUNK_LEN; else export EKS_CHUNK_LEN=$L; fi
  timeout -k 10 300 python bench.py --videos 128 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/v128_L$L.log 2>&1 || exit $?
  python - gpurun_out/v128_L$L.log $L <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["roofline"]["kernels_ms"]
print(f"v128 L={sys.argv[2]:3s} ms={d['ms_per_step']:.3f} value={d['value']:.3e} " + " ".join(f"{n}={v:.3f}" for n, v in k.items()))
PY
done

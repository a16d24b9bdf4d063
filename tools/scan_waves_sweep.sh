set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out/sw
for c in 2 3 5; do for sw in 0 4 1; do
  if [ $sw = 0 ]; then unset EKS_SCAN_WAVES; else export EKS_SCAN_WAVES=$sw; fi
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/sw/c${c}_$sw.log 2>&1 || exit $?
  python - gpurun_out/sw/c${c}_$sw.log "c$c sw$sw" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["roofline"]["kernels_ms"]
print(f"{sys.argv[2]:10s} ms={d['ms_per_step']:.4f} " + " ".join(f"{n}={v:.4f}" for n, v in k.items()))
PY
done; done

# PCA Jacobi with reciprocal / rsqrt + Newton rotation parameters: the fit
# tests (multicam vs host, goldens, wide fit) and the camera configurations'
# end to end.
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/g17; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_rt.py tests/test_gpu_fit_mask.py tests/test_gpu_configs.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for c in 3 "3 --cameras 6" "3 --cameras 8" 2; do
  name=$(echo "c$c" | tr -d ' -')
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > $O/$name.log 2>&1 || exit $?
  python - $O/$name.log $name <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
e = d["end_to_end"]
print(f"{sys.argv[2]:14s} ms={d['ms_per_step']:.4f} e2e={e['ms_per_step']:.4f} " + " ".join(f"{n}={v:.4f}" for n, v in e["kernels_ms"].items()), flush=True)
PY
done
echo done

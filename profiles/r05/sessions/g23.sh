# The wide PCA.s round-robin schedule tabulated in LDS: fit tests, then the
# 6- / 8-camera configurations end to end.
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/g23; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_rt.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
for c in "3 --cameras 6" "3 --cameras 8"; do
  name=$(echo "c$c" | tr -d ' -')
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > $O/${name}_$rep.log 2>&1 || exit $?
  python - $O/${name}_$rep.log $name <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
e = d["end_to_end"]
k = e["kernels_ms"]
print(f"{sys.argv[2]:14s} ms={d['ms_per_step']:.4f} e2e={e['ms_per_step']:.4f} k_fitw_final={k.get('k_fitw_final')} k_fit_merge={k.get('k_fit_merge')}", flush=True)
PY
done
done
echo done

# The split selection's bin step folded into k_sel_hist (last block per row):
# the selection / fit tests, then configs 2 / 3 / 6 cameras end to end.
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/g25; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fit_mask.py tests/test_gpu_parity.py tests/test_gpu_rt.py tests/test_gpu_configs.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
for c in 2 3 "3 --cameras 6"; do
  name=$(echo "c$c" | tr -d ' -')
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > $O/${name}_$rep.log 2>&1 || exit $?
  python - $O/${name}_$rep.log $name <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
e = d["end_to_end"]
k = e["kernels_ms"]
print(f"{sys.argv[2]:14s} ms={d['ms_per_step']:.4f} e2e={e['ms_per_step']:.4f} " + " ".join(f"{n}={v:.4f}" for n, v in k.items() if 'sel' in n), flush=True)
PY
done
done
echo done

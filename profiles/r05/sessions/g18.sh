# PCA Jacobi stopping rule: default (1e-30 or no further decrease) and jt34
# (1e-34 or no further decrease): fit tests + the camera configurations.
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/g18; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_rt.py tests/test_gpu_configs.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for lib in default jt34; do
  if [ $lib = default ]; then unset EKS_LIB; else export EKS_LIB=exp/$lib/libeks_hip.so; fi
  for c in 3 "3 --cameras 6" "3 --cameras 8"; do
    name=$(echo "c$c" | tr -d ' -')
    timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > $O/${lib}_$name.log 2>&1 || exit $?
    python - $O/${lib}_$name.log ${lib}_$name <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
e = d["end_to_end"]
k = e["kernels_ms"]
print(f"{sys.argv[2]:20s} e2e={e['ms_per_step']:.4f} final={k.get('k_fit_final', k.get('k_fitw_final'))}", flush=True)
PY
  done
done
echo done

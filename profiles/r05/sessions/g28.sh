# One-block-per-row selection with 512 threads (sb512) against 256: the
# selection / mask tests, then config 4 / T = 4 000 end to end.
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/g28; mkdir -p $O
export EKS_LIB=exp/sb512/libeks_hip.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_fit_mask.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  for lib in default sb512; do
    if [ $lib = default ]; then unset EKS_LIB; else export EKS_LIB=exp/$lib/libeks_hip.so; fi
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/${lib}_v1024_$rep.log 2>&1 || exit $?
    python - $O/${lib}_v1024_$rep.log ${lib} <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
e = d["end_to_end"]
print(f"{sys.argv[2]:8s} e2e={e['ms_per_step']:.4f} k_fit_select={e['kernels_ms']['k_fit_select']:.4f} k_fit_worst={e['kernels_ms']['k_fit_worst']:.4f}", flush=True)
PY
  done
  unset EKS_LIB
done
echo done

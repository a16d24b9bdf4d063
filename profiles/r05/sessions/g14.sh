# k_c0_shared with LDS-staged member loads (default) and k_c1_elem at three
# waves per SIMD for the pupil shape (c1w3, built before the staging).
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/g14; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_pupil.py tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
summ() { python - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["roofline"]["kernels_ms"]
f = d.get("flop_roofline") or {}
print(f"{sys.argv[2]:12s} ms={d['ms_per_step']:.4f} ksum={sum(k.values()):.4f} " + (f"flopfrac={f['frac']:.3f} " if f else "") + " ".join(f"{n}={v:.4f}" for n, v in k.items()), flush=True)
PY
}
for rep in 1 2; do
  for lib in default c1w3; do
    if [ $lib = default ]; then unset EKS_LIB; else export EKS_LIB=exp/$lib/libeks_hip.so; fi
    timeout -k 10 300 python bench.py --config 5 --steps 10 --warmup 3 --no-cpu-baseline > $O/${lib}_c5_$rep.log 2>&1 || exit $?
    summ $O/${lib}_c5_$rep.log ${lib}_c5
  done
  unset EKS_LIB
done
echo done

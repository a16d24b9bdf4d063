# A/B of the wave-merged selection histograms (haggb0) and the register-
# resident long-row forms (haggb1: 1024 x 10, haggb2: 512 x 20) against the
# g5 library, end to end at config 4 / T = 4000 / config 2.
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/g7; mkdir -p $O
summ() { python - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
e = d.get("end_to_end") or {}
print(f"{sys.argv[2]:16s} ms={d['ms_per_step']:.4f} e2e={e.get('ms_per_step', 0):.4f} " + " ".join(f"{n}={v:.4f}" for n, v in e.get("kernels_ms", {}).items() if n.startswith(("k_fit", "k_sel"))), flush=True)
PY
}
export EKS_LIB=exp/haggb0/libeks_hip.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_fit_mask.py tests/test_gpu_parity.py  -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_haggb0.log 2>&1 || { tail -20 $O/pytest_haggb0.log; exit 1; }
tail -1 $O/pytest_haggb0.log
for rep in 1 2; do
for lib in haggb0 g5lib haggb1 haggb2; do
  export EKS_LIB=exp/$lib/libeks_hip.so
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/${lib}_v1024_$rep.log 2>&1 || exit $?
  summ $O/${lib}_v1024_$rep.log ${lib}_v1024
  timeout -k 10 300 python bench.py --frames 4000 --steps 10 --warmup 2 --no-cpu-baseline > $O/${lib}_t4000_$rep.log 2>&1 || exit $?
  summ $O/${lib}_t4000_$rep.log ${lib}_t4000
done
done
for lib in haggb0 g5lib; do
  export EKS_LIB=exp/$lib/libeks_hip.so
  timeout -k 10 300 python bench.py --config 2 --steps 20 --warmup 3 --no-cpu-baseline > $O/${lib}_c2.log 2>&1 || exit $?
  summ $O/${lib}_c2.log ${lib}_c2
done
echo done

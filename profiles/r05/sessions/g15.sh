# Config 5: chunks per thread of the chained chunk scans (EKS_SCAN_QT; the
# default picks 4 for the sweep's 64 x 17 858 chunks).
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/g15; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_pupil.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
summ() { python - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["roofline"]["kernels_ms"]
print(f"{sys.argv[2]:12s} ms={d['ms_per_step']:.4f} ksum={sum(k.values()):.4f} " + " ".join(f"{n}={v:.4f}" for n, v in k.items()), flush=True)
PY
}
for rep in 1 2; do
  for q in 0 2 8 16; do
    if [ $q = 0 ]; then unset EKS_SCAN_QT; else export EKS_SCAN_QT=$q; fi
    timeout -k 10 300 python bench.py --config 5 --steps 10 --warmup 3 --no-cpu-baseline > $O/q${q}_c5_$rep.log 2>&1 || exit $?
    summ $O/q${q}_c5_$rep.log q${q}_c5
  done
  unset EKS_SCAN_QT
done
echo done

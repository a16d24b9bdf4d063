# A/B of the rebuilt library (accumulation dedupe + YEV ring depth 4) against
# the g5 library and the YEV depth-2 variant, interleaved on one box.
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/g6; mkdir -p $O
summ() { python - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["roofline"]["kernels_ms"]
e = d.get("end_to_end") or {}
print(f"{sys.argv[2]:14s} ms={d['ms_per_step']:.4f} " + " ".join(f"{n}={v:.4f}" for n, v in k.items()), flush=True)
if e: print(f"{'':14s} e2e={e['ms_per_step']:.4f} " + " ".join(f"{n}={v:.4f}" for n, v in e["kernels_ms"].items()), flush=True)
PY
}
timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
for lib in default g5lib yevd2; do
  if [ $lib = default ]; then unset EKS_LIB; else export EKS_LIB=exp/$lib/libeks_hip.so; fi
  for v in 1024 128; do
    timeout -k 10 300 python bench.py --videos $v --steps 20 --warmup 3 --no-cpu-baseline > $O/${lib}_v${v}_$rep.log 2>&1 || exit $?
    summ $O/${lib}_v${v}_$rep.log ${lib}_v${v}
  done
done
done
echo done

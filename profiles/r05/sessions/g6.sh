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
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
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
for lib in sel2; do
  export EKS_LIB=exp/$lib/libeks_hip.so
  timeout -k 10 300 python -u -m pytest tests/test_gpu_fit_mask.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_$lib.log 2>&1 || { tail -20 $O/pytest_$lib.log; exit 1; }
  tail -1 $O/pytest_$lib.log
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/${lib}_v1024.log 2>&1 || exit $?
  summ $O/${lib}_v1024.log ${lib}_v1024
done
unset EKS_LIB
for L in 8 16 24 32; do
  EKS_CHUNK_LEN=$L timeout -k 10 300 python bench.py --config 2 --steps 20 --warmup 3 --no-cpu-baseline > $O/c2_L$L.log 2>&1 || exit $?
  summ $O/c2_L$L.log c2_L$L
  EKS_CHUNK_LEN=$L timeout -k 10 300 python bench.py --config 3 --steps 20 --warmup 3 --no-cpu-baseline > $O/c3_L$L.log 2>&1 || exit $?
  summ $O/c3_L$L.log c3_L$L
done
echo done

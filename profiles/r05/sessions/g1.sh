set -o pipefail
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/g1; mkdir -p $O
summ() { python - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["roofline"]["kernels_ms"]
print(f"{sys.argv[2]:12s} ms={d['ms_per_step']:.3f} frac={d['roofline']['frac']:.3f} " + " ".join(f"{n}={v:.3f}" for n, v in k.items()), flush=True)
PY
}
for v in 1024 128; do
  for lib in base fast1 pf mm; do
    if [ $lib = base ]; then unset EKS_LIB; else export EKS_LIB=exp/$lib/libeks_hip.so; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --videos $v > $O/${lib}_v$v.log 2>&1 || exit $?
    summ $O/${lib}_v$v.log ${lib}_v$v
  done
done
unset EKS_LIB
EKS_LIB=exp/stamps/libeks_hip.so timeout -k 10 300 python tools/stamps_run.py > $O/stamps1024.log 2>&1 || exit $?
cat $O/stamps1024.log
EKS_LIB=exp/stamps/libeks_hip.so timeout -k 10 300 python tools/stamps_run.py --videos 128 > $O/stamps128.log 2>&1 || exit $?
cat $O/stamps128.log
EKS_LIB=exp/pf/libeks_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_chain.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_pf.log 2>&1
rc=$?; tail -3 $O/pytest_pf.log; exit $rc

# Round 5 A/B call 2: the candidate build's GPU tests, config-4 A/B (round-4
# library vs candidate vs ring-depth variants), phase stamps, configs 2 / 3.
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/g2; mkdir -p $O
summ() { python - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["roofline"]["kernels_ms"]
e = d.get("end_to_end") or {}
print(f"{sys.argv[2]:12s} ms={d['ms_per_step']:.4f} frac={d['roofline']['frac']:.3f} " + " ".join(f"{n}={v:.4f}" for n, v in k.items()), flush=True)
if e: print(f"{'':12s} e2e={e['ms_per_step']:.4f} " + " ".join(f"{n}={v:.4f}" for n, v in e["kernels_ms"].items()), flush=True)
PY
}
EKS_LIB=exp/cur/libeks_hip.so timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/pytest_cur.log 2>&1
rc=$?; tail -5 $O/pytest_cur.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for v in 1024 128; do
  for lib in base cur d3 d4; do
    export EKS_LIB=exp/$lib/libeks_hip.so
    timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --videos $v > $O/${lib}_v$v.log 2>&1 || exit $?
    summ $O/${lib}_v$v.log ${lib}_v$v
  done
done
export EKS_LIB=exp/stamps/libeks_hip.so
timeout -k 10 300 python tools/stamps_run.py > $O/stamps1024.log 2>&1 || exit $?
cat $O/stamps1024.log
timeout -k 10 300 python tools/stamps_run.py --videos 128 > $O/stamps128.log 2>&1 || exit $?
cat $O/stamps128.log
for lib in base cur; do
  export EKS_LIB=exp/$lib/libeks_hip.so
  for c in "2" "3" "3 --cameras 6"; do
    name=$(echo "c$c" | tr -d ' -')
    timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline > $O/${lib}_$name.log 2>&1 || exit $?
    summ $O/${lib}_$name.log ${lib}_$name
  done
done

# Round 5 A/B call 3: candidate (eager aggregates, k3_bwd look-back for every
# batch, ring depth 3, register-resident selection, straight-line mask
# accumulation) vs round 4 and single-knob variants; stamps; configs 2/3/5;
# a rocprofv3 kernel trace of the candidate at config 4.
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/g3; mkdir -p $O
summ() { python - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["roofline"]["kernels_ms"]
e = d.get("end_to_end") or {}
print(f"{sys.argv[2]:12s} ms={d['ms_per_step']:.4f} frac={d['roofline']['frac']:.3f} " + " ".join(f"{n}={v:.4f}" for n, v in k.items()), flush=True)
if e: print(f"{'':12s} e2e={e['ms_per_step']:.4f} " + " ".join(f"{n}={v:.4f}" for n, v in e["kernels_ms"].items()), flush=True)
PY
}
EKS_LIB=exp/cur3/libeks_hip.so timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/pytest_cur3.log 2>&1
rc=$?; tail -4 $O/pytest_cur3.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for v in 1024 128; do
  for lib in base cur3 noeager nolball; do
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
export EKS_LIB=exp/cur3/libeks_hip.so
for c in "2" "3" "3 --cameras 6" "5"; do
  name=$(echo "c$c" | tr -d ' -')
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline > $O/cur3_$name.log 2>&1 || exit $?
  summ $O/cur3_$name.log cur3_$name
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_c4 -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/prof_c4.log 2>&1 || exit $?
echo profiled

# Round 5 A/B call 4: the default build (early chain polls, ring 3, one-wave
# wide PCA, register-resident selection) -- GPU tests, config-4 A/B against
# round 4 and no-early-poll, stamps, configs 2/3/5, rocprofv3 trace + HBM passes.
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/g4; mkdir -p $O
summ() { python - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["roofline"]["kernels_ms"]
e = d.get("end_to_end") or {}
print(f"{sys.argv[2]:12s} ms={d['ms_per_step']:.4f} frac={d['roofline']['frac']:.3f} " + " ".join(f"{n}={v:.4f}" for n, v in k.items()), flush=True)
if e: print(f"{'':12s} e2e={e['ms_per_step']:.4f} " + " ".join(f"{n}={v:.4f}" for n, v in e["kernels_ms"].items()), flush=True)
PY
}
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -4 $O/pytest.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -2 $O/smoke.log
for v in 1024 128; do
  for lib in base default noearly; do
    if [ $lib = default ]; then unset EKS_LIB; else export EKS_LIB=exp/$lib/libeks_hip.so; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --videos $v > $O/${lib}_v$v.log 2>&1 || exit $?
    summ $O/${lib}_v$v.log ${lib}_v$v
  done
done
export EKS_LIB=exp/stamps/libeks_hip.so
timeout -k 10 300 python tools/stamps_run.py > $O/stamps1024.log 2>&1 || exit $?
cat $O/stamps1024.log
unset EKS_LIB
for c in "2" "3" "3 --cameras 6" "3 --cameras 8" "5"; do
  name=$(echo "c$c" | tr -d ' -')
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline > $O/$name.log 2>&1 || exit $?
  summ $O/$name.log $name
done
TAG=r05 bash tools/gpu_profile.sh > $O/profile.log 2>&1 || exit $?
echo profiled; cat gpurun_out/prof_r05/status.txt

# Warm replays sized by time (>= W and >= ~30 ms) before the timed region, at
# the driver's --steps 20 --warmup 5: config 4 and its shards, configs 2 / 5.
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/g22; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_pupil.py tests/test_gpu_rt.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
summ() { python - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["roofline"]["kernels_ms"]
e = d.get("end_to_end") or {}
print(f"{sys.argv[2]:10s} ms={d['ms_per_step']:.4f} frac={d['roofline']['frac']:.3f} ksum={sum(k.values()):.4f} warm={d.get('warmup_replays')} e2e={e.get('ms_per_step', 0):.4f}", flush=True)
PY
}
for rep in 1 2; do
  for v in 1024 128 256; do
    timeout -k 10 300 python bench.py --videos $v --steps 20 --warmup 5 --no-cpu-baseline > $O/v${v}_$rep.log 2>&1 || exit $?
    summ $O/v${v}_$rep.log v${v}
  done
  for c in 2 5 "3 --cameras 6"; do
    name=$(echo "c$c" | tr -d ' -')
    timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > $O/${name}_$rep.log 2>&1 || exit $?
    summ $O/${name}_$rep.log $name
  done
done
# k_fit_worst's member ring 2 / 8 frames deep (default 4): config 4 end to end
for rep in 1 2; do
  for lib in default wd2 wd8; do
    if [ $lib = default ]; then unset EKS_LIB; else export EKS_LIB=exp/$lib/libeks_hip.so; fi
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/${lib}_e2e_$rep.log 2>&1 || exit $?
    python - $O/${lib}_e2e_$rep.log ${lib} <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
e = d["end_to_end"]
print(f"{sys.argv[2]:8s} e2e={e['ms_per_step']:.4f} k_fit_worst={e['kernels_ms']['k_fit_worst']:.4f}", flush=True)
PY
  done
  unset EKS_LIB
done
echo done

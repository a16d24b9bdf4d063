# (1) the bench with its warm-up replays right before the timed region, at
# the driver's --steps 20 --warmup 5; (2) config 5 with the pupil sweep's
# y / ev ring in SGPRs (c1w0) and the same at 3 waves per SIMD (c1w3).
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/g12; mkdir -p $O
summ() { python - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["roofline"]["kernels_ms"]
f = d.get("flop_roofline") or {}
print(f"{sys.argv[2]:16s} ms={d['ms_per_step']:.4f} frac={d['roofline']['frac']:.3f} ksum={sum(k.values()):.4f} " + (f"flopfrac={f['frac']:.3f} " if f else "") + " ".join(f"{n}={v:.4f}" for n, v in k.items()), flush=True)
PY
}
for lib in c1w0 c1w3; do
  export EKS_LIB=exp/$lib/libeks_hip.so
  timeout -k 10 300 python -u -m pytest tests/test_gpu_pupil.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_$lib.log 2>&1 || { tail -20 $O/pytest_$lib.log; exit 1; }
  tail -1 $O/pytest_$lib.log
done
unset EKS_LIB
for rep in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/def_v1024_$rep.log 2>&1 || exit $?
  summ $O/def_v1024_$rep.log def_v1024
  python -c "import json; d=json.loads(open('$O/def_v1024_$rep.log').read().strip().splitlines()[-1]); print('   e2e', round(d['end_to_end']['ms_per_step'], 4), d['end_to_end'].get('hip_graph'))"
  timeout -k 10 300 python bench.py --videos 128 --steps 20 --warmup 5 --no-cpu-baseline > $O/def_v128_$rep.log 2>&1 || exit $?
  summ $O/def_v128_$rep.log def_v128
  for lib in default c1w0 c1w3; do
    if [ $lib = default ]; then unset EKS_LIB; else export EKS_LIB=exp/$lib/libeks_hip.so; fi
    timeout -k 10 300 python bench.py --config 5 --steps 10 --warmup 2 --no-cpu-baseline > $O/${lib}_c5_$rep.log 2>&1 || exit $?
    summ $O/${lib}_c5_$rep.log ${lib}_c5
  done
  unset EKS_LIB
done
timeout -k 10 300 python bench.py --videos 256 --steps 20 --warmup 5 --no-cpu-baseline > $O/def_v256.log 2>&1 || exit $?
summ $O/def_v256.log def_v256
for c in 2 3 "3 --cameras 6"; do
  name=$(echo "c$c" | tr -d ' -')
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_$name.log 2>&1 || exit $?
  python - $O/bench_$name.log $name <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
e = d["end_to_end"]
print(f"{sys.argv[2]:12s} ms={d['ms_per_step']:.4f} e2e={e['ms_per_step']:.4f} graph={e.get('hip_graph')} ksum_e2e={sum(e['kernels_ms'].values()):.4f}", flush=True)
PY
done
echo done

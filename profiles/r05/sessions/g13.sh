# The full rebuild (pupil sweep's y / ev ring in SGPRs, fit accumulation
# lanes, bench warm-up replays, end-to-end graph): the whole -m gpu suite
# first (a failure ends the call), then the bench lines.
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/g13; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
summ() { python - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["roofline"]["kernels_ms"]
f = d.get("flop_roofline") or {}
e = d.get("end_to_end") or {}
print(f"{sys.argv[2]:12s} ms={d['ms_per_step']:.4f} frac={d['roofline']['frac']:.3f} ksum={sum(k.values()):.4f} " + (f"flopfrac={f['frac']:.3f} " if f else "") + (f"e2e={e['ms_per_step']:.4f} graph={e.get('hip_graph')} " if e else "") + " ".join(f"{n}={v:.4f}" for n, v in k.items()), flush=True)
PY
}
for rep in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/v1024_$rep.log 2>&1 || exit $?
  summ $O/v1024_$rep.log v1024
  timeout -k 10 300 python bench.py --videos 128 --steps 20 --warmup 5 --no-cpu-baseline > $O/v128_$rep.log 2>&1 || exit $?
  summ $O/v128_$rep.log v128
  timeout -k 10 300 python bench.py --config 5 --steps 10 --warmup 2 --no-cpu-baseline > $O/c5_$rep.log 2>&1 || exit $?
  summ $O/c5_$rep.log c5
done
timeout -k 10 300 python bench.py --videos 256 --steps 20 --warmup 5 --no-cpu-baseline > $O/v256.log 2>&1 || exit $?
summ $O/v256.log v256
for c in 2 3 "3 --cameras 6" "3 --cameras 8"; do
  name=$(echo "c$c" | tr -d ' -')
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > $O/$name.log 2>&1 || exit $?
  summ $O/$name.log $name
done
echo done

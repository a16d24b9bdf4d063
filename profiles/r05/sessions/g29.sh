# Per-rank shard sizes of the driver's 1/2/4/8-GPU scaling runs, each on one
# GPU at the driver's --steps 20 --warmup 5 (v1024 / v512 / v256 / v128), and
# config 4 over 100 timed steps (steady state).
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/g29; mkdir -p $O
summ() { python - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["roofline"]["kernels_ms"]
print(f"{sys.argv[2]:10s} ms={d['ms_per_step']:.4f} value={d['value']:.3e} frac={d['roofline']['frac']:.3f} ksum={sum(k.values()):.4f} warm={d.get('warmup_replays')}", flush=True)
PY
}
for v in 1024 512 256 128; do
  timeout -k 10 300 python bench.py --videos $v --steps 20 --warmup 5 --no-cpu-baseline > $O/v$v.log 2>&1 || exit $?
  summ $O/v$v.log v$v
done
timeout -k 10 300 python bench.py --steps 100 --warmup 5 --no-cpu-baseline > $O/v1024_s100.log 2>&1 || exit $?
summ $O/v1024_s100.log v1024_s100
echo done

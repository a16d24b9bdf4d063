# Graph replay vs eager launches of the same step (config 4, its 8- / 4-GPU
# shards): ms_per_step against the per-kernel event sum.
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/g10; mkdir -p $O
summ() { python - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["roofline"]["kernels_ms"]
print(f"{sys.argv[2]:16s} ms={d['ms_per_step']:.4f} ksum={sum(k.values()):.4f} " + " ".join(f"{n}={v:.4f}" for n, v in k.items()), flush=True)
PY
}
for rep in 1 2; do
for v in 1024 128 256; do
  timeout -k 10 300 python bench.py --videos $v --steps 20 --warmup 3 --no-cpu-baseline > $O/graph_v$v.log 2>&1 || exit $?
  summ $O/graph_v$v.log graph_v$v
  timeout -k 10 300 python bench.py --videos $v --steps 20 --warmup 3 --no-cpu-baseline --no-graph > $O/eager_v$v.log 2>&1 || exit $?
  summ $O/eager_v$v.log eager_v$v
  timeout -k 10 300 python bench.py --videos $v --steps 100 --warmup 3 --no-cpu-baseline > $O/graph100_v$v.log 2>&1 || exit $?
  summ $O/graph100_v$v.log graph100_v$v
done
done
echo done

# Complete per-kernel breakdowns of the small configurations' end to end
# (16 profiler marks per call: the split-selection fit's merge and final
# kernels were past the old 8).
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/g16; mkdir -p $O
for c in 2 3 "3 --cameras 6" "3 --cameras 8" "4 --videos 128"; do
  name=$(echo "c$c" | tr -d ' -')
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > $O/$name.log 2>&1 || exit $?
  python - $O/$name.log $name <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
e = d["end_to_end"]
print(f"{sys.argv[2]:14s} ms={d['ms_per_step']:.4f} e2e={e['ms_per_step']:.4f} ksum={sum(e['kernels_ms'].values()):.4f} " + " ".join(f"{n}={v:.4f}" for n, v in e["kernels_ms"].items()), flush=True)
PY
done
echo done

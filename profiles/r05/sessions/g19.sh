# Compiled r = 3, n = 12 kernels (six cameras): the whole -m gpu suite, then
# the 6-camera configuration (smoothing and end to end) and config 3.
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/g19; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for c in "3 --cameras 6" 3 "3 --cameras 6"; do
  name=$(echo "c$c" | tr -d ' -')
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > $O/$name.log 2>&1 || exit $?
  python - $O/$name.log $name <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
e = d["end_to_end"]
print(f"{sys.argv[2]:14s} ms={d['ms_per_step']:.4f} algo={d['config'].get('algo')} e2e={e['ms_per_step']:.4f} smooth: " + " ".join(f"{n}={v:.4f}" for n, v in d["roofline"]["kernels_ms"].items()), flush=True)
PY
done
echo done

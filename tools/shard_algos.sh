set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
for nv in 128 256 512; do for a in 2 3; do
  timeout -k 10 300 python bench.py --videos $nv --algo $a --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/sh_${nv}_$a.log 2>&1 || exit $?
  python - gpurun_out/sh_${nv}_$a.log $nv $a <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], sys.argv[3], f"ms={d['ms_per_step']:.3f}", d["roofline"]["kernels_ms"])
PY
done; done

#!/bin/bash
# Infinity Cache (MALL) probe for the algo-3 member re-read: per-kernel time
# per keypoint-timestep and L2->fabric read requests (all / destined for
# DRAM) at batch sizes whose per-step traffic fits the 256 MB MALL (16 videos:
# 109 MB of members) or not (64, 1024 videos).  Each step re-smooths the same
# batch, so a resident batch is re-read from the MALL by BOTH member passes.
set -o pipefail
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
OUT=gpurun_out/${TAG:-mall}
mkdir -p $OUT
for nv in ${VIDEOS:-16 64 1024}; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --videos $nv --algo 3 > $OUT/bench_v$nv.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --kernel-include-regex 'k3_' --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum \
      -d /tmp/mall_v$nv -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --videos $nv --algo 3 > $OUT/pmc_v$nv.log 2>&1 || exit $?
  f=$(find /tmp/mall_v$nv -name "*counter_collection.csv" | head -1)
  [ -n "$f" ] || { echo "no counter file for $nv videos"; exit 1; }
  python3 - "$f" $nv $OUT/bench_v$nv.log >> $OUT/summary.txt <<'PY'
import csv, json, sys
from collections import defaultdict
f, nv, bl = sys.argv[1], sys.argv[2], sys.argv[3]
acc = defaultdict(lambda: defaultdict(list))
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0].replace("eks::", "")
    acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
if not acc:
    sys.exit("no counter rows")
d = json.loads(open(bl).read().strip().splitlines()[-1])
u = d["roofline"]["units_per_launch"]
print(f"videos={nv} units={u} ms={d['ms_per_step']:.4f} frac={d['roofline']['frac']:.3f}")
for k, v in d["roofline"]["kernels_ms"].items():
    # the bench's per-kernel names are the kernel names (k3_fwd, k3_bwd, ...)
    c = acc[k] if k in acc else {}
    rq = sum(c.get("TCC_EA0_RDREQ_sum", [0])) / max(1, len(c.get("TCC_EA0_RDREQ_sum", [1])))
    dr = sum(c.get("TCC_EA0_RDREQ_DRAM_sum", [0])) / max(1, len(c.get("TCC_EA0_RDREQ_DRAM_sum", [1])))
    print(f"  {k:10s} {v*1e-3/u*1e12:8.2f} ps/kp-ts  rdreq/kp-ts {rq/u:7.3f}  dram rdreq/kp-ts {dr/u:7.3f}")
PY
done
cat $OUT/summary.txt

#!/bin/bash
# Effective shader clock of the algo-3 kernels per library variant: one
# rocprofv3 --pmc pass (GRBM_GUI_ACTIVE, SQ_WAVE_CYCLES, SQ_BUSY_CYCLES) per
# variant over a short bench; clock = GRBM_GUI_ACTIVE / 8 XCDs / duration.
#   VARIANTS="r05 default" BENCH_ARGS="--videos 1024" bash tools/clk.sh
set -o pipefail
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out/clk
for v in ${VARIANTS:-default}; do
  if [ "$v" = default ]; then unset EKS_LIB; else export EKS_LIB=exp/$v/libeks_hip.so; fi
  rm -rf /tmp/clk_$v
  timeout -s KILL 120 rocprofv3 --kernel-include-regex 'k3_' --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU \
      -d /tmp/clk_$v -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 \
      --no-cpu-baseline --no-graph ${BENCH_ARGS} > gpurun_out/clk/$v.log 2>&1 || { echo "rocprof failed $v"; tail -5 gpurun_out/clk/$v.log; exit 1; }
  for f in $(find /tmp/clk_$v -name "*counter_collection.csv" -o -name "*kernel_trace.csv"); do
    cp $f gpurun_out/clk/${v}_$(basename $f)
  done
  python3 - gpurun_out/clk/${v}_run_counter_collection.csv $v <<'PY'
import csv, sys
from collections import defaultdict
per = defaultdict(float); dur = {}
for row in csv.DictReader(open(sys.argv[1])):
    k = row["Kernel_Name"].split("(")[0].split("<")[0].split("::")[-1]
    per[(row["Dispatch_Id"], k, row["Counter_Name"])] += float(row["Counter_Value"] or 0)
    if "Start_Timestamp" in row and row.get("End_Timestamp"):
        dur[(row["Dispatch_Id"], k)] = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9
acc = defaultdict(lambda: defaultdict(list))
for (d, k, c), v in per.items():
    acc[k][c].append(v)
for k in sorted(acc):
    c = {n: sum(v) / len(v) for n, v in acc[k].items()}
    ds = [t for (d, kk), t in dur.items() if kk == k]
    t = sum(ds) / len(ds) if ds else float("nan")
    print(f"{sys.argv[2]:8s} {k:8s} dur {t*1e3:.3f} ms  clock {c['GRBM_GUI_ACTIVE']/8/t/1e9:.2f} GHz  "
          f"waves/SIMD {4*c['SQ_WAVE_CYCLES']/(c['GRBM_GUI_ACTIVE']/8)/1024:.2f}  VALU insts {c['SQ_INSTS_VALU']:.3g}")
PY
done

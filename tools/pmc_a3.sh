#!/bin/bash
# Counters of the algo-3 kernels (k3_fwd / k3_bwd), one --pmc pass each
# (MI355X_MICROARCH.md: counters in their own runs, kernel-trace only).
set -o pipefail
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
OUT=gpurun_out/${TAG:-pmc_a3}; RAW=/tmp/pmc_a3
mkdir -p $OUT $RAW
rm -f $OUT/summary.txt
i=0
for ctr in ${CTRS:-FETCH_SIZE WRITE_SIZE SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE}; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-include-regex "${KRX:-k3_}" --pmc $ctr -d $RAW/p$i -o run --output-format csv -- \
      python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > $OUT/p$i.log 2>&1 || exit $?
  f=$(find $RAW/p$i -name "*counter_collection.csv" | head -1)
  python3 - "$f" "$ctr" <<'PY' >> $OUT/summary.txt
import csv, sys, collections
acc = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if r["Counter_Name"] != sys.argv[2]:
        continue
    acc[r["Kernel_Name"].split("(")[0].replace("void ", "")[:70]].append(float(r["Counter_Value"]))
for k, v in acc.items():
    print(f"{sys.argv[2]:22s} {k:70s} n={len(v):3d} avg={sum(v)/len(v):.6g}")
PY
done
cat $OUT/summary.txt

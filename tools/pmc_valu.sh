#!/bin/bash
# VALU issue counters of the smoother kernels (separate --pmc passes).
set -o pipefail
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
OUT=gpurun_out/pmc_valu; RAW=/tmp/pmc_valu
mkdir -p $OUT $RAW
i=0
for ctr in "VALUBusy" "SQ_INSTS_VALU" "SQ_INSTS_SALU" "SQ_INSTS_VALU_FMA_F64" "SQ_WAVES"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-include-regex 'k_c[0-9]|k_fit' --pmc $ctr -d $RAW/p$i -o run --output-format csv -- \
      python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > $OUT/p$i.log 2>&1 || exit $?
  f=$(find $RAW/p$i -name "*counter_collection.csv" | head -1)
  python3 - "$f" "$ctr" <<'PY' >> $OUT/summary.txt
import csv, sys, collections
acc = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    acc[r["Kernel_Name"].split("(")[0].replace("void ", "")[:60]].append(float(r["Counter_Value"]))
for k, v in acc.items():
    print(f"{sys.argv[2]:24s} {k:60s} {sum(v)/len(v):.4g}")
PY
done
cat $OUT/summary.txt

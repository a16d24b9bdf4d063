#!/bin/bash
# PMC passes for the algo-3 kernels of the default bench (config 4, N = 1):
# one rocprofv3 --pmc run per counter group (MI355X_MICROARCH.md: at most 8
# SQ / 4 TCC / 2 GRBM counters per pass), kernel-filtered, 2 timed steps.
# Raw output stays in /tmp on the box; the counter CSVs are copied back.
#   TAG=r04 BENCH_ARGS="--videos 1024" bash tools/gpu_pmc.sh
set -o pipefail
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
TAG=${TAG:-pmc}
RAW=/tmp/pmc_$TAG
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT $RAW
RX=${RX:-'k3_'}
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
pass() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-include-regex "$RX" --pmc "$@" -d $RAW/$name -o run \
      --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-graph \
      ${BENCH_ARGS} > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc ($*)" >> $OUT/status.txt
  for f in $(find $RAW/$name -name "*counter_collection.csv"); do
    sz=$(stat -c %s "$f")
    if [ "$sz" -lt 20000000 ]; then cp "$f" $OUT/${name}_$(basename $f); fi
  done
  return $rc
}
pass sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY \
     SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT || exit $?
pass lvl SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS \
     SQ_INSTS_SALU GRBM_GUI_ACTIVE || true
pass valu VALUBusy || true
pass mem MemUnitStalled || true
pass fetch FETCH_SIZE || exit $?
pass write WRITE_SIZE || exit $?
python3 tools/pmc_summary.py $OUT > $OUT/summary.txt 2>&1 || true

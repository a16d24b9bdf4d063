#!/bin/bash
# rocprofv3 kernel-trace summary + HBM counters (separate --pmc passes, as
# MI355X_MICROARCH.md prescribes) of the default bench workload.  Raw
# profiler output goes to /tmp on the box; only summaries are copied back.
set -o pipefail
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
TAG=${1:-r01}
RAW=/tmp/prof_$TAG
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT $RAW
step() {  # name, timeout, rocprof args...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t rocprofv3 "$@" -d $RAW/$name -o run --output-format csv -- \
      python3 bench.py --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $OUT/status.txt
  (cd $RAW && find $name -type f -printf "%s %p\n") >> $OUT/files.txt
  for f in $(find $RAW/$name -name "*stats.csv" -o -name "*counter_collection.csv" -o -name "*agent_info.csv"); do
    sz=$(stat -c %s "$f")
    if [ "$sz" -lt 20000000 ]; then cp "$f" $OUT/${name}_$(basename $f); fi
  done
  return $rc
}
RX='k_c[0-9]|k3_|k_model|k_smooth_seq|k_fit'
if [ -z "$NO_TRACE" ]; then step trace 600 --kernel-trace --stats || exit $?; fi
STEPS=2 step pmc_fetch 600 --kernel-include-regex "$RX" --pmc FETCH_SIZE || exit $?
STEPS=2 step pmc_write 600 --kernel-include-regex "$RX" --pmc WRITE_SIZE || exit $?

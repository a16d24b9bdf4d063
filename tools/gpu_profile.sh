#!/bin/bash
# rocprofv3 kernel-trace summary + HBM counters (separate --pmc passes, as
# MI355X_MICROARCH.md prescribes) of the default bench workload.
set -o pipefail
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
TAG=${1:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
ARGS="--steps 5 --warmup 1 --no-cpu-baseline"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py $ARGS > $OUT/bench_trace.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline > $OUT/pmc_fetch.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline > $OUT/pmc_write.log 2>&1 || exit $?
find $OUT -name "*.csv" | head -50 > $OUT/files.txt

#!/bin/bash
# Round profiles: rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE passes of
# every bench workload (config 4 and its 8/4/2-GPU shards: counters only;
# configs 2 / 3 / 5), each step under its own time limit.  Summarise
# afterwards with tools/prof_summary.py (see tools/prof_round.sh).
set -o pipefail
R=${ROUND:-r03}
for spec in "c4 --videos 1024" "c4v512 --videos 512" "c4v256 --videos 256" "c4v128 --videos 128" \
            "c2 --config 2" "c3 --config 3" "c5 --config 5"; do
  set -- $spec
  name=$1; shift
  case " ${ONLY:-c4 c4v512 c4v256 c4v128 c2 c3 c5} " in *" $name "*) ;; *) continue ;; esac
  nt=""
  case $name in c4v*) nt=1 ;; esac
  NO_TRACE=$nt BENCH_ARGS="$*" bash tools/gpu_profile.sh ${R}_$name || exit $?
done

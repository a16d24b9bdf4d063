#!/bin/bash
# one build -> measure iteration on the GPU box: the whole -m gpu suite, the
# default (config 4) bench line without the CPU leg, then FETCH_SIZE and
# WRITE_SIZE passes over the eks kernels (separate --pmc runs).  SKIP_TESTS=1
# skips pytest; CONFIGS="2 3" adds bench lines of other configs.
set -o pipefail
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
OUT=gpurun_out/iter
mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
      > $OUT/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $OUT/pytest.log; exit 1; }
  tail -1 $OUT/pytest.log
fi
summ() {
  python - "$1" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(sys.argv[1], f"ms={d['ms_per_step']:.4f} frac={r['frac']:.4f}", r.get("kernels_ms"))
PY
}
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/b4.log 2>&1 || exit $?
summ $OUT/b4.log
for c in $CONFIGS; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline > $OUT/b$c.log 2>&1 || exit $?
  summ $OUT/b$c.log
done
[ -n "$NO_PMC" ] && exit 0
RAW=/tmp/iter_prof
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 -s KILL 240 rocprofv3 --kernel-include-regex 'k3_|k_model' --pmc $ctr -d $RAW/$ctr -o run \
      --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/pmc_$ctr.log 2>&1 || exit $?
  f=$(find $RAW/$ctr -name "*counter_collection.csv" | head -1)
  python - "$f" $ctr <<'PY'
import csv, sys, collections
acc = collections.defaultdict(list)
for row in csv.DictReader(open(sys.argv[1])):
    acc[row["Kernel_Name"].split("(")[0][-60:]].append(float(row["Counter_Value"]))
for k, v in acc.items():
    # FETCH_SIZE / WRITE_SIZE are per-dispatch sums over instances (KB)
    print(sys.argv[2], k, f"calls={len(v)} mean_KB={sum(v)/len(v):.0f}")
PY
done

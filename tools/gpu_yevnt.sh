#!/bin/bash
# non-temporal y / ev plane loads in algo 3 (the end-to-end fit -> smooth
# hand-off): config 4 end-to-end line, default build vs variant, alternated
set -o pipefail
OUT=gpurun_out/${1:-yevnt}
mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
for v in base yevnt base yevnt; do
  if [ $v = base ]; then L=eks_amd/lib/libeks_hip.so; else L=exp/$v/libeks_hip.so; fi
  EKS_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_$v.log 2>&1 || exit $?
  python -c "
import json
d=json.loads([x for x in open('$OUT/bench_$v.log') if x.startswith('{')][-1])
e=d['end_to_end']
print('$v', round(d['ms_per_step'],4), 'e2e', round(e['ms_per_step'],4), {k: e['kernels_ms'][k] for k in ('k3_elem','k3_coarse','k3_fine','k3_final')})"
done

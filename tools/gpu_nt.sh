#!/bin/bash
# non-temporal member loads / output stores (tools/build_variant.sh variants
# of eks_shape_22.hip): config 4 and config 2 bench per variant
set -o pipefail
OUT=gpurun_out/${1:-nt}
mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
for v in base ntload ntout ntboth base; do
  if [ $v = base ]; then L=eks_amd/lib/libeks_hip.so; else L=exp/$v/libeks_hip.so; fi
  for c in 4 2; do
    EKS_LIB=$L timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > $OUT/bench_${v}_c$c.log 2>&1 || exit $?
    python -c "
import json
d=json.loads([x for x in open('$OUT/bench_${v}_c$c.log') if x.startswith('{')][-1])
print('$v c$c', round(d['ms_per_step'],4), round(d['roofline']['frac'],4), d['roofline']['kernels_ms'])"
  done
done

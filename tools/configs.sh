#!/bin/bash
# Bench lines of the other BASELINE configurations (and config-3 variants)
# for each library variant: default = eks_amd/lib, NAME = exp/NAME.
#   VARIANTS="r05 default" bash tools/configs.sh
set -o pipefail
mkdir -p gpurun_out/cfg
export PYTHONDONTWRITEBYTECODE=1
CASES=${CASES:-"c2:--config 2|c3:--config 3|c3v6:--config 3 --cameras 6|c3v8:--config 3 --cameras 8|c5:--config 5"}
IFS='|' read -ra CS <<< "$CASES"
for v in ${VARIANTS:-default}; do
  if [ "$v" = default ]; then unset EKS_LIB; else export EKS_LIB=exp/$v/libeks_hip.so; fi
  for c in "${CS[@]}"; do
    tag=${c%%:*}; args=${c#*:}
    log=gpurun_out/cfg/${v}_$tag.log
    timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline $args > $log 2>&1 \
      || { echo "bench failed: $log"; tail -5 $log; exit 1; }
    python - $log "$v $tag" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
e = d.get("end_to_end") or {}
k = e.get("kernels_ms", {})
fit = sum(v for n, v in k.items() if "fit" in n or "sel" in n)
print(f"{sys.argv[2]:16s} ms={d['ms_per_step']:.4f} frac={d['roofline']['frac']:.4f}"
      + (f" e2e={e['ms_per_step']:.4f} fit={fit:.4f}" if e else "")
      + (f" flop={d['flop_roofline']['frac']:.3f}" if "flop_roofline" in d else ""))
PY
  done
done

#!/bin/bash
# config 2: member / y-ev prefetch distance variants (exp/d4, exp/d8) x chunk length
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
CONFIG=2 STEPS=30 VARIANTS="d4 d8" bash tools/variant_bench.sh || exit 1
for L in 16 24 48; do
  EKS_CHUNK_LEN=$L CONFIG=2 STEPS=30 VARIANTS="d8" bash tools/variant_bench.sh | sed "s/^/L=$L /" || exit 1
done

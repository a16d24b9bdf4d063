#!/bin/bash
# Build a tuning variant of libeks_hip.so: recompile the given translation
# units with extra flags, link with the default objects of the others.
#   tools/build_variant.sh NAME "FLAGS" unit1.hip [unit2.hip ...]
# -> exp/NAME/libeks_hip.so   (select it with EKS_LIB=exp/NAME/libeks_hip.so)
set -e
NAME=$1; FLAGS=$2; shift 2
OUT=exp/$NAME; mkdir -p $OUT/obj
OBJS=""
for src in eks_amd/csrc/*.hip eks_amd/csrc/*.cpp; do
  b=$(basename $src); b=${b%.*}
  o=eks_amd/lib/obj/$b.o
  hit=""
  for u in "$@"; do [ "$(basename $u .hip)" = "$b" ] && hit=1; done
  if [ -n "$hit" ]; then
    /opt/rocm/bin/hipcc $FLAGS -O3 -std=c++17 -fPIC --offload-arch=gfx950 -c eks_amd/csrc/$b.hip -o $OUT/obj/$b.o
    OBJS="$OBJS $OUT/obj/$b.o"
  else
    OBJS="$OBJS $o"
  fi
done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $OBJS -pthread -o $OUT/libeks_hip.so
echo built $OUT/libeks_hip.so

#!/bin/bash
# A/B variants of the single-view shape (config 4's kernels) only: compile
# eks_shape_22.hip from the CURRENT tree with extra flags, link it with the
# last full build's other objects -> exp/NAME/libeks_hip.so (EKS_LIB=...).
# For benches of config 4 only: the other shapes keep the last full build's
# code (a changed header is not re-read by them).
#   tools/build_22.sh NAME [-DFLAG=v ...]
set -e
NAME=$1; shift
OUT=exp/$NAME; rm -rf $OUT; mkdir -p $OUT/obj
/opt/rocm/bin/hipcc "$@" -O3 -std=c++17 -fPIC --offload-arch=gfx950 --offload-compress \
    -c eks_amd/csrc/eks_shape_22.hip -o $OUT/obj/eks_shape_22.o
OBJS=$OUT/obj/eks_shape_22.o
for o in eks_amd/lib/obj/*.o; do
  [ "$(basename $o)" = eks_shape_22.o ] || OBJS="$OBJS $o"
done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $OBJS -pthread -o $OUT/libeks_hip.so
rm -rf $OUT/obj
echo built $OUT/libeks_hip.so

#!/bin/bash
# Build a tuning variant of libeks_hip.so from a patched copy of the sources:
#   tools/build_patched.sh NAME PATCH unit1 [unit2 ...]
# copies eks_amd/csrc + include to exp/NAME/, applies PATCH (a diff against
# eks_amd/csrc, -p1 relative to the repo root: `git diff > x.patch` form),
# recompiles the listed units there and links them with the default objects
# of the others -> exp/NAME/libeks_hip.so (select with EKS_LIB=...).
set -e
NAME=$1; PATCH=$2; shift 2
OUT=exp/$NAME; rm -rf $OUT; mkdir -p $OUT/obj $OUT/src
cp -r eks_amd include $OUT/src/
(cd $OUT/src && patch -p1 -s < ../../../$PATCH)
OBJS=""
for src in eks_amd/csrc/*.hip eks_amd/csrc/*.cpp; do
  b=$(basename $src); b=${b%.*}
  [ "$b" = "torch_ops" ] && continue
  hit=""
  for u in "$@"; do [ "$(basename $u .hip)" = "$b" ] && hit=1; done
  if [ -n "$hit" ]; then
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -c $OUT/src/eks_amd/csrc/$b.hip -o $OUT/obj/$b.o &
    OBJS="$OBJS $OUT/obj/$b.o"
  else
    OBJS="$OBJS eks_amd/lib/obj/$b.o"
  fi
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $OBJS -pthread -o $OUT/libeks_hip.so
rm -rf $OUT/src $OUT/obj
echo built $OUT/libeks_hip.so

#!/bin/bash
# A tuning variant of libeks_hip.so from the CURRENT working tree: recompile
# the listed units, link them with the objects of the last full build
# (eks_amd/lib/obj) for the others -> exp/NAME/libeks_hip.so (EKS_LIB=...).
#   tools/build_cur.sh NAME [-DFLAG ...] unit1.hip [unit2.hip ...]
set -e
# The other units come from the last full build: a header changed since then
# (a struct layout, an inline function) would mix two definitions of the same
# weak symbols in one library (ChunkPlan / make_plan: a GPU memory fault in
# round 5).  Refuse; run python -m eks_amd.build first.
oldest=$(ls -tr eks_amd/lib/obj/*.o | head -n 1)
for h in eks_amd/csrc/*.hpp include/*.h; do
  if [ "$h" -nt "$oldest" ]; then
    echo "build_cur.sh: $h is newer than the last full build ($oldest): rebuild first" >&2
    exit 2
  fi
done
NAME=$1; shift
FLAGS=""; while [[ "$1" == -* ]]; do FLAGS="$FLAGS $1"; shift; done
OUT=exp/$NAME; rm -rf $OUT; mkdir -p $OUT/obj
OBJS=""
for src in eks_amd/csrc/*.hip eks_amd/csrc/*.cpp; do
  b=$(basename $src); b=${b%.*}
  [ "$b" = "torch_ops" ] && continue
  hit=""
  for u in "$@"; do [ "$(basename $u .hip)" = "$b" ] && hit=1; done
  if [ -n "$hit" ]; then
    /opt/rocm/bin/hipcc $FLAGS -O3 -std=c++17 -fPIC --offload-arch=gfx950 --offload-compress -c $src -o $OUT/obj/$b.o &
    OBJS="$OBJS $OUT/obj/$b.o"
  else
    OBJS="$OBJS eks_amd/lib/obj/$b.o"
  fi
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $OBJS -pthread -o $OUT/libeks_hip.so
rm -rf $OUT/obj
echo built $OUT/libeks_hip.so

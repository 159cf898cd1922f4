#!/bin/bash
# Build an alternative libmmad_hip.so with one source recompiled under extra -D flags:
#   bash tools/build_variant.sh <name> <source.hip> -DFLAG ...   -> varlib/<name>/libmmad_hip.so
# (run in the build container; MMAD_LIB_PATH=varlib/<name>/libmmad_hip.so selects it)
set -e
NAME=$1; SRC=$2; shift 2
OUT=varlib/$NAME
mkdir -p $OUT
FL="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -Wno-unused-function -Wno-unused-variable"
base=$(basename $SRC .hip)
/opt/rocm/bin/hipcc $FL "$@" -c multimodal_alzheimer_amd/csrc/$SRC -o $OUT/$base.o
objs=""
for o in build/obj/*.o; do
  [ "$(basename $o .o)" = "$base" ] && objs="$objs $OUT/$base.o" || objs="$objs $o"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libmmad_hip.so $objs
echo built $OUT/libmmad_hip.so

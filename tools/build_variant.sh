#!/bin/bash
# Builds a variant of the library with one source recompiled under extra flags, for an A/B through
# B2P_LIB_PATH: bash tools/build_variant.sh <out.so> <source.hip> <hipcc flags...>
# (the other objects come from build/obj of the current build)
set -e
OUT=$1; SRC=$2; shift 2
ROOT=$(cd $(dirname $0)/.. && pwd)
OBJ=/tmp/variant_$(basename $SRC).o
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -Wno-unused-result "$@" -c $ROOT/wav2vec2forbrain_amd/csrc/$SRC -o $OBJ
OBJS=$(ls $ROOT/build/obj/*.o | grep -v "/$SRC.o$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT $OBJS $OBJ
echo "built $OUT"

#!/bin/bash
# Build an A/B variant of libkrylov_hip.so with extra -D flags on one HIP
# source (SRC, default kt_kernels.hip; the other objects are the default build's):
#   [SRC=kt_pairs.hip] tools/build_variant.sh NAME "-DKT_X=1 ..."   ->  var/NAME/libkrylov_hip.so
# Select it at run time with KT_LIB=var/NAME/libkrylov_hip.so.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; FLAGS=$2; SRC=${SRC:-kt_kernels.hip}; OBJ=${SRC%.hip}.o
make -s -C "$ROOT/krylov_robustness_amd/csrc" >/dev/null
B=$ROOT/build/csrc; O=$ROOT/var/$NAME; mkdir -p "$O"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall -Wno-unused-function --offload-arch=gfx950 -munsafe-fp-atomics \
    $FLAGS -c "$ROOT/krylov_robustness_amd/csrc/$SRC" -o "$O/$OBJ"
OBJS=$(ls $B/*.o | grep -v "/$OBJ\$")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -lpthread -L/opt/rocm/lib -lrocsolver -lrocblas \
    "$O/$OBJ" $OBJS -o "$O/libkrylov_hip.so"
rm -f "$O/$OBJ"
echo "$O/libkrylov_hip.so"

#!/bin/bash
# Build an A/B variant of libkrylov_hip.so with extra -D flags on kt_kernels.hip
# only (the other objects are the default build's):
#   tools/build_variant.sh NAME "-DKT_X=1 ..."   ->  var/NAME/libkrylov_hip.so
# Select it at run time with KT_LIB=var/NAME/libkrylov_hip.so.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; FLAGS=$2
make -s -C "$ROOT/krylov_robustness_amd/csrc" >/dev/null
B=$ROOT/build/csrc; O=$ROOT/var/$NAME; mkdir -p "$O"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall -Wno-unused-function --offload-arch=gfx950 -munsafe-fp-atomics \
    $FLAGS -c "$ROOT/krylov_robustness_amd/csrc/kt_kernels.hip" -o "$O/kt_kernels.o"
OBJS=$(ls $B/*.o | grep -v kt_kernels.o)
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -lpthread -L/opt/rocm/lib -lrocsolver -lrocblas \
    "$O/kt_kernels.o" $OBJS -o "$O/libkrylov_hip.so"
rm -f "$O/kt_kernels.o"
echo "$O/libkrylov_hip.so"

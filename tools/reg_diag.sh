#!/bin/bash
# Config 5's candidate kernel (k_pair_reg) phase clocks: the KT_FUSED_PROF
# build, and the same with the SpMM's X gathers removed (KT_REG_DIAG=1;
# numbers of that build are wrong by construction, only its clocks mean
# anything).  Diagnostic libraries are built into diag/ by:
#   make -C krylov_robustness_amd/csrc OUT=../../diag/libkrylov_fprof.so BUILD=../../build/fprof EXTRA=-DKT_FUSED_PROF
#   make ... OUT=../../diag/libkrylov_fprof_d1.so BUILD=../../build/fprof_d1 EXTRA="-DKT_FUSED_PROF -DKT_REG_DIAG=1"
set -o pipefail
O=gpurun_out/${1:-regdiag}; mkdir -p $O
for v in fprof fprof_d1; do
    KT_LIB=$PWD/diag/libkrylov_$v.so timeout -k 10 120 python tools/greedy_split.py > $O/$v.txt 2>&1 || { tail -5 $O/$v.txt; exit 1; }
    echo "== $v"; grep -v amdgpu.ids $O/$v.txt | grep -v reg_prof; for it in 5 10 20 40; do grep "it=$it " $O/$v.txt | tail -1; done
done

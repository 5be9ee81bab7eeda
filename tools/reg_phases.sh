# Config 5 register-resident candidate kernel: phase clocks (KT_FUSED_PROF
# build, LDS accumulators) and vector work alone (KT_FUSED_NOEIG build).
set -o pipefail
O=gpurun_out/regph; mkdir -p $O
KT_LIB=$PWD/build/fprof/libkrylov_fprof.so timeout -k 10 120 python tools/greedy_split.py > $O/prof.txt 2>&1 || { tail -5 $O/prof.txt; exit 1; }
KT_LIB=$PWD/build/noeig/libkrylov_noeig.so timeout -k 10 120 python tools/greedy_split.py > $O/noeig.txt 2>&1 || { tail -5 $O/noeig.txt; exit 1; }
grep -v _prof $O/prof.txt | grep -v amdgpu.ids
for it in 5 10 20 40 100; do grep "it=$it " $O/prof.txt | tail -1; done
cat $O/noeig.txt | grep -v amdgpu.ids

# Config 5: register-resident candidate kernel (k_pair_reg) vs k_pair_fused
# (KT_PAIRS_REG=0): parity tests, step anatomy, the greedy bench, phase clocks
# (build/fprof: EXTRA=-DKT_FUSED_PROF, build/noeig: EXTRA=-DKT_FUSED_NOEIG).
set -o pipefail

O=gpurun_out/abreg; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_greedy.py > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -3 $O/t.log
for v in 0 1; do
  KT_PAIRS_REG=$v timeout -k 10 120 python tools/greedy_split.py > $O/split_$v.txt 2>/dev/null || exit 1
  KT_PAIRS_REG=$v timeout -k 10 200 python tests/perf/bench_greedy.py --cpu-steps 0 > $O/bench_$v.json 2>/dev/null || exit 1
done
KT_LIB=$PWD/build/fprof/libkrylov_fprof.so timeout -k 10 120 python tools/greedy_split.py > $O/prof.txt 2>&1 || exit 1
for v in 0 1; do echo "== KT_PAIRS_REG=$v"; cat $O/split_$v.txt; cut -c1-300 $O/bench_$v.json; done
grep "it=100 " $O/prof.txt | tail -2
# Config 5 register-resident candidate kernel: phase clocks (KT_FUSED_PROF
# build, LDS accumulators) and vector work alone (KT_FUSED_NOEIG build).

O=gpurun_out/regph; mkdir -p $O
KT_LIB=$PWD/build/fprof/libkrylov_fprof.so timeout -k 10 120 python tools/greedy_split.py > $O/prof.txt 2>&1 || { tail -5 $O/prof.txt; exit 1; }
KT_LIB=$PWD/build/noeig/libkrylov_noeig.so timeout -k 10 120 python tools/greedy_split.py > $O/noeig.txt 2>&1 || { tail -5 $O/noeig.txt; exit 1; }
grep -v _prof $O/prof.txt | grep -v amdgpu.ids
for it in 5 10 20 40 100; do grep "it=$it " $O/prof.txt | tail -1; done
cat $O/noeig.txt | grep -v amdgpu.ids

#!/bin/bash
# Config 5: step j+1 SpMM issued before step j eigenvalues in k_pair_reg (default) vs after the stop test (KT_REG_SPEC=0):
# greedy parity tests, phase clocks, the greedy bench (3 alternations).
set -o pipefail
O=gpurun_out/spec; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_greedy.py > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
for v in fprof0 fprof; do
  KT_LIB=$PWD/build/$v/libkrylov_$v.so timeout -k 10 120 python tools/greedy_split.py > $O/p_$v.txt 2>&1 || { tail -5 $O/p_$v.txt; exit 1; }
  echo "== $v"; grep "it=100 \|it=10 " $O/p_$v.txt | tail -2; grep '"tol"' $O/p_$v.txt | cut -c1-160
done
for r in 1 2 3; do
  for v in old new; do
    case $v in old) L=$PWD/build/old/libkrylov_old.so;; new) L=$PWD/krylov_robustness_amd/libkrylov_hip.so;; esac
    KT_LIB=$L timeout -k 10 200 python tests/perf/bench_greedy.py --cpu-steps 0 > $O/b_$v.json 2>/dev/null || exit 1
    echo "$v $(cut -c1-200 $O/b_$v.json)"
  done
done

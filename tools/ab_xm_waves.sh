#!/bin/bash
# Greedy eigenvalues: waves per projection in k_pair_reg, 4 (shipped) vs 2 and 1 (KT_XM_WAVES builds):
# greedy parity tests per variant, then bench_greedy alternating.
set -o pipefail
O=gpurun_out/xw; mkdir -p $O
for v in xw2 xw1; do
  KT_LIB=$PWD/build/$v/libkrylov_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_greedy.py -k "not register_kernel_matches_fused" > $O/t_$v.log 2>&1 || { echo "tests $v failed"; tail -30 $O/t_$v.log; exit 1; }
  echo "$v $(tail -1 $O/t_$v.log)"
done
for r in 1 2 3; do
  for v in ship xw2 xw1; do
    case $v in ship) L=$PWD/krylov_robustness_amd/libkrylov_hip.so;; *) L=$PWD/build/$v/libkrylov_$v.so;; esac
    KT_LIB=$L timeout -k 10 200 python tests/perf/bench_greedy.py --cpu-steps 0 > $O/b_$v.json 2>/dev/null || exit 1
    echo "$v $(python3 -c "import json; d=json.load(open('$O/b_$v.json')); print(round(d['gpu_seconds']*1e3,2), 'ms', d['rob_variation'])")"
  done
done

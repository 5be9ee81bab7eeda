#!/bin/bash
# Greedy eigenvalues: Newton accepted at a step below 64 atol (shipped) vs 4096 and 2^20 atol:
# (KT_BLK_NEWTON_ACCEPT builds) greedy parity tests, then bench_greedy alternating.
set -o pipefail
O=gpurun_out/nacc; mkdir -p $O
for v in na4096 na1048576; do
  KT_LIB=$PWD/build/$v/libkrylov_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_greedy.py > $O/t_$v.log 2>&1 || { echo "tests $v failed"; tail -30 $O/t_$v.log; exit 1; }
  echo "$v $(tail -1 $O/t_$v.log)"
done
for r in 1 2 3; do
  for v in ship na4096 na1048576; do
    case $v in ship) L=$PWD/krylov_robustness_amd/libkrylov_hip.so;; *) L=$PWD/build/$v/libkrylov_$v.so;; esac
    KT_LIB=$L timeout -k 10 200 python tests/perf/bench_greedy.py --cpu-steps 0 > $O/b_$v.json 2>/dev/null || exit 1
    echo "$v $(python3 -c "import json; d=json.load(open('$O/b_$v.json')); print(round(d['gpu_seconds']*1e3,2), 'ms', d['rob_variation'])")"
  done
done

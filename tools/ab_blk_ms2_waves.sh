#!/bin/bash
# Greedy eigenvalues with 2 waves per projection: 1 shift per lane (shipped) vs 2 (KT_BLK_MS=2 build):
# greedy parity tests, then bench_greedy alternating.
set -o pipefail
O=gpurun_out/ms2w; mkdir -p $O
for v in ms2; do
  KT_LIB=$PWD/build/$v/libkrylov_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_greedy.py > $O/t_$v.log 2>&1 || { echo "tests $v failed"; tail -30 $O/t_$v.log; exit 1; }
  echo "$v $(tail -1 $O/t_$v.log)"
done
for r in 1 2 3; do
  for v in ship ms2; do
    case $v in ship) L=$PWD/krylov_robustness_amd/libkrylov_hip.so;; *) L=$PWD/build/$v/libkrylov_$v.so;; esac
    KT_LIB=$L timeout -k 10 200 python tests/perf/bench_greedy.py --cpu-steps 0 > $O/b_$v.json 2>/dev/null || exit 1
    echo "$v $(python3 -c "import json; d=json.load(open('$O/b_$v.json')); print(round(d['gpu_seconds']*1e3,2), 'ms', d['rob_variation'])")"
  done
done

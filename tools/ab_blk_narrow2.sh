#!/bin/bash
# Greedy eigenvalues (1 shift per lane, 2 waves, Newton accepted at 2^20 atol): multisection to span/4096 before Newton (shipped) vs span/1024, span/256
# (KT_BLK_NARROW builds): greedy parity tests per variant, then bench_greedy alternating.
set -o pipefail
O=gpurun_out/narrow2; mkdir -p $O
for v in n1024 n256; do
  KT_LIB=$PWD/build/$v/libkrylov_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_greedy.py > $O/t_$v.log 2>&1 || { echo "tests $v failed"; tail -30 $O/t_$v.log; exit 1; }
  echo "$v $(tail -1 $O/t_$v.log)"
done
for r in 1 2 3; do
  for v in ship n1024 n256; do
    case $v in ship) L=$PWD/krylov_robustness_amd/libkrylov_hip.so;; *) L=$PWD/build/$v/libkrylov_$v.so;; esac
    KT_LIB=$L timeout -k 10 200 python tests/perf/bench_greedy.py --cpu-steps 0 > $O/b_$v.json 2>/dev/null || exit 1
    echo "$v $(python3 -c "import json; d=json.load(open('$O/b_$v.json')); print(round(d['gpu_seconds']*1e3,2), 'ms', d['rob_variation'])")"
  done
done

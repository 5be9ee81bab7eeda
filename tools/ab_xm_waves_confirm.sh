#!/bin/bash
# Adaptive eigenvalue waves (2 per projection while 2j <= 32, else 4; fused and register kernels
# alike) vs 4 always (build/old): every GPU test, then config 5 bench_greedy alternating.
set -o pipefail
O=gpurun_out/xwc; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for r in 1 2 3; do
  for v in w4 adaptive; do
    case $v in adaptive) L=$PWD/krylov_robustness_amd/libkrylov_hip.so;; w4) L=$PWD/build/old/libkrylov_old.so;; esac
    KT_LIB=$L timeout -k 10 200 python tests/perf/bench_greedy.py --cpu-steps 0 > $O/b_$v.json 2>/dev/null || exit 1
    echo "$v $(python3 -c "import json; d=json.load(open('$O/b_$v.json')); print(round(d['gpu_seconds']*1e3,2), 'ms', d['rob_variation'], d['first_edges'])")"
  done
done

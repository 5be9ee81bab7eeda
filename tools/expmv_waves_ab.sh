#!/bin/bash
# Per-term expmv kernel: 8 waves per block (default) vs 4 (build/w4): parity tests, trace_exp(A6) expmv Afun.
set -o pipefail
O=gpurun_out/ew; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_mctrace.py tests/test_gpu_mctrace_sharded.py > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
for r in 1 2 3; do
  for v in w4 w8; do
    case $v in w4) L=$PWD/build/w4/libkrylov_w4.so;; w8) L=$PWD/krylov_robustness_amd/libkrylov_hip.so;; esac
    KT_LIB=$L timeout -k 10 120 python tools/run_trace_exp_expmv.py > $O/x.txt 2>&1 || { tail -5 $O/x.txt; exit 1; }
    echo "$v $(grep trace_exp $O/x.txt)"
  done
done
timeout -k 10 300 python tests/perf/bench_config1.py > $O/c1.json 2> $O/c1.err || { tail -5 $O/c1.err; exit 1; }
cut -c1-900 $O/c1.json

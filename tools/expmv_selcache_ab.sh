#!/bin/bash
# expmv degree-selection cache: parity tests, trace_exp(A6) expmv Afun with / without the cache.
set -o pipefail
O=gpurun_out/sel; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_mctrace.py tests/test_gpu_mctrace_sharded.py > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
for r in 1 2 3; do
  for v in 0 1; do
    KT_EXPMV_SEL_CACHE=$v timeout -k 10 120 python tools/run_trace_exp_expmv.py > $O/x.txt 2>&1 || { tail -5 $O/x.txt; exit 1; }
    echo "cache=$v $(grep trace_exp $O/x.txt)"
  done
done

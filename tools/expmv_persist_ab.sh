#!/bin/bash
# Persistent expmv launch (k_expmv_run) vs the per-term launches: parity
# tests, then trace_exp(A6) with the expmv Afun under each form and grid size.
set -o pipefail
O=gpurun_out/xp; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_mctrace.py > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -3 $O/t.log
for v in "KT_EXPMV_PERSIST=0" "KT_EXPMV_PERSIST=1" "KT_EXPMV_GRID=64" "KT_EXPMV_GRID=128" "KT_EXPMV_GRID=400" "KT_TWIN=0"; do
  for r in 1 2; do
    env $v timeout -k 10 120 python tools/run_trace_exp_expmv.py > $O/r.txt 2>&1 || { cat $O/r.txt; exit 1; }
    echo "$v $(grep trace_exp $O/r.txt)"
  done
done

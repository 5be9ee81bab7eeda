#!/bin/bash
# Persistent expmv: parity tests, then in-kernel barrier clocks (KT_EXPMV_PROF=1)
# per variant (serial order), then trace_exp timings.
set -o pipefail
O=gpurun_out/xpp; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_mctrace.py > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -2 $O/t.log
for v in "KT_EXPMV_PERSIST=1 KT_EXPMV_RUN2=0" "KT_EXPMV_PERSIST=1"; do
  env $v KT_TWIN=0 KT_EXPMV_PROF=1 timeout -k 10 120 python tools/run_trace_exp_expmv.py > $O/p.txt 2>&1 || { cat $O/p.txt; exit 1; }
  echo "== $v"; grep -v amdgpu.ids $O/p.txt | tail -3
done
for v in "KT_EXPMV_PERSIST=0" "KT_EXPMV_PERSIST=1" "KT_EXPMV_PERSIST=1 KT_TWIN=0" "KT_EXPMV_PERSIST=0 KT_TWIN=0"; do
  for r in 1 2; do
    env $v timeout -k 10 120 python tools/run_trace_exp_expmv.py > $O/r.txt 2>&1 || { cat $O/r.txt; exit 1; }
    echo "$v $(grep trace_exp $O/r.txt)"
  done
done

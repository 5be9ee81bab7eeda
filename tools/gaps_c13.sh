#!/bin/bash
# Kernel-trace gap analysis: config 3 fun_and_grad (tools/prof_fg.py) and config 1 trace_exp (expmv Afun).
set -o pipefail
O=$PWD/gpurun_out/g13; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/fg -o g -- python3 tools/prof_fg.py > $O/fg.txt 2>&1 || { tail -20 $O/fg.txt; exit 1; }
grep "^fg" $O/fg.txt | tail -2
python3 tools/gaps.py $(find $O/fg -name "*kernel_trace.csv" | head -1) k_ts_step half | head -14
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/c1 -o g -- python3 tools/run_trace_exp_expmv.py > $O/c1.txt 2>&1 || { tail -20 $O/c1.txt; exit 1; }
grep trace_exp $O/c1.txt
python3 tools/gaps.py $(find $O/c1 -name "*kernel_trace.csv" | head -1) k_expmv_step half | head -14

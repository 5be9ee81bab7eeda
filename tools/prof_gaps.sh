#!/bin/bash
# Kernel trace of a python script (two identical calls inside) + gap analysis
# of the second call.  GPU box: bash tools/prof_gaps.sh TAG START_KERNEL script.py [args]
set -o pipefail
TAG=$1; START=$2; shift 2
OUT=$PWD/gpurun_out/$TAG
rm -rf $OUT; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o g -- python3 "$@" > $OUT/out.txt 2>&1 || { tail -20 $OUT/out.txt; exit 1; }
cat $OUT/out.txt | tail -3
python3 tools/gaps.py $(find $OUT/trace -name "*kernel_trace.csv" | head -1) "$START" half | tee $OUT/gaps.txt

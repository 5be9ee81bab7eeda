#!/bin/bash
# Kernel trace of a short default-lane bench run + occupancy timeline of its
# timed region (tools/timeline.py).  GPU box, repo root: bash tools/prof_timeline.sh TAG [bench args]
set -o pipefail
TAG=${1:-tl}; shift
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o tl -- python3 bench.py --steps 2 --warmup 1 --cpu-seconds 0 "$@" > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
TR=$(find $OUT/trace -name "*kernel_trace.csv" | head -1)
python3 tools/timeline.py $TR k_spmm_lanczos $((2 * 64 * 29)) 116 | tee $OUT/timeline.txt
cat $OUT/bench.json

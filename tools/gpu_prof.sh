#!/bin/bash
# rocprofv3 passes (each in its own run): kernel stats, then HBM counters.
# Usage: bash tools/gpu_prof.sh TAG "sweep args"
set -o pipefail
TAG=${1:-r01}
ARGS=${2:---blocks 16,128 --nprobes 64 --m 10}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o kt --output-format csv -- python3 tools/sweep_block.py $ARGS > $OUT/prof_stats.log 2>&1 || { tail -20 $OUT/prof_stats.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "spmm_gram|update_norm" -d $OUT/pmc_fetch -o f --output-format csv -- python3 tools/sweep_block.py $ARGS > $OUT/prof_fetch.log 2>&1 || { tail -20 $OUT/prof_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "spmm_gram|update_norm" -d $OUT/pmc_write -o w --output-format csv -- python3 tools/sweep_block.py $ARGS > $OUT/prof_write.log 2>&1 || { tail -20 $OUT/prof_write.log; exit 1; }
find $OUT -name "*.csv" | head -20

#!/bin/bash
# rocprofv3 passes on the bench workload, each in its own run:
#   1. kernel trace + stats   2. FETCH_SIZE   3. WRITE_SIZE
# Usage (GPU box, repo root): bash tools/gpu_prof.sh TAG [extra bench args]
set -o pipefail
TAG=${1:-r01}; shift
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT profiles
export TMPDIR=/tmp
BENCH="bench.py --steps 1 --warmup 1 --cpu-seconds 0 --lanes 1 $*"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/stats -o kt --output-format csv -- python3 $BENCH > $OUT/prof_stats.log 2>&1 || { tail -20 $OUT/prof_stats.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "spmm_dot|spmm_lanczos|k_update" -d $OUT/pmc_fetch -o f --output-format csv -- python3 $BENCH --no-profile > $OUT/prof_fetch.log 2>&1 || { tail -20 $OUT/prof_fetch.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "spmm_dot|spmm_lanczos|k_update" -d $OUT/pmc_write -o w --output-format csv -- python3 $BENCH --no-profile > $OUT/prof_write.log 2>&1 || { tail -20 $OUT/prof_write.log; exit 1; }
python3 tools/pmc_traffic.py $(find $OUT/pmc_fetch -name "*counter_collection.csv") $(find $OUT/pmc_write -name "*counter_collection.csv") $OUT/traffic.json
cp $(find $OUT/stats -name "*kernel_stats.csv") $OUT/kernel_stats.csv

#!/bin/bash
# Config-5 A/B of k_pair_reg builds on one box (boxes differ by up to 8 %):
#   bash tools/pair_ab.sh TAG "NAME1 NAME2 ..." ["PROF1 PROF2 ..."]
# NAME = a var/NAME build (tools/build_variant.sh) or "lib" (the in-tree
# library); each is timed by tests/perf/bench_greedy.py twice, interleaved.
# PROF names are -DKT_FUSED_PROF builds: their per-phase device clocks
# (one reg_prof line per launch of tools/pair_prof.py) go to PROF.log.  The greedy / pair tests run
# first on the in-tree library (NOTEST=1: timing only).
set -o pipefail
TAG=$1; NAMES=$2; PROFS=$3
O=$PWD/gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
[ -n "$NOTEST" ] || timeout -k 10 600 python -u -m pytest tests/test_gpu_greedy.py tests/test_gpu_configs.py -k "greedy or pairs" \
    -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
lib() { [ "$1" = lib ] && echo "$PWD/krylov_robustness_amd/libkrylov_hip.so" || echo "$PWD/var/$1/libkrylov_hip.so"; }
for rep in 1 2; do
    for v in $NAMES; do
        r=$(KT_LIB=$(lib $v) timeout -k 10 300 python tests/perf/bench_greedy.py --cpu-steps 0 --repeat 5 2> $O/$v.err) \
            || { tail -20 $O/$v.err; exit 1; }
        echo "{\"variant\": \"$v\", \"rep\": $rep, \"result\": $r}" | tee -a $O/ab.jsonl | cut -c1-200
    done
done
for v in $PROFS; do
    KT_LIB=$(lib $v) timeout -k 10 300 python tools/pair_prof.py 6 > $O/$v.log 2> $O/$v.err \
        || { tail -20 $O/$v.err; exit 1; }
    tail -1 $O/$v.log | cut -c1-200
done

#!/bin/bash
# Same-box A/B of library builds on the config-4 reference composition
# (tools/expmv_c4.py: 3 trace_exp calls with the expmv Afun, seeds 0-2; the
# first is cold) and the default bench line without its CPU legs:
#   bash tools/expmv_ab.sh TAG "NAME1 NAME2 ..."   (NAME: var/NAME build or "lib")
set -o pipefail
TAG=$1; NAMES=$2
O=$PWD/gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
lib() { [ "$1" = lib ] && echo "$PWD/krylov_robustness_amd/libkrylov_hip.so" || echo "$PWD/var/$1/libkrylov_hip.so"; }
for rep in 1 2; do
    for v in $NAMES; do
        KT_LIB=$(lib $v) timeout -k 10 300 python tools/expmv_c4.py 3 > $O/c4_${v}_$rep.jsonl 2> $O/c4_$v.err \
            || { tail -20 $O/c4_$v.err; exit 1; }
        echo "$v $rep $(tail -2 $O/c4_${v}_$rep.jsonl | tr '\n' ' ' | cut -c1-300)"
    done
done
for v in $NAMES; do
    KT_LIB=$(lib $v) timeout -k 10 300 python bench.py --cpu-seconds 0 --ref-cpu-seconds 0 > $O/bench_$v.json 2> $O/bench_$v.err \
        || { tail -20 $O/bench_$v.err; exit 1; }
    echo "$v $(cut -c1-200 $O/bench_$v.json)"
done

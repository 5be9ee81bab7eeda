#!/bin/bash
# Same-box A/B of var/kk_nodpp (-DKT_SHFL_DPP=0) and the in-tree library on the
# config-1 and config-3 drivers (tests/perf/bench_config{1,3}.py), twice each.
set -o pipefail
O=$PWD/gpurun_out/${1:-kk2}; mkdir -p $O
for rep in 1 2; do for v in kk_nodpp lib; do
  L=$PWD/var/$v/libkrylov_hip.so; [ $v = lib ] && L=$PWD/krylov_robustness_amd/libkrylov_hip.so
  for s in bench_config1 bench_config3; do
    KT_LIB=$L timeout -k 10 300 python tests/perf/$s.py > $O/${s}_${v}_$rep.json 2> $O/$s.err || { tail -5 $O/$s.err; exit 1; }
    echo "$v $rep $s $(cut -c1-250 $O/${s}_${v}_$rep.json)"
  done
done; done

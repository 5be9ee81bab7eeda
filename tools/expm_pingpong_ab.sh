#!/bin/bash
# Device expm squarings ping-ponged between two buffers (no device-to-device copy per
# squaring) vs the round-2 copy-back form (build/old): Krylov GPU tests, then config 3
# fun_and_grad call times alternating the two libraries.
set -o pipefail
O=gpurun_out/epp; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_krylov.py tests/test_gpu_datasets.py > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for r in 1 2 3; do
  for v in old new; do
    case $v in old) L=$PWD/build/old/libkrylov_old.so;; new) L=$PWD/krylov_robustness_amd/libkrylov_hip.so;; esac
    KT_LIB=$L timeout -k 10 120 python tools/prof_fg.py > $O/f_$v.txt 2>&1 || { tail -5 $O/f_$v.txt; exit 1; }
    echo "$v $(grep '^fg' $O/f_$v.txt | awk '{print $2}' | tr '\n' ' ') $(grep '^fg' $O/f_$v.txt | tail -1 | awk '{print $4}')"
  done
done

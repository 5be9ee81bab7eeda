#!/bin/bash
# Gram slab count (rows per slab, KT_GRAM_ROWS) for the block-Krylov Gram G = X Y':
# config 3 fun_and_grad call times (the Hawaii LCC, n = 21,774: 1024 rows -> 21 slabs).
set -o pipefail
O=gpurun_out/gram; mkdir -p $O
for r in 1 2; do
  for g in 1024 512 340 256; do
    KT_GRAM_ROWS=$g timeout -k 10 120 python tools/prof_fg.py > $O/f_$g.txt 2>&1 || { tail -5 $O/f_$g.txt; exit 1; }
    echo "rows=$g $(grep '^fg' $O/f_$g.txt | awk '{print $2}' | tr '\n' ' ') $(grep '^fg' $O/f_$g.txt | tail -1 | awk '{print $4}')"
  done
done

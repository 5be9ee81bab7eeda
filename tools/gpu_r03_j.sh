# config 3 fun_and_grad: Householder sweep forms A/B (two-launch default, persistent KT_TSQR_PERSIST=1, one-launch KT_TSQR_STEP1=1)
set -e
O=gpurun_out/r03j; mkdir -p $O
for r in 1 2; do
  for v in "KT_DUMMY=1" "KT_TSQR_PERSIST=1" "KT_TSQR_STEP1=1"; do
    env $v timeout -k 10 120 python tools/prof_fg.py > $O/fg.txt 2>&1
    echo "$v: $(grep '^fg' $O/fg.txt | cut -c1-10 | tr '\n' ' ')"
  done
done

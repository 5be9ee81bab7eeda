set -e
O=gpurun_out/r03r; mkdir -p $O
for r in 1 2; do
KT_QR_SHIFTED=0 timeout -k 10 120 python tools/prof_fg_exp.py > $O/a.txt 2>&1; echo "householder: $(grep fg_exp $O/a.txt | cut -c8-14 | tr '\n' ' ')"
timeout -k 10 120 python tools/prof_fg_exp.py > $O/b.txt 2>&1; echo "shifted: $(grep fg_exp $O/b.txt | cut -c8-14 | tr '\n' ' ')"
done

set -e
O=gpurun_out/fgexp10; mkdir -p $O
KT_FG_TIMING=1 timeout -k 10 120 python tools/prof_fg_exp.py > $O/timing.txt 2>&1
KT_DEVMAT_FILL=1 KT_FG_TIMING=1 timeout -k 10 120 python tools/prof_fg_exp.py > $O/timing_fill.txt 2>&1
grep "query-spin 1\|query-spin 2\|query-spin 3\|fg_exp" $O/timing.txt | tail -6
echo == fill
grep "query\|fg_exp" $O/timing_fill.txt | tail -12

# config 3 fun_and_grad: catch the sporadic +6 ms calls with the phase timers
set -e
O=gpurun_out/r03k; mkdir -p $O
KT_FG_REPS=10 KT_FG_TIMING=1 timeout -k 10 200 python tools/prof_fg.py > $O/timing.txt 2>&1
grep "^fg" $O/timing.txt | tr '\n' ' '

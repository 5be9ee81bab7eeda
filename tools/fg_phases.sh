# Config 3 fun_and_grad phases per Krylov step (KT_FG_TIMING=1), twin and serial
set -e
O=gpurun_out/fgp; mkdir -p $O
KT_FG_TIMING=1 timeout -k 10 120 python tools/prof_fg.py > $O/twin.txt 2>&1
KT_FG_TIMING=1 KT_TWIN=0 timeout -k 10 120 python tools/prof_fg.py > $O/serial.txt 2>&1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$O/prof -o fg -- python3 tools/prof_fg.py > $O/prof.txt 2>&1
python3 tools/gaps.py $(find $O/prof -name "*kernel_trace.csv" | head -1) k_ts_step half > $O/gaps.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$O/c1 -o c1 -- python3 tools/run_trace_exp_expmv.py > $O/c1.txt 2>&1
python3 tools/gaps.py $(find $O/c1 -name "*kernel_trace.csv" | head -1) k_expmv_step half > $O/c1_gaps.txt

# fun_and_grad_krylov_exp on India: phase timers and a kernel trace (pipelined, own GEMM kernels)
set -e
O=gpurun_out/fgexp2; mkdir -p $O
KT_FG_TIMING=1 timeout -k 10 120 python tools/prof_fg_exp.py > $O/timing.txt 2>&1
KT_FG_TIMING=1 KT_GEMM_ROCBLAS=1 timeout -k 10 120 python tools/prof_fg_exp.py > $O/timing_rocblas.txt 2>&1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$O/prof -o fg -- python3 tools/prof_fg_exp.py > $O/prof.txt 2>&1
cp $(find $O/prof -name "*kernel_stats.csv" | head -1) $O/kernel_stats.csv

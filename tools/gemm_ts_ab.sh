# kt_gemm_ts.hip (custom gram / combine) vs rocBLAS (KT_GEMM_ROCBLAS=1): GPU tests, config 3 fg A/B,
# one-step kernel timeline of the new path.
set -e
O=gpurun_out/gemmts; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
for r in 1 2; do
KT_GEMM_ROCBLAS=1 timeout -k 10 120 python tools/prof_fg.py > $O/rocblas$r.txt 2>&1
timeout -k 10 120 python tools/prof_fg.py > $O/custom$r.txt 2>&1
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$O/prof -o fg -- python3 tools/prof_fg.py > $O/prof.txt 2>&1
python3 tools/step_timeline.py $(find $O/prof -name "*kernel_trace.csv" | head -1) -1 4 v > $O/step.txt

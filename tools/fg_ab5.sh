set -e
O=gpurun_out/fgab5; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_qr.py tests/test_gpu_krylov.py tests/test_gpu_configs.py tests/test_gpu_mctrace.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || true
for r in 1 2; do
KT_TSQR_FUSED=0 timeout -k 10 120 python tools/prof_fg.py > $O/unfused$r.txt 2>&1
timeout -k 10 120 python tools/prof_fg.py > $O/fused$r.txt 2>&1
done
KT_FG_TIMING=1 timeout -k 10 120 python tools/prof_fg.py > $O/phases.txt 2>&1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$O/prof -o fg -- python3 tools/prof_fg.py > $O/prof.txt 2>&1
python3 tools/step_timeline.py $(find $O/prof -name "*kernel_trace.csv" | head -1) -1 4 v > $O/step.txt

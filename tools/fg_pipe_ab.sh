# Config 3 fun_and_grad: pipelined projections (default) vs serial loops (KT_FU_PIPE=0 KT_TFU_PIPE=0),
# per-step phases of the pipelined run, then the block-Krylov GPU tests.
set -e
O=gpurun_out/fgpipe; mkdir -p $O
for r in 1 2; do
KT_FU_PIPE=0 KT_TFU_PIPE=0 timeout -k 10 120 python tools/prof_fg.py > $O/serial$r.txt 2>&1
timeout -k 10 120 python tools/prof_fg.py > $O/pipe$r.txt 2>&1
done
KT_FG_TIMING=1 timeout -k 10 120 python tools/prof_fg.py > $O/pipe_phases.txt 2>&1
timeout -k 10 600 python -u -m pytest tests/test_gpu_krylov.py tests/test_gpu_configs.py tests/test_gpu_mctrace.py tests/test_gpu_frechet.py tests/test_gpu_fme.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1

# y-form hot path: SLQ GPU tests, then lanes-2 sweep timing (P = 16, n = 1M Chung-Lu).
set -e
mkdir -p gpurun_out/yform
timeout -k 10 600 python -u -m pytest tests/test_gpu_slq.py tests/test_gpu_mctrace.py -x -q --timeout 300 --timeout-method thread > gpurun_out/yform/pytest.log 2>&1 || { tail -30 gpurun_out/yform/pytest.log; exit 1; }
tail -2 gpurun_out/yform/pytest.log
timeout -k 10 500 python tools/sweep_block.py --config sf1m --nprobes 1024 --blocks 16 --variants ynt_lanes2,ynt,ynt_lanes2 > gpurun_out/yform/start.txt 2>&1
cat gpurun_out/yform/start.txt

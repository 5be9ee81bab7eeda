# y-form hot path: full GPU tests, then sweep lanes for the y-form pass (P = 16, n = 1M Chung-Lu).
set -e
mkdir -p gpurun_out/yform
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/yform/pytest.log 2>&1 || { tail -30 gpurun_out/yform/pytest.log; exit 1; }
tail -2 gpurun_out/yform/pytest.log
timeout -k 10 500 python tools/sweep_block.py --config sf1m --nprobes 1024 --blocks 16 --variants y_lanes2,ynt_lanes2,y_lanes3,ynt_lanes3,y_lanes4,ynt_lanes4,y_lanes2,ynt_lanes2 > gpurun_out/yform/lanes.txt 2>&1
cat gpurun_out/yform/lanes.txt

# y-form pass: write-through (sc1) y_{j+1} stores vs nontemporal; parity under sc1 first.
set -e
mkdir -p gpurun_out/yform
KT_KY_FLAGS=16 timeout -k 10 600 python -u -m pytest tests/test_gpu_slq.py -x -q --timeout 300 --timeout-method thread > gpurun_out/yform/pytest_sc1.log 2>&1 || { tail -30 gpurun_out/yform/pytest_sc1.log; exit 1; }
tail -1 gpurun_out/yform/pytest_sc1.log
timeout -k 10 500 python tools/sweep_block.py --config sf1m --nprobes 512 --blocks 16 --variants ynt,ysc1,ynt_lanes2,ysc1_lanes2,ynt,ysc1 > gpurun_out/yform/sc1.txt 2>&1
cat gpurun_out/yform/sc1.txt

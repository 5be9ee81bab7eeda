# y-form pass at P = 8 / 16 / 32 (n = 1M Chung-Lu), 1 and 2 lanes.
set -e
mkdir -p gpurun_out/yform
timeout -k 10 500 python tools/sweep_block.py --config sf1m --nprobes 512 --blocks 8,16,32 --variants ynt,ynt_lanes2 > gpurun_out/yform/blocks.txt 2>&1
cat gpurun_out/yform/blocks.txt

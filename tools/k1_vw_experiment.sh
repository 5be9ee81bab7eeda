# K1 lane width (KT_K1_VW = doubles per lane) and 8-deep gather issue, built on the box.
set -e
mkdir -p gpurun_out/vw
timeout -k 10 500 python tools/sweep_block.py --config sf1m --nprobes 512 --blocks 16 --variants ntyk2,mlpk2,ntyk2_lanes3,mlpk2_lanes3 > gpurun_out/vw/vw4.txt 2>&1
make -C krylov_robustness_amd/csrc -j16 BUILD=../../build/vw8 EXTRA=-DKT_K1_VW=8 > gpurun_out/vw/build8.log 2>&1
timeout -k 10 500 python tools/sweep_block.py --config sf1m --nprobes 512 --blocks 16 --variants ntyk2,mlpk2,ntyk2_lanes3,mlpk2_lanes3 > gpurun_out/vw/vw8.txt 2>&1
echo done

# Builds K1/K2 with 4 doubles per lane for wide probe blocks (KT_VEC_MINP) on the
# box and times P = 16 / 32 on the headline graph against the default build.
set -e
mkdir -p gpurun_out/v4
timeout -k 10 500 python tools/sweep_block.py --config sf1m --nprobes 512 --blocks 16,32 --variants ntyk2_lanes3,ntyk2 > gpurun_out/v4/base.txt 2>&1
for MINP in 32 16; do
  make -C krylov_robustness_amd/csrc -j16 BUILD=../../build/v$MINP EXTRA=-DKT_VEC_MINP=$MINP > gpurun_out/v4/build$MINP.log 2>&1
  timeout -k 10 500 python tools/sweep_block.py --config sf1m --nprobes 512 --blocks 16,32 --variants ntyk2_lanes3,ntyk2 > gpurun_out/v4/minp$MINP.txt 2>&1
done
echo done

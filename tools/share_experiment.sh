# Plain default bench line + one rank's share at N = 2/4/8 (1024/N probes) measured on one GPU.
set -e
mkdir -p gpurun_out/share
timeout -k 10 600 python bench.py > gpurun_out/share/bench_default.json 2> gpurun_out/share/bench_default.err
cat gpurun_out/share/bench_default.json
for np in 512 256 128; do
  for l in 1 2 3; do
    timeout -k 10 300 python bench.py --nprobes $np --lanes $l --cpu-seconds 0 --steps 10 --no-profile > gpurun_out/share/share_${np}_l$l.json 2>> gpurun_out/share/share.err
    python3 -c "import json,sys; d=json.load(open('gpurun_out/share/share_${np}_l$l.json')); print('probes $np lanes $l ms/eval', d['ms_per_step'])"
  done
done
timeout -k 10 300 python bench.py --config er100k --cpu-seconds 10 > gpurun_out/share/bench_er100k.json 2>> gpurun_out/share/share.err
timeout -k 10 300 python bench.py --config er100k --cpu-seconds 0 --explicit > gpurun_out/share/bench_er100k_explicit.json 2>> gpurun_out/share/share.err
cat gpurun_out/share/bench_er100k.json gpurun_out/share/bench_er100k_explicit.json

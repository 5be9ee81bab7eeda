set -o pipefail
bash tools/gpu_run.sh tests r05a || exit 1
bash tools/gpu_run.sh smoke r05a || exit 1
mkdir -p gpurun_out/r05a/cfg
for s in bench_config1 bench_config3; do
  timeout -k 10 300 python tests/perf/$s.py > gpurun_out/r05a/cfg/$s.json 2> gpurun_out/r05a/cfg/$s.err || exit 1
  KT_TSQR_GRAPH=0 timeout -k 10 300 python tests/perf/$s.py > gpurun_out/r05a/cfg/${s}_nograph.json 2> gpurun_out/r05a/cfg/${s}_nograph.err || exit 1
done

#!/bin/bash
# Secondary-config measurements in one GPU call (each JSON line under gpurun_out/TAG/).
# Usage (GPU box, repo root): bash tools/gpu_configs.sh TAG
set -o pipefail
TAG=${1:-cfg}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for s in bench_config1 bench_config3 bench_greedy bench_hessian; do
    timeout -k 10 300 python tests/perf/$s.py > $OUT/$s.json 2> $OUT/$s.err || { echo "$s FAILED"; tail -5 $OUT/$s.err; exit 1; }
    echo "== $s"; cut -c1-600 $OUT/$s.json
done
timeout -k 10 300 python bench.py --config er100k --steps 20 --warmup 2 --cpu-seconds 5 > $OUT/bench_er100k.json 2> $OUT/bench_er100k.err || { tail -5 $OUT/bench_er100k.err; exit 1; }
echo "== er100k"; cut -c1-300 $OUT/bench_er100k.json

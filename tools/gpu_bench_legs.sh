#!/bin/bash
# Bench legs on the GPU box (repo root): default line, weighted, mc_trace headline.
# Usage: bash tools/gpu_bench_legs.sh TAG
set -o pipefail
TAG=${1:-dev}
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 400 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
cut -c1-400 $O/bench_default.json
timeout -k 10 400 python -u bench.py --weighted --cpu-seconds 0 > $O/bench_weighted.json 2> $O/bench_weighted.err || { tail -20 $O/bench_weighted.err; exit 1; }
timeout -k 10 400 python -u bench.py --estimator mc_trace --steps 10 --cpu-seconds 0 > $O/bench_mc.json 2> $O/bench_mc.err || { tail -20 $O/bench_mc.err; exit 1; }
echo done

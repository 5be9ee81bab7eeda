#!/bin/bash
# One GPU call: parity tests, block sweep, bench, rocprof kernel stats + HBM counters.
# Usage (on the GPU box, from the repo root): bash tools/gpu_round.sh TAG [sweep-blocks]
set -o pipefail
TAG=${1:-r01}
BLOCKS=${2:-8,16,32,64,128}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 400 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/sweep_block.py --nprobes 256 --blocks $BLOCKS > $OUT/sweep.log 2>&1 || exit $?
cat $OUT/sweep.log
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --cpu-seconds 10 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json

#!/bin/bash
# Config 5 host path: greedy parity tests, bench (3 repeats), kernel-trace gap analysis.
set -o pipefail
O=gpurun_out/gh; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_greedy.py tests/test_gpu_datasets.py tests/test_gpu_krylov.py > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
timeout -k 10 300 python tests/perf/bench_greedy.py --cpu-steps 0 --repeat 3 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cut -c1-260 $O/bench.json
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $PWD/$O/prof -o g -- python3 tests/perf/bench_greedy.py --cpu-steps 0 --repeat 1 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
F=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python3 tools/gaps.py $F k_pair_reg 0 | head -12

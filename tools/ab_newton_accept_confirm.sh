#!/bin/bash
# Newton acceptance at 2^20 atol as the default: every GPU test, then config 5 bench_greedy.
set -o pipefail
O=gpurun_out/naccc; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for r in 1 2; do
  timeout -k 10 200 python tests/perf/bench_greedy.py --cpu-steps 0 > $O/b.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('$O/b.json')); print(round(d['gpu_seconds']*1e3,2), 'ms', d['rob_variation'], d['first_edges'])"
done

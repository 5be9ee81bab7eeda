#!/bin/bash
# expmv host stop flag (default) vs queueing every term (KT_EXPMV_STOPFLAG=0): tests, trace_exp(A6) timings, config-1 bench.
set -o pipefail
O=gpurun_out/sf; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_mctrace.py tests/test_gpu_mctrace_sharded.py > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
for r in 1 2 3; do
  for v in 0 1; do
    KT_EXPMV_STOPFLAG=$v timeout -k 10 120 python tools/run_trace_exp_expmv.py > $O/x.txt 2>&1 || { tail -5 $O/x.txt; exit 1; }
    echo "stopflag=$v $(grep trace_exp $O/x.txt)"
  done
done
timeout -k 10 300 python tests/perf/bench_config1.py > $O/c1.json 2> $O/c1.err || { tail -5 $O/c1.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/c1.json').read().strip().splitlines()[-1]); print('config1 trace_exp_expmv', d['trace_exp_expmv']['device_s'], 'rel_vs_oracle', d['trace_exp_expmv']['rel_vs_oracle'])"

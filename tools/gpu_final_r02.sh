#!/bin/bash
# Round-2 closing check in one call: every GPU test, smoke, the default bench
# (rocprofv3 kernel stats of the same command), secondary configs.
set -o pipefail
O=gpurun_out/final5; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
grep smoke $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-700 $O/bench.json
bash tools/gpu_configs.sh final5_cfg || exit 1

# Round 3 closing evidence: -m gpu suite, smoke, default bench, secondary configs, rocprof of the default command
set -e
O=gpurun_out/r03close; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err; cut -c1-300 $O/bench.json
bash tools/gpu_configs.sh r03close_cfg
bash tools/prof_closing.sh

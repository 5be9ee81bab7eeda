# Round 3 re-entry: the whole -m gpu suite, smoke and the default bench on HEAD, then the secondary configs.
set -e
O=gpurun_out/r03b; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
tail -3 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err
cut -c1-400 $O/bench.json
bash tools/gpu_configs.sh r03b_cfg

set -e
O=gpurun_out/r03n; mkdir -p $O
timeout -k 10 300 python tests/perf/bench_config3.py > $O/c3.json 2>$O/c3.err; tail -1 $O/c3.json
timeout -k 10 300 python tests/perf/bench_greedy.py > $O/g.json 2>$O/g.err; tail -1 $O/g.json | cut -c1-300
timeout -k 10 300 python -u -m pytest tests/test_gpu_greedy.py tests/test_gpu_configs.py -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu_prof.sh r03prof
cat gpurun_out/r03prof/traffic.json | head -30

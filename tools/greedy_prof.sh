# Config-5 greedy: parity tests, bench (3 repeats), rocprofv3 kernel stats.
set -e
mkdir -p gpurun_out/gp
timeout -k 10 400 python -m pytest tests/test_gpu_greedy.py tests/test_gpu_datasets.py -q -x > gpurun_out/gp/tests.log 2>&1
timeout -k 10 300 python tests/perf/bench_greedy.py --cpu-steps 0 --repeat 3 > gpurun_out/gp/bench.json 2> gpurun_out/gp/bench.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/gp/prof -o run -- python3 $GRAFT_REPO_ROOT/tests/perf/bench_greedy.py --cpu-steps 0 --repeat 1 > $GRAFT_REPO_ROOT/gpurun_out/gp/prof.log 2>&1
echo done

# A/B of mc_trace's round layouts at config 4 (bench.py --estimator mc_trace):
# the default layout, the next-S-term guess (KT_MC_AHEAD=1:
# always ahead = one 32-wide explicit sweep per round), every column explicit
# (KT_LC_YFORM=0); then the default bench.  Results in gpurun_out/ab1/.
set -o pipefail
mkdir -p gpurun_out/ab1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_mctrace.py tests/test_gpu_mctrace_sharded.py tests/test_gpu_config4.py > gpurun_out/ab1/tests.log 2>&1 || exit 1
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --estimator mc_trace --steps 8 --cpu-seconds 0 --ref-cpu-seconds 0 \
    > gpurun_out/ab1/bench_$name.json 2> gpurun_out/ab1/bench_$name.err
}
run layout_default || exit 1
run ahead1 KT_MC_AHEAD=1 || exit 1
run explicit KT_LC_YFORM=0 || exit 1
timeout -k 10 400 python bench.py > gpurun_out/ab1/bench_default.json 2> gpurun_out/ab1/bench_default.err || exit 1

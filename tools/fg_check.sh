set -e
mkdir -p gpurun_out/fg
timeout -k 10 600 python -m pytest tests/test_gpu_krylov.py tests/test_gpu_frechet.py tests/test_gpu_fme.py tests/test_gpu_mctrace.py -q -x > gpurun_out/fg/tests.log 2>&1
KT_EIG_STATS=1 timeout -k 10 200 python tools/prof_fg.py > gpurun_out/fg/run.log 2>&1
timeout -k 10 300 python tests/perf/bench_config3.py > gpurun_out/fg/config3.json 2> gpurun_out/fg/config3.err

# Headline refresh on the GPU box: probe-path tests, rocprofv3 passes
# (tools/gpu_prof.sh), then the default bench line.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_slq.py tests/test_gpu_mctrace.py -q -x > gpurun_out/slq_tests.log 2>&1
bash tools/gpu_prof.sh r01
timeout -k 10 600 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
echo done

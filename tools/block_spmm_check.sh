set -e
mkdir -p gpurun_out/ck
timeout -k 10 800 python -m pytest tests/test_gpu_datasets.py tests/test_gpu_greedy.py tests/test_gpu_krylov.py tests/test_gpu_fme.py tests/test_gpu_frechet.py tests/test_gpu_centrality.py tests/test_gpu_mctrace.py tests/test_gpu_qr.py -q -x > gpurun_out/ck/tests.log 2>&1
timeout -k 10 300 python tests/perf/bench_greedy.py --graph as_735 --miobi make --cpu-steps 0 --repeat 2 > gpurun_out/ck/as735.json 2>/dev/null
timeout -k 10 300 python tests/perf/bench_greedy.py --cpu-steps 0 --repeat 3 > gpurun_out/ck/india.json 2>/dev/null
echo done

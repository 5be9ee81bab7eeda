# config 3 / config 1 kernel-trace gap analysis after the round-3 changes, plus a quick parity check of the cleaned build
set -e
timeout -k 10 300 python -u -m pytest tests/test_gpu_krylov.py tests/test_gpu_configs.py tests/test_gpu_omega_sweep.py -x -q --timeout 240 --timeout-method thread > gpurun_out/r03e_tests.log 2>&1 || { tail -20 gpurun_out/r03e_tests.log; exit 1; }
tail -1 gpurun_out/r03e_tests.log
bash tools/gaps_c13.sh

# fill-kernel experiment, the Omega-sweep test, then the y-form pass diagnostics
set -e
bash tools/fg_exp_prof7.sh
timeout -k 10 300 python -u -m pytest tests/test_gpu_omega_sweep.py -x -v --timeout 240 --timeout-method thread > gpurun_out/omega_test.log 2>&1 || { tail -30 gpurun_out/omega_test.log; exit 1; }
tail -2 gpurun_out/omega_test.log
bash tools/ky_diag.sh
cat gpurun_out/kydiag/timing.jsonl

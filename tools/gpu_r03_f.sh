# one-launch-per-column Householder sweep: parity, then config 3 A/B
set -e
O=gpurun_out/r03f; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_qr.py tests/test_gpu_krylov.py tests/test_gpu_configs.py tests/test_gpu_omega_sweep.py tests/test_gpu_mctrace.py tests/test_gpu_fme.py tests/test_gpu_frechet.py -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  KT_TSQR_STEP1=0 timeout -k 10 120 python tools/prof_fg.py > $O/fg_two$r.txt 2>&1; echo "two-launch: $(grep '^fg' $O/fg_two$r.txt | cut -c1-10 | tr '\n' ' ')"
  timeout -k 10 120 python tools/prof_fg.py > $O/fg_one$r.txt 2>&1; echo "one-launch: $(grep '^fg' $O/fg_one$r.txt | cut -c1-10 | tr '\n' ' ')"
done
timeout -k 10 200 python tests/perf/bench_config3.py > $O/c3.json 2>&1; tail -1 $O/c3.json | cut -c1-900
timeout -k 10 200 python tests/perf/bench_config1.py > $O/c1.json 2>&1; tail -1 $O/c1.json | cut -c1-900

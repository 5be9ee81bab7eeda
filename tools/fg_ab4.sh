set -e
O=gpurun_out/fgab4; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_krylov.py tests/test_gpu_configs.py tests/test_gpu_frechet.py tests/test_gpu_fme.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || true
for r in 1 2; do
KT_NORM_POW=0 timeout -k 10 120 python tools/prof_fg.py > $O/nopow$r.txt 2>&1
timeout -k 10 120 python tools/prof_fg.py > $O/pow$r.txt 2>&1
done
KT_FG_TIMING=1 timeout -k 10 120 python tools/prof_fg.py > $O/phases.txt 2>&1

# shifted CholeskyQR3 for block Arnoldi (KT_QR_SHIFTED=1): parity under it, then an in-process A/B on config 3
set -e
O=gpurun_out/r03p; mkdir -p $O
KT_QR_SHIFTED=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_krylov.py tests/test_gpu_configs.py tests/test_gpu_omega_sweep.py tests/test_gpu_frechet.py -x -q --timeout 240 --timeout-method thread > $O/par.log 2>&1 || { tail -40 $O/par.log; exit 1; }
tail -1 $O/par.log
timeout -k 10 300 python tools/fg_ab_inproc.py 24 KT_DUMMY=1 KT_QR_SHIFTED=1 KT_QR_SHIFTED=1,KT_TSQR_PERSIST=2 > $O/ab.txt 2>&1; cat $O/ab.txt

# device-side shifted CholeskyQR3: parity, then in-process A/B on config 3 and the India exp driver timing
set -e
O=gpurun_out/r03q; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_qr.py tests/test_gpu_krylov.py tests/test_gpu_configs.py tests/test_gpu_omega_sweep.py tests/test_gpu_frechet.py -x -q --timeout 240 --timeout-method thread > $O/par.log 2>&1 || { tail -40 $O/par.log; exit 1; }
tail -1 $O/par.log
timeout -k 10 300 python tools/fg_ab_inproc.py 24 KT_DUMMY=1 KT_QR_SHIFTED=0 > $O/ab.txt 2>&1; cat $O/ab.txt
timeout -k 10 120 python tools/prof_fg_exp.py > $O/fgexp.txt 2>&1; grep fg_exp $O/fgexp.txt | tr '\n' ' '

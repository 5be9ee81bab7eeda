# one-barrier persistent Householder sweep (KT_TSQR_PERSIST=2): parity, then config 3 A/B
set -e
O=gpurun_out/r03o; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_qr.py -x -q --timeout 120 --timeout-method thread > $O/qr.log 2>&1 || { tail -30 $O/qr.log; exit 1; }
tail -1 $O/qr.log
KT_TSQR_PERSIST=2 timeout -k 10 400 python -u -m pytest tests/test_gpu_krylov.py tests/test_gpu_configs.py tests/test_gpu_omega_sweep.py -x -q --timeout 240 --timeout-method thread > $O/par.log 2>&1 || { tail -30 $O/par.log; exit 1; }
tail -1 $O/par.log
for r in 1 2; do
  KT_FG_REPS=8 timeout -k 10 200 python tools/prof_fg.py > $O/fg_def$r.txt 2>&1; echo "default: $(grep '^fg' $O/fg_def$r.txt | cut -c4-9 | tr '\n' ' ')"
  KT_TSQR_PERSIST=2 KT_FG_REPS=8 timeout -k 10 200 python tools/prof_fg.py > $O/fg_p2$r.txt 2>&1; echo "persist2: $(grep '^fg' $O/fg_p2$r.txt | cut -c4-9 | tr '\n' ' ')"
done

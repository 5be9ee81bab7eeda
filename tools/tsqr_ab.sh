#!/bin/bash
# Persistent reflector sweep (k_ts_qr) vs two launches per column: QR / block-Krylov
# parity tests, then config 3 and the Hessian driver under each form.
set -o pipefail
O=gpurun_out/tsqr; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_qr.py tests/test_gpu_krylov.py tests/test_gpu_mctrace.py tests/test_gpu_frechet.py tests/test_gpu_fme.py tests/test_gpu_greedy.py > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
for r in 1 2; do
  for v in 0 1; do
    KT_TSQR_PERSIST=$v timeout -k 10 300 python tests/perf/bench_config3.py > $O/c3_$v.json 2> $O/c3_$v.err || { tail -5 $O/c3_$v.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/c3_$v.json').read().strip().splitlines()[-1]); print('persist=$v config3 fg_s', round(d['fg_s']*1e3,2), 'ms  pipeline', round(d['device_pipeline_s']*1e3,2), 'ms  fg_f_rel', d['fg_f_rel_diff'], 'gr_rel', d['fg_gr_rel_diff'])"
    KT_TSQR_PERSIST=$v timeout -k 10 300 python tests/perf/bench_hessian.py > $O/h_$v.json 2> $O/h_$v.err || { tail -5 $O/h_$v.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/h_$v.json').read().strip().splitlines()[-1]); print('persist=$v hessian fg_s', round(d['fg_s']*1e3,2), 'hess_s', round(d['hessian_s']*1e3,2), d['fg_f_rel_diff'], d['hessian_rel_diff'])"
    KT_TSQR_PERSIST=$v timeout -k 10 120 python tools/run_trace_exp_expmv.py > $O/x_$v.txt 2>&1 || { tail -5 $O/x_$v.txt; exit 1; }
    echo "persist=$v $(grep trace_exp $O/x_$v.txt)"
  done
done

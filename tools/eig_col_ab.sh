#!/bin/bash
# Host eigenvalues by column tridiagonalisation (default) vs tred2 (KT_EIG_COLTRIDIAG=0): tests, config 3, Hessian driver.
set -o pipefail
O=gpurun_out/ec; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_krylov.py tests/test_gpu_frechet.py tests/test_gpu_fme.py tests/test_gpu_mctrace.py tests/test_gpu_greedy.py tests/test_gpu_datasets.py tests/test_host_eig.py > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
for r in 1 2; do
  for v in 0 1; do
    KT_EIG_COLTRIDIAG=$v timeout -k 10 300 python tests/perf/bench_config3.py > $O/c3_$v.json 2> $O/c3_$v.err || { tail -5 $O/c3_$v.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/c3_$v.json').read().strip().splitlines()[-1]); print('coltri=$v config3 fg', round(d['fg_s']*1e3,2), 'ms pipeline', round(d['device_pipeline_s']*1e3,2), 'fg_f_rel', d['fg_f_rel_diff'], 'gr_rel', d['fg_gr_rel_diff'])"
    KT_EIG_COLTRIDIAG=$v timeout -k 10 300 python tests/perf/bench_hessian.py > $O/h_$v.json 2> $O/h_$v.err || { tail -5 $O/h_$v.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/h_$v.json').read().strip().splitlines()[-1]); print('coltri=$v hessian fg', round(d['fg_s']*1e3,2), 'hess', round(d['hessian_s']*1e3,2), d['fg_f_rel_diff'], d['hessian_rel_diff'])"
  done
done

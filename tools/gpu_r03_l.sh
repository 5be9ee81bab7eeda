# persistent twin / speculative threads: parity, then config 3 (10 calls) and config 1 timing
set -e
O=gpurun_out/r03l; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_mctrace.py tests/test_gpu_mctrace_sharded.py tests/test_gpu_krylov.py tests/test_gpu_configs.py -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
KT_FG_REPS=10 timeout -k 10 200 python tools/prof_fg.py > $O/fg.txt 2>&1; echo "fg: $(grep '^fg' $O/fg.txt | cut -c1-10 | tr '\n' ' ')"
KT_FG_REPS=10 timeout -k 10 200 python tools/prof_fg.py > $O/fg2.txt 2>&1; echo "fg: $(grep '^fg' $O/fg2.txt | cut -c1-10 | tr '\n' ' ')"
for r in 1 2; do timeout -k 10 200 python tests/perf/bench_config1.py > $O/c1.json 2>&1
python3 -c "import json; d=json.loads(open('$O/c1.json').read().strip().splitlines()[-1]); print('config1 expmv', round(d['trace_exp_expmv']['device_s']*1e3,2), 'ms, lanczos round', round(d['mc_trace_lanczos_round']['device_s']*1e3,2), 'ms, trace_exp lanczos', round(d['trace_exp_lanczos']['device_s']*1e3,2))"; done
timeout -k 10 120 python tools/prof_fg_exp.py > $O/fgexp.txt 2>&1; grep fg_exp $O/fgexp.txt | tr '\n' ' '

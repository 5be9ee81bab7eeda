# host launch rate from 1-4 threads, and config 1's trace_exp (expmv Afun) variants
set -e
O=gpurun_out/r03h; mkdir -p $O
timeout -k 10 120 ./tools/launch_rate/launch_rate > $O/launch_rate.txt 2>&1; cat $O/launch_rate.txt
for v in "KT_DUMMY=1" "KT_EXPMV_STOPFLAG=0" "KT_MC_SPEC=0" "KT_TWIN=0"; do
  env $v timeout -k 10 200 python tests/perf/bench_config1.py > $O/c1.json 2>&1
  python3 -c "import json; d=json.loads(open('$O/c1.json').read().strip().splitlines()[-1]); print('$v', 'expmv', round(d['trace_exp_expmv']['device_s']*1e3,2), 'ms')"
done

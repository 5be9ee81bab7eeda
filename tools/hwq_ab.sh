# Does the 20-30 ms first-dispatch stall of the pipelined fun_update follow the HSA queue count?
set -e
O=gpurun_out/hwq; mkdir -p $O
for q in 1 2 4 8; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 120 python tools/prof_fg_exp.py > $O/fgexp_q$q.txt 2>&1
  echo "== q$q"; grep fg_exp $O/fgexp_q$q.txt | tr '\n' ' '; echo
done
for q in 1 2 4; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 120 python tools/prof_fg.py > $O/fg3_q$q.txt 2>&1
  echo "== config3 fg q$q"; grep "^fg" $O/fg3_q$q.txt | tr '\n' ' '; echo
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python tests/perf/bench_config1.py > $O/c1_q$q.json 2>&1
  python3 -c "import json,sys; d=json.loads(open('$O/c1_q$q.json').read().strip().splitlines()[-1]); print('config1 q$q expmv', d['trace_exp_expmv']['device_s'], 'lanczos', d['trace_exp_lanczos']['device_s'])"
done

set -e
O=gpurun_out/r03m; mkdir -p $O
KT_GEMM_TS_MIN_N=0 timeout -k 10 120 python tools/prof_fg_exp.py > $O/fgexp_ts.txt 2>&1; echo "India ts: $(grep fg_exp $O/fgexp_ts.txt | cut -c1-15 | tr '\n' ' ')"
timeout -k 10 120 python tools/prof_fg_exp.py > $O/fgexp.txt 2>&1; echo "India default: $(grep fg_exp $O/fgexp.txt | cut -c1-15 | tr '\n' ' ')"
timeout -k 10 200 python tests/perf/bench_config3.py > $O/c3.json 2>&1
python3 -c "import json; d=json.loads(open('$O/c3.json').read().strip().splitlines()[-1]); print({k: d[k] for k in ('normest_s','tr_sinh_slq_s','fme_s','fg_s','device_pipeline_s','fg_f_rel_diff','fme_max_rel_diff')})"
timeout -k 10 200 python tests/perf/bench_hessian.py > $O/h.json 2>&1; tail -1 $O/h.json | cut -c1-400
timeout -k 10 200 python tests/perf/bench_greedy.py > $O/g.json 2>&1; tail -1 $O/g.json | cut -c1-300

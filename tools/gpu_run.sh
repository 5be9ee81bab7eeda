#!/bin/bash
# One parametrised GPU-box script for the round's measurements (replaces the
# per-call lease scripts).  Run from the repo root on the GPU box:
#   bash tools/gpu_run.sh TASK TAG [extra bench args]
# TASK
#   tests    the -m gpu suite (pytest, one process)           -> gpu_tests.log
#   smoke    __graft_entry__.smoke()                           -> smoke.log
#   bench    bench legs: default line, --weighted, --estimator mc_trace, er100k
#   configs  secondary configs (tests/perf/bench_*.py) + er100k bench
#   prof     rocprofv3 --kernel-trace --stats of the default bench command,
#            reconciled with the line it printed (tools/reconcile_trace.py)
#   secondary latency floors (tools/latency_floor) + kernel stats of the
#            config-1/3/5 drivers under rocprofv3
#   timeline rocprofv3 kernel trace of the er100k bench, per-evaluation
#            breakdown (tools/eval_timeline.py)
#   mctl     kernel trace of the mc_trace leg, per-evaluation breakdown
#            (tools/mc_timeline.py)
#   rehearse `python bench.py --gpus 2` (self-launched ranks) on one GPU, gloo
#   pmc      FETCH_SIZE / WRITE_SIZE passes (separate runs) of `bench.py
#            --steps 1 --lanes 1 [extra]` -> traffic.json section
#            (SECTION env, default sf1m)
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
TASK=$1; TAG=${2:-dev}; shift 2 || true
O=$PWD/gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
case $TASK in
tests)
    timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" \
        > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
    tail -3 $O/gpu_tests.log ;;
smoke)
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
    tail -1 $O/smoke.log ;;
bench)
    timeout -k 10 400 python -u bench.py "$@" > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
    timeout -k 10 400 python -u bench.py --weighted --cpu-seconds 0 > $O/bench_weighted.json 2> $O/bench_weighted.err || { tail -20 $O/bench_weighted.err; exit 1; }
    timeout -k 10 400 python -u bench.py --estimator mc_trace --steps 20 --cpu-seconds 0 > $O/bench_mc_trace.json 2> $O/bench_mc_trace.err || { tail -20 $O/bench_mc_trace.err; exit 1; }
    timeout -k 10 400 python -u bench.py --config er100k --steps 100 --warmup 5 --cpu-seconds 5 > $O/bench_er100k.json 2> $O/bench_er100k.err || { tail -20 $O/bench_er100k.err; exit 1; }
    for f in bench_default bench_weighted bench_mc_trace bench_er100k; do echo "== $f"; cut -c1-300 $O/$f.json; done ;;
configs)
    for s in bench_config1 bench_config3 bench_greedy bench_hessian; do
        timeout -k 10 300 python tests/perf/$s.py > $O/$s.json 2> $O/$s.err || { echo "$s FAILED"; tail -5 $O/$s.err; exit 1; }
        echo "== $s"; cut -c1-400 $O/$s.json
    done ;;
prof)
    ( cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o def \
        -- python3 $GRAFT_REPO_ROOT/bench.py "$@" > $O/bench.json 2> $O/bench.err ) || { tail -20 $O/bench.err; exit 1; }
    cp $(find $O/stats -name "*kernel_stats.csv") $O/kernel_stats.csv
    python3 tools/reconcile_trace.py $(find $O/stats -name "*kernel_trace.csv") $O/bench.json $O/reconcile.json || exit 1
    rm -f $(find $O/stats -name "*kernel_trace.csv")
    cat $O/reconcile.json; head -6 $O/kernel_stats.csv | cut -c1-200 ;;
timeline)
    # kernel trace of the er100k bench (config 2), evaluation by evaluation
    ( cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/tl -o tl \
        -- python3 $GRAFT_REPO_ROOT/bench.py --config er100k --steps 100 --warmup 5 --cpu-seconds 0 --mc-steps 0 "$@" \
        > $O/bench_er100k_traced.json 2> $O/tl.err ) || { tail -20 $O/tl.err; exit 1; }
    python3 tools/eval_timeline.py $(find $O/tl -name "*kernel_trace.csv") ${SWEEPS:-2} 100 $O/er100k_eval_timeline.json || exit 1
    gzip -f $(find $O/tl -name "*kernel_trace.csv") ;;
secondary)
    # latency floors + rocprofv3 kernel stats of the secondary configs' drivers
    timeout -k 10 120 tools/latency_floor/latency_floor > $O/latency_floor.txt 2>&1 || { cat $O/latency_floor.txt; exit 1; }
    cat $O/latency_floor.txt
    for s in bench_config1 bench_config3 bench_greedy; do
        ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/st_$s -o $s \
            -- python3 $GRAFT_REPO_ROOT/tests/perf/$s.py > $O/$s.json 2> $O/$s.err ) || { tail -5 $O/$s.err; exit 1; }
        cp $(find $O/st_$s -name "*kernel_stats.csv") $O/${s}_kernel_stats.csv
        gzip -f $(find $O/st_$s -name "*kernel_trace.csv")
        echo "== $s"; cut -c1-300 $O/$s.json
    done ;;
mctl)
    # kernel trace of the mc_trace leg (trace_exp, Lanczos-exp Afun), evaluation by evaluation
    ( cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/mctl -o mctl \
        -- python3 $GRAFT_REPO_ROOT/bench.py --estimator mc_trace --steps 10 --cpu-seconds 0 --ref-cpu-seconds 0 \
        --no-profile "$@" > $O/bench_mc_traced.json 2> $O/mctl.err ) || { tail -20 $O/mctl.err; exit 1; }
    python3 tools/mc_timeline.py $(find $O/mctl -name "*kernel_trace.csv") 10 $O/mc_timeline.json || exit 1
    gzip -f $(find $O/mctl -name "*kernel_trace.csv") ;;
rehearse)
    # the driver's N = 2 command as it may run it (no torchrun: bench.py starts
    # the ranks itself), both ranks on GPU 0 over gloo, default config
    KT_BENCH_ONE_DEVICE=1 timeout -k 10 500 python -u bench.py --gpus 2 --dist-backend gloo "$@" \
        > $O/bench_2ranks_self_launch.json 2> $O/bench_2ranks_self_launch.err || { tail -20 $O/bench_2ranks_self_launch.err; exit 1; }
    cut -c1-400 $O/bench_2ranks_self_launch.json ;;
pmc)
    SEC=${SECTION:-sf1m}
    B="$GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 --cpu-seconds 0 --lanes 1 --mc-steps 1 --no-profile $*"
    R="spmm_dot|spmm_lanczos|k_update"
    ( cd /tmp && timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$R" -d $O/pmc_fetch -o f --output-format csv -- python3 $B > $O/pmc_fetch.log 2>&1 ) || { tail -20 $O/pmc_fetch.log; exit 1; }
    ( cd /tmp && timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$R" -d $O/pmc_write -o w --output-format csv -- python3 $B > $O/pmc_write.log 2>&1 ) || { tail -20 $O/pmc_write.log; exit 1; }
    ( cd /tmp && timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "$R" -d $O/pmc_hit -o h --output-format csv -- python3 $B > $O/pmc_hit.log 2>&1 ) || { tail -20 $O/pmc_hit.log; exit 1; }
    python3 tools/pmc_traffic.py $(find $O/pmc_fetch -name "*counter_collection.csv") $(find $O/pmc_write -name "*counter_collection.csv") $O/traffic.json $SEC \
        $(find $O/pmc_hit -name "*counter_collection.csv") || exit 1 ;;
expmv)
    # the reference composition at config 4 (tools/expmv_c4.py): kernel trace
    # of the default term kernel and of the KT_EXPMV_ROWS=0 split kernel
    # (per-term statistics, tools/expmv_terms.py), then FETCH / WRITE / hit
    # passes of the default term kernel (tools/pmc_traffic.py, section expmv_c4)
    for v in rows split; do
        E=""; [ $v = split ] && E="KT_EXPMV_ROWS=0"
        ( cd /tmp && env $E timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_$v -o c4 \
            -- python3 $GRAFT_REPO_ROOT/tools/expmv_c4.py 1 > $O/c4_$v.jsonl 2> $O/c4_$v.err ) || { tail -20 $O/c4_$v.err; exit 1; }
        cp $(find $O/tr_$v -name "*kernel_stats.csv") $O/kernel_stats_$v.csv
        python3 tools/expmv_terms.py $(find $O/tr_$v -name "*kernel_trace.csv") $O/terms_$v.json || exit 1
        rm -f $(find $O/tr_$v -name "*kernel_trace.csv")
        cat $O/c4_$v.jsonl
    done
    B="$GRAFT_REPO_ROOT/tools/expmv_c4.py 1"
    R="k_expmv_rows"
    ( cd /tmp && timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$R" -d $O/pmc_fetch -o f --output-format csv -- python3 $B > $O/pmc_fetch.log 2>&1 ) || { tail -20 $O/pmc_fetch.log; exit 1; }
    ( cd /tmp && timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$R" -d $O/pmc_write -o w --output-format csv -- python3 $B > $O/pmc_write.log 2>&1 ) || { tail -20 $O/pmc_write.log; exit 1; }
    ( cd /tmp && timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "$R" -d $O/pmc_hit -o h --output-format csv -- python3 $B > $O/pmc_hit.log 2>&1 ) || { tail -20 $O/pmc_hit.log; exit 1; }
    python3 tools/pmc_traffic.py $(find $O/pmc_fetch -name "*counter_collection.csv") $(find $O/pmc_write -name "*counter_collection.csv") $O/traffic.json expmv_c4 \
        $(find $O/pmc_hit -name "*counter_collection.csv") || exit 1
    rm -f $(find $O/pmc_fetch $O/pmc_write $O/pmc_hit -name "*counter_collection.csv")
    cat $O/traffic.json ;;
*)
    echo "unknown task $TASK"; exit 2 ;;
esac

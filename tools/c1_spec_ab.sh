set -e
O=gpurun_out/c1spec; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_mctrace.py tests/test_gpu_mctrace_sharded.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || true
for r in 1 2; do
KT_MC_SPEC=0 timeout -k 10 300 python tests/perf/bench_config1.py > $O/nospec$r.json 2>$O/nospec$r.err
timeout -k 10 300 python tests/perf/bench_config1.py > $O/spec$r.json 2>$O/spec$r.err
done

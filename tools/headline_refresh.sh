# Headline refresh on the GPU box: probe-path tests, rocprofv3 passes
# (tools/gpu_prof.sh: stats + FETCH/WRITE PMC passes), then the default bench
# command under rocprofv3 --kernel-trace (tools/prof_default_cmd.sh) and its
# reconciliation with the bench line.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_slq.py tests/test_gpu_mctrace.py -q -x > gpurun_out/slq_tests.log 2>&1
bash tools/gpu_prof.sh r01
cp gpurun_out/r01/traffic.json profiles/traffic.json
bash tools/prof_default_cmd.sh
python3 tools/reconcile_trace.py gpurun_out/defcmd/kernel_trace.csv gpurun_out/defcmd/bench.json gpurun_out/defcmd/reconcile.json
echo done

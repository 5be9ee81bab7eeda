# Round 3, first GPU pass: CPU share probe, the whole -m gpu suite, smoke, default bench.
set -e
mkdir -p gpurun_out/r03a
{ nproc; python -c "import os; print('affinity', len(os.sched_getaffinity(0)))"; cat /sys/fs/cgroup/cpu.max 2>/dev/null || echo no-cpu.max; echo "OMP=$OMP_NUM_THREADS"; } > gpurun_out/r03a/cpu_share.txt 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03a/gpu_tests.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03a/smoke.log 2>&1
timeout -k 10 600 python bench.py > gpurun_out/r03a/bench.json 2> gpurun_out/r03a/bench.err
echo done

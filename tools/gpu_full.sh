set -e
mkdir -p gpurun_out/full
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/full/gpu_tests.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/full/smoke.log 2>&1
timeout -k 10 600 python bench.py > gpurun_out/full/bench.json 2> gpurun_out/full/bench.err
echo done

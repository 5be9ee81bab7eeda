# Block SpMM lane width (KT_BLK_VW): configs 3 and 5 and greedy make on as_735, default vs 4 doubles per lane.
set -e
mkdir -p gpurun_out/bv
run() {
  timeout -k 10 300 python tests/perf/bench_greedy.py --cpu-steps 0 --repeat 3 > gpurun_out/bv/india_$1.json 2>/dev/null
  timeout -k 10 300 python tests/perf/bench_greedy.py --graph as_735 --miobi make --cpu-steps 0 --repeat 2 > gpurun_out/bv/as735_$1.json 2>/dev/null
  timeout -k 10 300 python tools/prof_fg.py > gpurun_out/bv/fg_$1.txt 2>&1
}
run vw2
make -C krylov_robustness_amd/csrc -j16 BUILD=../../build/bv4 EXTRA=-DKT_BLK_VW=4 > gpurun_out/bv/build4.log 2>&1
timeout -k 10 400 python -m pytest tests/test_gpu_greedy.py tests/test_gpu_krylov.py -q -x > gpurun_out/bv/tests4.log 2>&1
run vw4
echo done

set -o pipefail
O=gpurun_out/gs2; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_greedy.py > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
for v in old nonewton new; do
  case $v in old) L=$PWD/build/old/libkrylov_old.so;; nonewton) L=$PWD/build/nonewton/libkrylov_nonewton.so;; new) L=$PWD/krylov_robustness_amd/libkrylov_hip.so;; esac
  KT_LIB=$L timeout -k 10 120 python tools/greedy_split.py > $O/split_$v.txt 2>/dev/null || exit 1
  KT_LIB=$L timeout -k 10 200 python tests/perf/bench_greedy.py --cpu-steps 0 > $O/bench_$v.json 2>/dev/null || exit 1
done
for v in old nonewton new; do echo "== $v"; cat $O/split_$v.txt; cut -c1-300 $O/bench_$v.json; done

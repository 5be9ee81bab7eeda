# rocprofv3 kernel stats of tests/perf/bench_greedy.py on one graph / mode: $1 graph, $2 break|make
set -e
OUT=$PWD/gpurun_out/gpg_$1_$2
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o g -- python3 $GRAFT_REPO_ROOT/tests/perf/bench_greedy.py --graph $1 --miobi $2 --cpu-steps 0 --repeat 1 > $OUT/bench.json 2> $OUT/bench.err
cp $(find $OUT/prof -name "*kernel_stats.csv") $OUT/kernel_stats.csv
echo done

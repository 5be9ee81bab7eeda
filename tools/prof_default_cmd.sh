# rocprofv3 kernel stats of the exact default bench command (default lanes, timed
# region + the isolated single-lane roofline pass + CPU baseline).
set -e
OUT=$PWD/gpurun_out/defcmd
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o def -- python3 $GRAFT_REPO_ROOT/bench.py > $OUT/bench.json 2> $OUT/bench.err
cp $(find $OUT/stats -name "*kernel_stats.csv") $OUT/kernel_stats.csv
cp $(find $OUT/stats -name "*kernel_trace.csv") $OUT/kernel_trace.csv
echo done

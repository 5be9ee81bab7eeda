# kernel stats of config 3's fun_and_grad with the one- and two-launch Householder sweeps
set -e
O=$PWD/gpurun_out/qrab; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/one -o k -- python3 tools/prof_fg.py > $O/one.txt 2>&1
KT_TSQR_STEP1=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/two -o k -- python3 tools/prof_fg.py > $O/two.txt 2>&1
for v in one two; do echo "== $v"; python3 - $(find $O/$v -name "*kernel_stats.csv") <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:10]:
    print(f"{r['Name'][:44]:44s} {int(r['Calls']):6d} {int(r['TotalDurationNs'])/1e6:8.2f} ms avg {float(r['AverageNs'])/1e3:7.2f} us")
PY
done

# rocprofv3 kernel stats of the config-5 greedy bench (device-queued loop)
set -e
O=gpurun_out/grprof; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/p -o run --output-format csv -- python3 tests/perf/bench_greedy.py --cpu-steps 0 --repeat 3 > $O/log.txt 2>&1
find $O/p -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/grprof/kernel_stats.csv")))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:10]:
    print(f'{r["Name"][:60]:60s} {int(r["Calls"]):6d} calls {float(r["AverageNs"])/1e3:8.2f} us avg {float(r["TotalDurationNs"])/1e6:8.2f} ms')
PY

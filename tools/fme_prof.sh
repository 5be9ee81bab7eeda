# rocprofv3 kernel stats of config 3's function_multiple_entries call (20 calls, pipelined form)
set -e
O=gpurun_out/fmeprof; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/p -o run --output-format csv -- python3 tools/fme_ab_inproc.py 20 KT_FME_PIPE=1 > $O/log.txt 2>&1
find $O/p -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/fmeprof/kernel_stats.csv")))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print(f'{r["Name"][:70]:70s} {int(r["Calls"]):6d} calls {float(r["AverageNs"])/1e3:8.2f} us avg {float(r["TotalDurationNs"])/1e6:8.2f} ms')
print("total kernel ms", tot / 1e6)
PY

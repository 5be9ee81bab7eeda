#!/bin/bash
# slq tests after the plan change, config 2 bench default, config-3 fg profile.
set -o pipefail
O=gpurun_out/b1; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_slq.py tests/test_gpu_bench.py > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
timeout -k 10 200 python bench.py --config er100k --steps 20 --warmup 3 --cpu-seconds 10 > $O/er.json 2> $O/er.err || { tail $O/er.err; exit 1; }
cut -c1-400 $O/er.json
bash tools/prof_fg.sh > $O/fg.txt 2>&1 || { tail $O/fg.txt; exit 1; }
grep "^fg" gpurun_out/fg/run.log | tail -2
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/fg/prof/**/*kernel_stats.csv", recursive=True)
rows = list(csv.DictReader(open(f[0])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print("kernel total ms", tot / 1e6)
for r in rows[:14]:
    print(r["Name"][:70], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "us avg", round(float(r["Percentage"]), 1), "%")
PY

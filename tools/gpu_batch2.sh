#!/bin/bash
# slq plan test; greedy kernel trace + gap analysis of the config-5 run.
set -o pipefail
O=gpurun_out/b2; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_slq.py > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $PWD/$O/prof -o g -- python3 tests/perf/bench_greedy.py --cpu-steps 0 --repeat 1 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
F=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python3 tools/gaps.py $F k_pair_reg 0 | head -30
python3 - "$F" <<'PY'
import csv, sys
rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(sys.argv[1])))
reg = [r for r in rows if "k_pair_reg" in r[2]]
d = sorted((e - s) / 1e3 for s, e, _ in reg)
print("k_pair_reg launches", len(reg), "median us", d[len(d)//2], "sum ms", sum(d) / 1e3)
if len(reg) > 1:
    print("first->last k_pair_reg span ms", (reg[-1][1] - reg[0][0]) / 1e6)
PY

#!/bin/bash
# rocprofv3 kernel trace of one trace_exp(A6) with the expmv Afun; prints the
# step-kernel duration statistics (tools/run_trace_exp_expmv.py).
set -o pipefail
OUT=gpurun_out/c1prof
rm -rf $OUT; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o c1 --output-format csv -- python tools/run_trace_exp_expmv.py > $OUT/out.txt 2>&1 || exit $?
grep trace_exp $OUT/out.txt
python - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/c1prof/c1_kernel_trace.csv")))
st = [r for r in rows if "expmv_step" in r["Kernel_Name"]]
d = sorted(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in st)
print("step kernels", len(st), "median ns", d[len(d) // 2], "p90", d[9 * len(d) // 10], "sum ms", sum(d) / 1e6)
for x in list(csv.DictReader(open("gpurun_out/c1prof/c1_kernel_stats.csv")))[:6]:
    print(x["Name"][:50], x["Calls"], x["AverageNs"], x["Percentage"])
PY

# PMC counters of the register candidate kernel (noeig build; one pass).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/regpmc; mkdir -p $O
rocprofv3 -L > $O/avail.txt 2>&1 || true
grep -o "SQ_[A-Z_0-9]*" $O/avail.txt | sort -u > $O/sq.txt || true
KT_LIB=$PWD/build/noeig/libkrylov_noeig.so timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_SALU -d $O/p1 -o run --output-format csv -- python3 tools/greedy_split.py > $O/run1.log 2>&1 || { tail -20 $O/run1.log; exit 1; }
find $O/p1 -name "*counter_collection.csv" | head -1 | xargs -I{} cp {} $O/c1.csv
python3 - <<'PY'
import csv, collections
rows = list(csv.DictReader(open("gpurun_out/regpmc/c1.csv")))
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in rows:
    k = r["Kernel_Name"][:40]
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in acc.items():
    if "pair_reg" in k:
        print(k, {c: f"{v:.3g}" for c, v in d.items()})
PY

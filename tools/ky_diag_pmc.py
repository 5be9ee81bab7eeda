"""Median per launch of every counter of k_spmm_lanczos<P> (not the start
pass) in rocprofv3 counter_collection.csv files; FETCH_SIZE / WRITE_SIZE are
KB (FETCH_SIZE doubled per the gfx950 calibration, MI355X_MICROARCH.md §HBM).
Usage: python tools/ky_diag_pmc.py OUT_JSON TAG CSV [CSV ...]"""
import collections
import csv
import json
import sys

out, tag, files = sys.argv[1], sys.argv[2], sys.argv[3:]
vals = collections.defaultdict(list)
for f in files:
    for r in csv.DictReader(open(f)):
        if "k_spmm_lanczos<" not in r["Kernel_Name"]:
            continue
        vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
res = {k: sorted(v)[len(v) // 2] for k, v in vals.items()}
if "FETCH_SIZE" in res:
    res["fetch_bytes_x2"] = 2.0 * 1024.0 * res["FETCH_SIZE"]
if "WRITE_SIZE" in res:
    res["write_bytes"] = 1024.0 * res["WRITE_SIZE"]
if "TCC_HIT_sum" in res and "TCC_MISS_sum" in res:
    res["l2_hit_rate"] = res["TCC_HIT_sum"] / (res["TCC_HIT_sum"] + res["TCC_MISS_sum"])
res["launches"] = {k: len(v) for k, v in vals.items()}
try:
    allres = json.load(open(out))
except (OSError, ValueError):
    allres = {}
allres.setdefault(tag, {}).update(res)
json.dump(allres, open(out, "w"), indent=1)
print(tag, json.dumps(res))

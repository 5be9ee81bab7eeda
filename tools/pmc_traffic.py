"""Summarise rocprofv3 counter passes into per-launch HBM traffic.

FETCH_SIZE and WRITE_SIZE come from SEPARATE --pmc passes (they do not fit
one TCC pass on gfx950).  Per /opt/skills/guides/MI355X_MICROARCH.md §HBM,
FETCH_SIZE reports half the bytes of wide (16 B/lane) coalesced reads on
gfx950, so it is doubled; WRITE_SIZE is exact for 16 B/lane stores.  The
doubling is checked on k_update, whose read bytes are known exactly (24nP).
Usage: python tools/pmc_traffic.py FETCH_CSV WRITE_CSV OUT_JSON [SECTION [HIT_CSV]]
(with SECTION the result is merged into OUT_JSON under that key, e.g. sf1m,
er100k, sf1m_weighted -- the bench workload bench.py looks it up by).
"""
import collections
import csv
import json
import re
import sys


def per_kernel(path, counter):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        m = re.search(r"kt::(k_\w+)<([^>]*)>", r["Kernel_Name"])
        key = f"{m.group(1)}<{m.group(2)}>" if m else r["Kernel_Name"][:60]
        agg[key].append(float(r["Counter_Value"]) * 1024.0)  # KB -> bytes
    return {k: sorted(v)[len(v) // 2] for k, v in agg.items()}  # median per launch


def per_kernel_raw(path, counter):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        m = re.search(r"kt::(k_\w+)<([^>]*)>", r["Kernel_Name"])
        key = f"{m.group(1)}<{m.group(2)}>" if m else r["Kernel_Name"][:60]
        agg[key].append(float(r["Counter_Value"]))
    return {k: sorted(v)[len(v) // 2] for k, v in agg.items()}


def main(fetch_csv, write_csv, out_json, section=None, hit_csv=None):
    f = per_kernel(fetch_csv, "FETCH_SIZE")
    w = per_kernel(write_csv, "WRITE_SIZE")
    hit = per_kernel_raw(hit_csv, "TCC_HIT_sum") if hit_csv else {}
    miss = per_kernel_raw(hit_csv, "TCC_MISS_sum") if hit_csv else {}
    res = {}
    for k in sorted(set(f) | set(w)):
        fb = 2.0 * f.get(k, 0.0)
        wb = w.get(k, 0.0)
        res[k] = {"fetch_bytes_x2": fb, "write_bytes": wb, "hbm_bytes_per_launch": fb + wb}
        if k in hit and hit[k] + miss.get(k, 0.0) > 0:
            res[k]["l2_hit_rate"] = hit[k] / (hit[k] + miss.get(k, 0.0))
    doc = ("median per launch; FETCH_SIZE doubled per the gfx950 calibration "
           "(MI355X_MICROARCH.md §HBM); Infinity-Cache hits are counted by these "
           "memory-side counters")
    import os
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from krylov_robustness_amd._lib import source_digest
    res["_build"] = {"csrc_sha256": source_digest(),
                     "note": "digest of the library sources these counters were measured on "
                             "(krylov_robustness_amd._lib.source_digest)"}
    if section:
        try:
            allr = json.load(open(out_json))
        except (OSError, ValueError):
            allr = {"_doc": doc}
        allr[section] = res
        json.dump(allr, open(out_json, "w"), indent=1)
    else:
        res["_doc"] = doc
        json.dump(res, open(out_json, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:6])

"""Per-term statistics of the expmv term kernels from a rocprofv3 kernel trace
(trace_exp with the expmv Afun, tools/expmv_c4.py):
  python tools/expmv_terms.py KERNEL_TRACE_CSV [OUT_JSON]
Launches of k_expmv_rows / k_expmv_step longer than 12 us are active terms
(a term past its stage's stop returns at once); prints count, mean and
median duration of each group per kernel."""
import collections
import csv
import json
import re
import sys


def gaps(path, top=12):
    """Idle time of the device between consecutive kernels (all kernels of
    the trace), the largest gaps with the kernels either side."""
    ks = []
    for r in csv.DictReader(open(path)):
        m = re.search(r"kt::(k_\w+)", r["Kernel_Name"])
        ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), m.group(1) if m else r["Kernel_Name"][:40]))
    ks.sort()
    g, end, prev = [], None, None
    for s0, e0, nm in ks:
        if end is not None and s0 > end:
            g.append(((s0 - end) / 1e3, prev, nm))
        if end is None or e0 > end:
            end, prev = e0, nm
    g.sort(reverse=True)
    span = (max(e for _, e, _ in ks) - min(s for s, _, _ in ks)) / 1e3 if ks else 0.0
    return {"span_us": round(span, 1), "idle_us": round(sum(x[0] for x in g), 1),
            "idle_over_50us": round(sum(x[0] for x in g if x[0] > 50), 1),
            "largest": [(round(a, 1), b, c) for a, b, c in g[:top]]}


def main(path, out=None):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        m = re.search(r"kt::(k_expmv_\w+)<([^>]*)>", r["Kernel_Name"])
        if not m:
            continue
        d[f"{m.group(1)}<{m.group(2)}>"].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    res = {}
    for k, v in d.items():
        act = sorted(x for x in v if x > 12.0)
        idle = sorted(x for x in v if x <= 12.0)
        res[k] = {"launches": len(v), "active": len(act),
                  "active_mean_us": round(sum(act) / len(act), 2) if act else None,
                  "active_median_us": round(act[len(act) // 2], 2) if act else None,
                  "active_total_ms": round(sum(act) / 1e3, 2),
                  "noop": len(idle), "noop_mean_us": round(sum(idle) / len(idle), 2) if idle else None}
    res["_gaps"] = gaps(path)
    print(json.dumps(res, indent=1))
    if out:
        json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:])

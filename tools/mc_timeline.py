"""Where one mc_trace (trace_exp, Lanczos-exp Afun) evaluation's wall time
goes, from a rocprofv3 kernel trace of `bench.py --estimator mc_trace
--steps K --no-profile` (the timed evaluations are the K evaluations after the
warm-up one).  Every evaluation launches the same sequence (same rounds), so
the trace splits into equal-count chunks; per evaluation: wall time to the
next one's first launch, the union of all
kernel intervals (GPU busy), per-kernel summed durations and unions, and the
idle gaps (nothing running for > 2 us) labelled by the kernel after them.
Medians over the timed evaluations.
Usage: python tools/mc_timeline.py KERNEL_TRACE_CSV TIMED_EVALS [OUT_JSON]"""
import csv
import json
import re
import statistics as st
import sys
from collections import defaultdict


def union(iv):
    tot, cs, ce = 0, None, None
    for a, b in sorted(iv):
        if ce is None or a > ce:
            if ce is not None:
                tot += ce - cs
            cs, ce = a, b
        else:
            ce = max(ce, b)
    return tot + ((ce - cs) if ce is not None else 0)


def short(name):
    m = re.search(r"kt::(k_\w+(?:<\d+)?)", name)
    return m.group(1) if m else name.split("(")[0][:40]


def main(path, evals, out=None):
    evals = int(evals)
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]))
                for r in csv.DictReader(open(path)))
    # the trace holds the warm-up evaluation and the timed ones, each with the
    # same launch sequence (same rounds): equal-count chunks
    total = evals + 1
    if len(ev) % total:
        raise SystemExit(f"{len(ev)} launches do not split into {total} equal evaluations")
    per_eval = len(ev) // total
    starts = [k * per_eval for k in range(total)] + [len(ev)]
    starts = starts[1:]
    res = []
    for k in range(len(starts) - 1):
        i0, i1 = starts[k], starts[k + 1]
        win = ev[i0:i1]
        t0 = ev[i0][0]
        t1 = ev[i1][0] if i1 < len(ev) else max(b for _, b, _ in win)
        per = defaultdict(lambda: [0, []])
        for a, b, nm in win:
            per[nm][0] += b - a
            per[nm][1].append((a, b))
        gaps, ce = defaultdict(float), None
        for a, b, nm in win:
            if ce is not None and a > ce + 2000:
                gaps[nm] += (a - ce) / 1e3
            ce = b if ce is None else max(ce, b)
        res.append({"wall_ms": (t1 - t0) / 1e6, "busy_ms": union([(a, b) for a, b, _ in win]) / 1e6,
                    "kernels": {nm: {"n": len(v[1]), "sum_ms": v[0] / 1e6, "union_ms": union(v[1]) / 1e6}
                                for nm, v in per.items()},
                    "idle_before_us": dict(gaps)})
    med = {"wall_ms": st.median(r["wall_ms"] for r in res), "busy_ms": st.median(r["busy_ms"] for r in res)}
    names = set().union(*(r["kernels"] for r in res))
    med["kernels"] = {nm: {k: st.median(r["kernels"].get(nm, {k: 0})[k] for r in res) for k in ("n", "sum_ms", "union_ms")}
                      for nm in sorted(names, key=lambda x: -res[0]["kernels"].get(x, {"sum_ms": 0})["sum_ms"])}
    gnames = set().union(*(r["idle_before_us"] for r in res))
    med["idle_before_us"] = {nm: st.median(r["idle_before_us"].get(nm, 0.0) for r in res)
                             for nm in sorted(gnames, key=lambda x: -res[0]["idle_before_us"].get(x, 0.0))}
    out_d = {"evaluations": len(res), "median": med}
    print(json.dumps({"wall_ms": med["wall_ms"], "busy_ms": med["busy_ms"],
                      "top": list(med["kernels"].items())[:8],
                      "idle_top": list(med["idle_before_us"].items())[:8]}, indent=1))
    if out:
        with open(out, "w") as f:
            json.dump(out_d, f, indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:])

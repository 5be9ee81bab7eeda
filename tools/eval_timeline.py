"""Where one Hutchinson evaluation's wall time goes, from a rocprofv3 kernel
trace of `bench.py` (timed region only).  An evaluation starts at its first
k_spmm_lanczos_start launch (one per probe sweep); its wall time runs to the
next evaluation's first start launch.  Per evaluation: the union of all
kernel intervals (GPU busy), per-kernel summed durations and unions, the
idle gap before the next evaluation (host quadrature + the next call's
launch latency) and idle gaps inside it.  Medians over evaluations.
Usage: python tools/eval_timeline.py KERNEL_TRACE_CSV SWEEPS_PER_EVAL TIMED_EVALS [OUT_JSON]"""
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
    m = re.search(r"kt::(k_\w+)", name)
    return m.group(1) if m else name.split("(")[0][:40]


def main(path, sweeps, evals, out=None):
    sweeps, evals = int(sweeps), int(evals)
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]))
                for r in csv.DictReader(open(path)))
    starts = [i for i, e in enumerate(ev) if e[2] == "k_spmm_lanczos_start"]
    # the isolated roofline pass (4 sweeps) follows the timed region; the timed
    # region's evaluations are the `evals` groups of `sweeps` start launches before it
    first = starts[len(starts) - 4 - sweeps * evals::sweeps][:evals + 1]
    res = []
    for k in range(evals):
        i0 = first[k]
        i1 = first[k + 1] if k + 1 < len(first) else None
        t0 = ev[i0][0]
        t1 = ev[i1][0] if i1 is not None else None
        if t1 is None:
            break
        win = [e for e in ev[i0:i1]]
        busy = union([(a, b) for a, b, _ in win])
        last_end = max(b for _, b, _ in win)
        per = defaultdict(lambda: [0, []])
        for a, b, nm in win:
            per[nm][0] += b - a
            per[nm][1].append((a, b))
        # idle gaps (> 2 us with nothing running), each labelled by the kernel after it
        gaps, ce = [], None
        for a, b, nm in sorted(win):
            if ce is not None and a > ce + 2000:
                gaps.append((a - ce, nm))
            ce = b if ce is None else max(ce, b)
        gaps.sort(reverse=True)
        inner = sum(g for g, _ in gaps)
        host = gaps[0][0] if gaps and gaps[0][1] == "k_rademacher_signs" else 0  # the call turnaround
        small = defaultdict(lambda: [0, 0])
        for g, nm in gaps:
            if not (host and (g, nm) == gaps[0]):
                small[nm][0] += g
                small[nm][1] += 1
        res.append({"wall": t1 - t0, "busy": busy, "tail_gap": t1 - last_end, "inner_gaps": inner,
                    "host_turnaround": host, "other_gaps": {k: v for k, v in small.items()},
                    "kernels": {nm: {"sum": v[0], "union": union(v[1]), "launches": len(v[1])}
                                for nm, v in per.items()}})
    med = lambda xs: st.median(xs) / 1e3  # us
    names = sorted({nm for r in res for nm in r["kernels"]})
    summ = {"evals": len(res), "wall_us": med([r["wall"] for r in res]),
            "gpu_busy_us": med([r["busy"] for r in res]),
            "tail_gap_us": med([r["tail_gap"] for r in res]),
            "inner_gaps_us": med([r["inner_gaps"] for r in res]),
            "host_turnaround_us": med([r["host_turnaround"] for r in res]),
            "host_turnaround_basis": "the idle gap before the next call's first kernel (k_rademacher_signs): "
                                     "sync, host quadrature, the reduction, the next call's set-up",
            "other_gaps_by_next_kernel": {nm: {"sum_us": med([r["other_gaps"].get(nm, [0, 0])[0] for r in res]),
                                               "count": st.median([r["other_gaps"].get(nm, [0, 0])[1] for r in res])}
                                          for nm in sorted({k for r in res for k in r["other_gaps"]})},
            "kernels": {nm: {"sum_us": med([r["kernels"].get(nm, {"sum": 0})["sum"] for r in res]),
                             "union_us": med([r["kernels"].get(nm, {"union": 0})["union"] for r in res]),
                             "launches": st.median([r["kernels"].get(nm, {"launches": 0})["launches"] for r in res])}
                        for nm in names}}
    summ["busy_frac"] = summ["gpu_busy_us"] / summ["wall_us"]
    print(json.dumps(summ, indent=1))
    if out:
        json.dump(summ, open(out, "w"), indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:5])

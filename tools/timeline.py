"""Occupancy timeline of the timed region from a rocprofv3 kernel trace:
how much of the wall time has 0 / 1 / 2+ dominant-kernel launches in
flight, and what else runs.  Usage:
python tools/timeline.py KERNEL_TRACE_CSV KERNEL_SUBSTR TIMED_LAUNCHES ISO_LAUNCHES"""
import csv
import sys
from collections import defaultdict


def main(path, ksub, timed, iso):
    timed, iso = int(timed), int(iso)
    rows = list(csv.DictReader(open(path)))
    ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
    ev.sort()
    dom = [e for e in ev if ksub in e[2] and "_start" not in e[2]]
    sel = dom[len(dom) - iso - timed:len(dom) - iso]
    t0, t1 = sel[0][0], max(e[1] for e in sel)
    win = [e for e in ev if e[1] > t0 and e[0] < t1]
    # sweep-line occupancy of the dominant kernel and of anything
    pts = []
    for s, e, k in win:
        s, e = max(s, t0), min(e, t1)
        d = 1 if (ksub in k and "_start" not in k) else 0
        pts.append((s, 1, d))
        pts.append((e, -1, -d))
    pts.sort()
    occ = defaultdict(int)   # dominant launches in flight -> ns
    busy_any = 0
    n_any = n_dom = 0
    last = t0
    for t, da, dd in pts:
        if t > last:
            occ[n_dom] += t - last
            if n_any > 0:
                busy_any += t - last
            last = t
        n_any += da
        n_dom += dd
    wall = t1 - t0
    per = defaultdict(lambda: [0, 0])
    for s, e, k in win:
        name = k.split("(")[0].replace("void ", "")
        per[name][0] += 1
        per[name][1] += min(e, t1) - max(s, t0)
    print(f"window {wall / 1e6:.2f} ms, {len(sel)} dominant launches")
    for k in sorted(occ):
        print(f"  {k} dominant in flight: {occ[k] / wall * 100:6.2f} %  ({occ[k] / 1e6:.2f} ms)")
    print(f"  any kernel busy: {busy_any / wall * 100:.2f} %")
    for name, (c, ns) in sorted(per.items(), key=lambda x: -x[1][1]):
        print(f"  {name:70s} {c:7d} launches {ns / 1e6:9.2f} ms  avg {ns / c / 1e3:8.2f} us")


if __name__ == "__main__":
    main(*sys.argv[1:5])

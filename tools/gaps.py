"""Kernel-trace gap analysis of the LAST `window` of a run: wall span, kernel
busy time (union), launches, and host gaps (> 4 us with no kernel running)
binned by the kernel that follows them.
Usage: python tools/gaps.py KERNEL_TRACE_CSV START_KERNEL_SUBSTR [OCCURRENCE]
The window starts at the OCCURRENCE-th (default: last; "half": the middle
one, i.e. the second of two identical calls) launch whose name contains
START_KERNEL_SUBSTR."""
import csv
import sys
from collections import defaultdict


def main(path, start_sub, occ=None):
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                for r in csv.DictReader(open(path)))
    idx = [i for i, e in enumerate(ev) if start_sub in e[2]]
    i0 = idx[len(idx) // 2] if occ == "half" else (idx[int(occ)] if occ is not None else idx[-1])
    win = ev[i0:]
    t0, t1 = win[0][0], max(e[1] for e in win)
    busy, last_end, gaps = 0, t0, defaultdict(lambda: [0, 0])
    cur_s, cur_e = win[0][0], win[0][1]
    for s, e, k in win[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            g = s - cur_e
            if g > 4000:
                name = k.split("(")[0].replace("void ", "")[:60]
                gaps[name][0] += 1
                gaps[name][1] += g
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    wall = t1 - t0
    print(f"window {wall / 1e6:.2f} ms, {len(win)} launches, kernels busy {busy / 1e6:.2f} ms "
          f"({busy / wall * 100:.1f} %), idle {(wall - busy) / 1e6:.2f} ms")
    tot = sum(v[1] for v in gaps.values())
    print(f"gaps > 4 us: {sum(v[0] for v in gaps.values())} totalling {tot / 1e6:.2f} ms, by the kernel after them:")
    for k, (c, g) in sorted(gaps.items(), key=lambda x: -x[1][1])[:12]:
        print(f"  {k:60s} {c:6d} gaps {g / 1e6:8.2f} ms")
    per = defaultdict(lambda: [0, 0])
    for s, e, k in win:
        name = k.split("(")[0].replace("void ", "")[:60]
        per[name][0] += 1
        per[name][1] += e - s
    print("kernels:")
    for k, (c, d) in sorted(per.items(), key=lambda x: -x[1][1])[:12]:
        print(f"  {k:60s} {c:6d} x {d / c / 1e3:8.2f} us = {d / 1e6:8.2f} ms")


if __name__ == "__main__":
    main(*sys.argv[1:4])

"""Print the kernel sequence of one block-Krylov step on one stream from a
rocprofv3 kernel trace: python tools/step_timeline.py TRACE.csv [call] [step]
(steps = spans between consecutive k_spmm_block launches of a thread)."""
import csv
import sys
from collections import defaultdict

path = sys.argv[1]
call = int(sys.argv[2]) if len(sys.argv) > 2 else -1
stepno = int(sys.argv[3]) if len(sys.argv) > 3 else 4
rows = list(csv.DictReader(open(path)))
by_thr = defaultdict(list)
for r in rows:
    by_thr[r["Thread_Id"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ", "")[:48], r["Stream_Id"]))
for thr, ev in by_thr.items():
    ev.sort()
    sp = [i for i, e in enumerate(ev) if "k_spmm_block" in e[2]]
    if len(sp) < 10:
        continue
    # calls: spmm launches separated by > 2 ms gaps
    calls = [[sp[0]]]
    for a, b in zip(sp, sp[1:]):
        if ev[b][0] - ev[a][0] > 3_000_000:
            calls.append([])
        calls[-1].append(b)
    c = calls[call]
    if stepno + 1 >= len(c):
        continue
    i0, i1 = c[stepno], c[stepno + 1]
    t0 = ev[i0][0]
    print(f"thread {thr}: step {stepno} of call {call}, {len(c)} spmm in call, span {(ev[i1][0] - t0) / 1e3:.1f} us")
    busy = 0
    prev_end = t0
    agg = defaultdict(lambda: [0, 0.0])
    for s, e, k, st in ev[i0:i1]:
        gap = (s - prev_end) / 1e3
        busy += e - s
        agg[k][0] += 1
        agg[k][1] += (e - s) / 1e3
        if len(sys.argv) > 4:
            print(f"  +{(s - t0) / 1e3:8.1f} gap {gap:6.1f} {k:48s} {(e - s) / 1e3:6.1f} us")
        prev_end = max(prev_end, e)
    print(f"  kernels busy {busy / 1e3:.1f} us")
    for k, (n, t) in sorted(agg.items(), key=lambda x: -x[1][1]):
        print(f"    {k:48s} {n:4d} x = {t:7.1f} us")

"""Mean per-Lanczos-step phase clocks (us) of workgroup 0 from the reg_prof
lines of -DKT_FUSED_PROF k_pair_reg builds (tools/pair_prof.py output).
Usage: python tools/pair_phases.py LOG [LOG ...]"""
import collections
import json
import re
import sys

for path in sys.argv[1:]:
    rows = [ln for ln in open(path) if ln.startswith("reg_prof")]
    tot, steps = collections.Counter(), 0
    for ln in rows[1:]:  # the first launch warms up
        d = dict(re.findall(r"(\w+)=([\d.]+)", ln))
        for k in ("start", "spmm", "A", "B", "C", "D", "E", "eig", "stop"):
            tot[k] += float(d[k])
        steps += int(d["iter"])
    us = {k: round(v / steps / 100.0, 2) for k, v in tot.items()}  # wall clock: 100 MHz
    print(json.dumps({"log": path, "launches": len(rows) - 1, "steps_per_launch": steps / max(1, len(rows) - 1),
                      "us_per_step": us, "total_us_per_step": round(sum(us.values()), 2)}))

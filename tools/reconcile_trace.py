"""Split a rocprofv3 kernel trace of the default bench command into the timed
region and the isolated single-lane roofline pass, for the dominant kernel,
and compare each with the bench line it produced.
Usage: python tools/reconcile_trace.py KERNEL_TRACE_CSV BENCH_JSON OUT_JSON"""
import csv
import json
import sys


def _union(iv):
    tot, cs, ce = 0, None, None
    for a, e in sorted(iv):
        if ce is None or a > ce:
            if ce is not None:
                tot += ce - cs
            cs, ce = a, e
        else:
            ce = max(ce, e)
    return tot + ((ce - cs) if ce is not None else 0)


def main(trace_csv, bench_json, out_json):
    b = json.loads(open(bench_json).read().strip().splitlines()[-1])
    roof = b["roofline"]
    kname = roof["kernel"].rstrip(">")  # e.g. k_spmm_lanczos<16
    allrows = list(csv.DictReader(open(trace_csv)))
    # the headline's launches end where the mc_trace leg starts: its first
    # explicit K1 (k_spmm_dot) launch (the leg's y-form sweeps launch the
    # headline kernel too)
    k1 = [int(r["Start_Timestamp"]) for r in allrows if "kt::k_spmm_dot<" in r["Kernel_Name"]]
    cut = min(k1) if k1 else None
    rows = [r for r in allrows if f"kt::{kname}," in r["Kernel_Name"]
            and (cut is None or int(r["Start_Timestamp"]) < cut)]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]  # us
    iso = (roof.get("isolated_pass") or {}).get("launches", roof["launches"])
    timed = b["steps"] * (b["config"]["probes_per_eval"] // b["config"]["probes_per_sweep"]) * \
        (b["config"]["lanczos_m"] - 1)
    t_iso, t_timed = dur[-iso:], dur[-iso - timed:-iso]
    # union of the timed region's launch intervals (lane overlap counted once)
    union = _union([(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows[-iso - timed:-iso]])
    out = {
        "command": "rocprofv3 --kernel-trace --stats -- python3 bench.py (default command)",
        "kernel": kname,
        "bench_value": b["value"],
        "launches_total": len(dur),
        "isolated_pass": {"launches": len(t_iso), "rocprof_avg_us": round(sum(t_iso) / len(t_iso), 2),
                          "bench_avg_launch_us": (roof.get("isolated_pass") or {}).get(
                              "avg_launch_us", roof["avg_launch_us"])},
        "timed_region": {"launches": len(t_timed),
                         "rocprof_union_busy_ms": round(union / 1e6, 3),
                         "bench_timed_region_busy_ms": roof.get("timed_region_busy_ms"),
                         "rocprof_union_us_per_launch": round(union / 1e3 / len(t_timed), 2),
                         "bench_avg_launch_us": roof["avg_launch_us"],
                         "rocprof_avg_us": round(sum(t_timed) / len(t_timed), 2),
                         "bench_timed_region_avg_launch_us_overlapped":
                             roof["timed_region_avg_launch_us_overlapped"],
                         "note": f"{b['config']['sweep_lanes']} sweep lanes in flight: launches "
                                 "share the chip"},
        "_doc": "rocprofv3 kernel trace of the default bench command split into the timed region "
                "(the steps x sweeps x (m-1) launches before the isolated pass) and the isolated "
                "single-lane roofline pass (the last `launches` launches before the mc_trace leg's "
                "first k_spmm_dot launch)",
    }
    mc = (b.get("mc_trace") or {}).get("roofline")
    if mc:
        # the mc_trace leg's serial roofline pass: the dominant kernel's
        # launches (every width it ran at) are the last `launches` launches of
        # that kernel in the run (the reference-composition leg after it runs
        # expmv kernels only)
        base = mc["kernel"].split("<")[0]
        widths = list(mc.get("launches_by_width", {}))
        allk = [r for r in allrows if any(f"kt::{base}<{P}," in r["Kernel_Name"] for P in widths)]
        allk.sort(key=lambda r: int(r["Start_Timestamp"]))
        last = allk[-mc["launches"]:]
        d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in last]
        out["mc_trace_serial_pass"] = {"kernel": mc["kernel"], "launches": len(d),
                                       "rocprof_avg_us": round(sum(d) / len(d), 2),
                                       "rocprof_union_us_per_launch": round(
                                           _union([(int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
                                                   for r in last]) / 1e3 / len(d), 2),
                                       "bench_avg_launch_us": mc["avg_launch_us"],
                                       "bench_avg_launch_us_overlapped": mc.get("avg_launch_us_overlapped")}
    json.dump(out, open(out_json, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])

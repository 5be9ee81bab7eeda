"""One expmv call's Taylor-term chain on dt_oregon A6 (config 1), alone on the
device: run under rocprofv3 --kernel-trace, then `python tools/expmv_chain.py
--analyse TRACE.csv` prints the per-launch durations of k_expmv_step and the
idle gaps between consecutive launches (the dependent-launch interval)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def run():
    import numpy as np
    import torch  # noqa: F401
    import krylov_robustness_amd as kra
    from conftest import load_graph
    A = load_graph("oregon_A6")
    ctx = kra.Context(0)
    D = kra.DeviceMatrix(A, ctx)
    B = np.sign(np.random.default_rng(0).standard_normal((A.shape[0], 10)))
    for r in range(6):
        t0 = time.perf_counter()
        F, s, m, mv = kra.expmv(1.0, D, B, ctx=ctx)
        dt = time.perf_counter() - t0
    print(json.dumps({"s": s, "m": m, "mv": mv, "ms": dt * 1e3, "us_per_mv": dt * 1e6 / mv}))


def analyse(path):
    import csv
    import gzip
    import statistics as st
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                for r in csv.DictReader(gzip.open(path, "rt") if path.endswith(".gz") else open(path)))
    k = [e for e in ev if "k_expmv_step" in e[2]]
    k = k[len(k) // 2:]  # the later calls (warm)
    dur = [(b - a) / 1e3 for a, b, _ in k]
    gaps = [(k[i + 1][0] - k[i][1]) / 1e3 for i in range(len(k) - 1)]
    gaps = [g for g in gaps if g < 50]  # within a stage
    print(json.dumps({"launches": len(k), "dur_us_median": st.median(dur), "dur_us_p10": sorted(dur)[len(dur) // 10],
                      "dur_us_p90": sorted(dur)[9 * len(dur) // 10], "gap_us_median": st.median(gaps),
                      "period_us_median": st.median(dur) + st.median(gaps)}))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--analyse":
        analyse(sys.argv[2])
    else:
        run()

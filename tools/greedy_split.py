"""Config-5 step anatomy (GPU): iteration counts of the first greedy step's
Q = 250 candidates at the real tolerance, and the per-step cost of the fused
candidate kernel at fixed step counts (tol = 1e-300), for the library in
KT_LIB (e.g. a KT_FUSED_NOEIG build = vector work only).  One JSON line each."""
import json
import os
import sys
import time

import torch  # noqa: F401
import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import krylov_robustness_amd as kra  # noqa: E402
from conftest import load_graph  # noqa: E402


def timed(f, rep=5):
    f()
    ts = []
    for _ in range(rep):
        t0 = time.perf_counter()
        r = f()
        ts.append(time.perf_counter() - t0)
    return min(ts) * 1e3, r


A = load_graph("india")
c = kra.compute_centrality(A)
ctx = kra.Context(0)
D = kra.DeviceMatrix(A, ctx)
tol = kra.default_greedy_tol(D, ctx=ctx)
B = -np.array([[0.0, 1.0], [1.0, 0.0]])
E = kra.find_top_edges(A, c, 250, "min")
lib = os.environ.get("KT_LIB", "default")
if "noeig" not in lib:
    ms, (xm, its, _) = timed(lambda: kra.trace_fun_update_pairs(D, E, B, tol, 100, ctx=ctx))
    h = np.bincount(its.astype(int))
    print(json.dumps({"lib": lib, "tol": tol, "ms": ms, "iters_max": int(its.max()), "iters_mean": float(its.mean()),
                      "iters_hist": {int(k): int(v) for k, v in enumerate(h) if v}}))
for it in (5, 10, 20, 40):
    ms, _ = timed(lambda: kra.trace_fun_update_pairs(D, E, B, 1e-300, it, ctx=ctx))
    print(json.dumps({"lib": lib, "q": 250, "it": it, "ms": ms, "us_per_step": 1e3 * ms / it}))

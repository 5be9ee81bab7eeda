"""Split one greedy step of config 5 into its parts (device pairs evaluation,
edge edit) and time the pairs evaluation under different candidate counts."""
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

A = load_graph(sys.argv[1] if len(sys.argv) > 1 else "india")
c = kra.compute_centrality(A)
ctx = kra.Context(0)
D = kra.DeviceMatrix(A, ctx)
tol = kra.default_greedy_tol(D, ctx=ctx)
B = -np.array([[0.0, 1.0], [1.0, 0.0]])
res = {}
for q in (1, 16, 64, 250):
    E = kra.find_top_edges(A, c, q, "min")
    kra.trace_fun_update_pairs(D, E, B, tol, 100, ctx=ctx)
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        xm, it, lk = kra.trace_fun_update_pairs(D, E, B, tol, 100, ctx=ctx)
        ts.append(time.perf_counter() - t0)
    res[f"pairs_q{q}_ms"] = 1e3 * min(ts)
    res[f"pairs_q{q}_maxiter"] = int(it.max())
E = kra.find_top_edges(A, c, 4, "min")
ts = []
for h in range(4):
    t0 = time.perf_counter()
    D.set_pairs(E[h:h + 1], 0.0)
    ts.append(time.perf_counter() - t0)
res["set_pairs_ms"] = 1e3 * min(ts)
print(json.dumps(res))

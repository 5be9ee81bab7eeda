import os, sys, time, json
import torch  # noqa
import numpy as np
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/tests")
import krylov_robustness_amd as kra
from conftest import load_graph
A = load_graph("india"); c = kra.compute_centrality(A); ctx = kra.Context(0); D = kra.DeviceMatrix(A, ctx)
B = -np.array([[0.0, 1.0], [1.0, 0.0]])
for q in (1, 250):
    E = kra.find_top_edges(A, c, q, "min")
    for it in (10, 28, 100):
        kra.trace_fun_update_pairs(D, E, B, 1e-300, it, ctx=ctx)
        t0 = time.perf_counter(); xm, its, _ = kra.trace_fun_update_pairs(D, E, B, 1e-300, it, ctx=ctx); t = time.perf_counter() - t0
        print(json.dumps({"lib": os.environ.get("KT_LIB", "default"), "q": q, "it": it, "ms": 1e3 * t, "maxiter": int(its.max())}))

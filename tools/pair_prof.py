"""One k_pair_reg launch per call on config 5's first greedy step (India, the
250 top-ranked candidate edges, break mode, the drivers' tolerance, it = 100),
repeated: with a -DKT_FUSED_PROF build (KT_LIB) every launch prints workgroup
0's per-phase device clocks (reg_prof lines).  Diagnostic builds' scores are
wrong by construction; only their clocks mean anything.
Usage: KT_LIB=... python tools/pair_prof.py [reps]"""
import os
import sys
import time

import torch  # noqa: F401  (torch's HIP runtime first)
import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import krylov_robustness_amd as kra  # noqa: E402
from conftest import load_graph  # noqa: E402

BREAK = -np.array([[0.0, 1.0], [1.0, 0.0]])
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
A = load_graph("india")
ctx = kra.Context(0)
D = kra.DeviceMatrix(A, ctx)
c = kra.compute_centrality(A)
E = kra.find_top_edges(A, c, 250, "min")
tol = kra.default_greedy_tol(D, ctx=ctx)
ts = []
for _ in range(reps):
    t0 = time.perf_counter()
    x, it, lk = kra.trace_fun_update_pairs(D, E, BREAK, tol, 100, ctx=ctx)
    ts.append(time.perf_counter() - t0)
    sys.stdout.flush()
print({"ms_min": 1e3 * min(ts), "iters_max": int(np.max(it)), "iters_mean": float(np.mean(it))})

"""Run config 3's fun_and_grad_krylov_fun stage a few times (for rocprofv3)."""
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

A = load_graph(sys.argv[1] if len(sys.argv) > 1 else "hawaii")
ctx = kra.Context(0)
D = kra.DeviceMatrix(A, ctx)
nrm = kra.normest(D, 1e-2, ctx=ctx)
c = kra.compute_centrality(A)
E = kra.find_top_edges(A, c, 100, "min")
temp, _ = kra.function_multiple_entries(D, E, "cosh", 1e-6 * np.cosh(nrm), 100, ctx=ctx)
ind = np.argsort(-temp, kind="stable")[:30]
Om, dfA = E[ind], temp[ind]
X = np.random.default_rng(11).uniform(-0.5, 1.0, size=30)
if X.sum() > 10:
    X *= 10 / X.sum()
U_cols = len(np.unique(Om))
for r in range(int(os.environ.get("KT_FG_REPS", "4"))):
    t0 = time.perf_counter()
    f, gr = kra.fun_and_grad_krylov_fun(X, D, Om, "sinh", "cosh", dfA, 1e-6 * np.sinh(nrm), 100, ctx=ctx)
    print(f"fg {time.perf_counter() - t0:.4f} s  f={f:.6f} distinct nodes {U_cols}", flush=True)

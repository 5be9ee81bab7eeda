"""fun_and_grad_krylov_exp (or, with --hess, hessianfcn_exp) on voltage India
as tests/perf/bench_hessian.py sets it up, repeated (for rocprofv3 / KT_EIG_STATS
timing)."""
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

hess = "--hess" in sys.argv
args = [a for a in sys.argv[1:] if not a.startswith("--")]
A = load_graph(args[0] if args else "india")
ctx = kra.Context(0)
D = kra.DeviceMatrix(A, ctx)
tol = 1e-8 * np.exp(kra.normest(D, 1e-2, ctx=ctx))
c = kra.compute_centrality(A)
E = kra.find_top_edges(A, c, 100, "min")
temp, _ = kra.function_multiple_entries(D, E, "exp", tol, 100, ctx=ctx)
ind = np.argsort(-temp, kind="stable")[:30]
Om, eA = E[ind], temp[ind]
w = np.asarray(A[Om[:, 0] - 1, Om[:, 1] - 1]).ravel()
X = np.random.default_rng(5).uniform(-0.5, 1.0, size=30) * w
if X.sum() > 10:
    X *= 10 / X.sum()
for r in range(4):
    t0 = time.perf_counter()
    if hess:
        H = kra.hessianfcn_exp(X, D, Om, tol, 100, ctx=ctx)
        print(f"hessianfcn_exp {time.perf_counter() - t0:.4f} s |H|={np.abs(H).sum():.10e}", flush=True)
    else:
        f, gr = kra.fun_and_grad_krylov_exp(X, D, Om, eA, tol, 100, ctx=ctx)
        print(f"fg_exp {time.perf_counter() - t0:.4f} s f={f:.10e}", flush=True)

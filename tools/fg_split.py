import os, sys, time
import torch  # noqa
import numpy as np
ROOT = "/root/repo"
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import krylov_robustness_amd as kra
from conftest import load_graph
A = load_graph("hawaii")
ctx = kra.Context(0)
D = kra.DeviceMatrix(A, ctx)
nrm = kra.normest(D, 1e-2, ctx=ctx)
c = kra.compute_centrality(A)
E = kra.find_top_edges(A, c, 100, "min")
temp, _ = kra.function_multiple_entries(D, E, "cosh", 1e-6 * np.cosh(nrm), 100, ctx=ctx)
ind = np.argsort(-temp, kind="stable")[:30]
Om, dfA = E[ind], temp[ind]
X = np.random.default_rng(11).uniform(-0.5, 1.0, size=30)
if X.sum() > 10: X *= 10 / X.sum()
tol = 1e-6 * np.sinh(nrm)
# U, B as fun_and_grad_krylov_fun builds them
nodes = np.unique(Om)
n = A.shape[0]
U = np.zeros((n, len(nodes)))
for t, v in enumerate(nodes): U[v - 1, t] = 1.0
B = np.zeros((len(nodes), len(nodes)))
pos = {v: t for t, v in enumerate(nodes)}
for (i, j), x in zip(Om, X):
    B[pos[i], pos[j]] += x; B[pos[j], pos[i]] += x
def best(f, r=4):
    ts = []
    for _ in range(r):
        t0 = time.perf_counter(); out = f(); ts.append(time.perf_counter() - t0)
    return min(ts), out
for twin in ("1", "0"):
    os.environ["KT_TWIN"] = twin
    t, _ = best(lambda: kra.fun_and_grad_krylov_fun(X, D, Om, "sinh", "cosh", dfA, tol, 100, ctx=ctx))
    print(f"fg KT_TWIN={twin}: {t*1e3:.2f} ms")
t, r = best(lambda: kra.trace_fun_update(D, U, B, tol, 100, 0, "sinh", ctx=ctx))
print(f"trace_fun_update(sinh) {t*1e3:.2f} ms iter {r[1]}")
t, r = best(lambda: kra.fun_update(D, U, B, "cosh", tol, 100, 0, ctx=ctx))
print(f"fun_update(cosh) {t*1e3:.2f} ms iter {r[1]}")

"""Config-3 objective diagnosis (GPU box): trace_fun_update(sinh) device vs
oracle per iteration cap, and the exact dense value by torch eigvalsh on the
GPU.  Test infrastructure: imports the oracle."""
import os, sys, json
import torch  # noqa
import numpy as np
ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import krylov_robustness_amd as kra
from conftest import load_graph
from oracle import krylov_oracle as ko
A = load_graph("hawaii"); n = A.shape[0]
ctx = kra.Context(0); D = kra.DeviceMatrix(A, ctx, check_symmetric=True)
nrm_d = kra.normest(D, 1e-2, ctx=ctx); nrm_o = ko.normest(A, 1e-2)
c = kra.compute_centrality(A); E = kra.find_top_edges(A, c, 100, "min")
tol_df = 1e-6 * np.cosh(nrm_d)
temp, fit = kra.function_multiple_entries(D, E, "cosh", tol_df, 100, ctx=ctx)
ind = np.argsort(-temp, kind="stable")[:30]; Om = E[ind]
rng = np.random.default_rng(11)
w = np.array([A[i - 1, j - 1] for i, j in Om]); X = rng.uniform(-0.5, 1.0, size=30) * w
if X.sum() > 10: X *= 10 / X.sum()
tol = 1e-6 * np.sinh(nrm_d)
U, B = ko.lowrank_from_edges(X, Om, n)
print("normest dev", nrm_d, "oracle", nrm_o, "rk", U.shape[1])
t_eff = tol * np.sinh(nrm_o)
Xd, itd, lkd = kra.trace_fun_update(D, U, B, t_eff, 100, 0, "sinh", ctx=ctx)
Xo, ito, lko = ko.trace_fun_update(A, U, B, t_eff, 100, 0, "sinh")
print("trace_fun_update dev", Xd, itd, lkd, "oracle", Xo, ito, lko, "rel", abs(Xd-Xo)/abs(Xo))
for itmax in range(2, 12):
    Xd, itd, _ = kra.trace_fun_update(D, U, B, 0.0, itmax, 0, "sinh", ctx=ctx)
    Xo, ito, _ = ko.trace_fun_update(A, U, B, 0.0, itmax, 0, "sinh")
    print(f"it={itmax:3d} dev {Xd:.15e} oracle {Xo:.15e} rel {abs(Xd-Xo)/abs(Xo):.2e}")
# exact: sum sinh(eig(A + U B U')) - sum sinh(eig(A)), dense fp64 eigvalsh on the GPU
import scipy.sparse as sp
Ad = torch.tensor(A.toarray(), dtype=torch.float64, device="cuda")
e1 = torch.linalg.eigvalsh(Ad)
Ut = torch.tensor(U, dtype=torch.float64, device="cuda"); Bt = torch.tensor(B, dtype=torch.float64, device="cuda")
At = Ad + Ut @ Bt @ Ut.T
At = (At + At.T) / 2
e2 = torch.linalg.eigvalsh(At)
exact = float((torch.sinh(e2) - torch.sinh(e1)).sum())
print("exact", repr(exact), "dev rel", abs(Xd - exact) / abs(exact), "oracle rel", abs(Xo - exact) / abs(exact))

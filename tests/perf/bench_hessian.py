"""The weighted Hessian drivers' evaluation (Tests/test_weighted_exp_hessian.m:
24-60 with fmincon's HessianFcn): voltage India (A / max(A), n = 3,228),
Omega = the 30 of find_top_edges(A, c, 100, 'min') with the largest
function_multiple_entries(A, E, @exp) (n >= ndense = 500), tol = 1e-8 *
exp(normest(A, 1e-2)), it = 100, at a seeded nonzero X.  Times one device
[f, gr] (fun_and_grad_krylov_exp) and one Hessian (hessianfcn_exp) and the
numpy oracle on the same inputs; one JSON line."""
import json
import os
import sys
import time

import torch  # noqa: F401  (torch's ROCm runtime first)
import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import krylov_robustness_amd as kra  # noqa: E402
from conftest import load_graph  # noqa: E402
from oracle import krylov_oracle as ko  # noqa: E402


def best(fn, rep=3):
    out, t = None, []
    for _ in range(rep):
        t0 = time.perf_counter()
        out = fn()
        t.append(time.perf_counter() - t0)
    return out, min(t)


def main():
    A = load_graph(sys.argv[1] if len(sys.argv) > 1 else "india")
    ctx = kra.Context(0)
    D = kra.DeviceMatrix(A, ctx)
    nrm = np.exp(kra.normest(D, 1e-2, ctx=ctx))
    tol = 1e-8 * nrm
    c = kra.compute_centrality(A)
    E = kra.find_top_edges(A, c, 100, "min")
    temp, _ = kra.function_multiple_entries(D, E, "exp", tol, 100, ctx=ctx)
    ind = np.argsort(-temp, kind="stable")[:30]
    Om, eA = E[ind], temp[ind]
    w = np.asarray(A[Om[:, 0] - 1, Om[:, 1] - 1]).ravel()
    X = np.random.default_rng(5).uniform(-0.5, 1.0, size=30) * w
    if X.sum() > 10:
        X *= 10 / X.sum()
    (f, gr), t_fg = best(lambda: kra.fun_and_grad_krylov_exp(X, D, Om, eA, tol, 100, ctx=ctx))
    H, t_h = best(lambda: kra.hessianfcn_exp(X, D, Om, tol, 100, ctx=ctx))
    t0 = time.perf_counter()
    fo, gro = ko.fun_and_grad_krylov_exp(X, A, Om, eA, tol, 100)
    t_fg_o = time.perf_counter() - t0
    t0 = time.perf_counter()
    Ho = ko.hessianfcn(X, A, Om, "exp", tol, 100)
    t_h_o = time.perf_counter() - t0
    out = {"workload": "weighted hessian India |Omega|=30 exp", "n": int(A.shape[0]), "nnz": int(A.nnz),
           "tol": tol, "fg_s": t_fg, "hessian_s": t_h, "oracle_fg_s": t_fg_o, "oracle_hessian_s": t_h_o,
           "fg_f_rel_diff": abs(f - fo) / abs(fo),
           "fg_gr_rel_diff": float(np.abs(gr - gro).max() / np.abs(gro).max()),
           "hessian_rel_diff": float(np.abs(H - Ho).max() / np.abs(Ho).max()),
           "hessian_symmetric": bool(np.allclose(H, H.T, rtol=0, atol=1e-12 * np.abs(H).max()))}
    print(json.dumps(out))


if __name__ == "__main__":
    main()

"""Golden fixtures for BASELINE configs 3 and 5 at full size (build container
only; the GPU tests read the JSON this writes, never this script's inputs).

  --config3  Transport Hawaii LCC (hawaii.npz), the pipeline of
             Tests/test_weighted_sinh_lbfgs.m:50-86 and :208:
               * normest(A, 1e-2)                             (fun_and_grad_krylov_fun.m:27)
               * tr(sinh(A)) per-probe quadratic forms, 256 Rademacher probes,
                 m = 30 (C restatement oracle/slq_ref.c; probes 0..7 also by
                 the numpy restatement)
               * mc_trace(Lanczos-sinh Afun, n, 1e-4, 1000, 1), the Hutch++
                 structure of mc_trace.m:42-58 (numpy restatement)
               * the 100 candidate edges (find_top_edges(A, c, 100, 'min')),
                 dfA = function_multiple_entries(A, E, @cosh, 1e-6 cosh(nrm), 100)
               * Omega = top 30 by dfA, a seeded nonzero X
               * [f, gr] = fun_and_grad_krylov_fun(X, A, Omega, @sinh, @cosh,
                 dfA, 1e-6 sinh(nrm), 100) and the exact objective
                 -(sum sinh(eig(A + U B U')) - sum sinh(eig(A))) (dense eigvalsh,
                 a few minutes) -> config3_values.json
  --config5  voltage India, greedy_krylov(A, 50, Q = min(nnz/2 - 50, 250), c,
             'min', 1e-6 exp(normest(A, 1e-2)), 100, inf, 0, 'break')
             (Tests/test_unweighted_break.m:56,72-74): the 50 selected edges,
             each step's variation, rob and a digest of A_new -> config5_values.json

Inputs that come from non-deterministic host helpers (the eigenvector
centrality of scipy's eigsh) are stored in the fixture and fed to both sides.
"""
from __future__ import annotations

import hashlib
import json
import os
import sys
import time

import numpy as np
import scipy.sparse as sp

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from oracle import krylov_oracle as ko  # noqa: E402
from oracle import slq_ref  # noqa: E402
from conftest import load_graph  # noqa: E402


def csc_digest(A):
    """sha256 over the sorted CSC arrays (int64 colptr, int64 rowind, f64 values)."""
    C = sp.csc_matrix(A)
    C.eliminate_zeros()
    C.sort_indices()
    h = hashlib.sha256()
    for a in (C.indptr.astype(np.int64), C.indices.astype(np.int64), C.data.astype(np.float64)):
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def centrality(A):
    """compute_centrality.m:15-17, abs(leading eigenvector) (dense eigh where
    it fits, else scipy eigsh); stored in the fixture."""
    import scipy.sparse.linalg as sla
    if A.shape[0] <= 4000:
        w, V = np.linalg.eigh(A.toarray())
        return np.abs(V[:, -1])
    _, u = sla.eigsh(A, k=1, which="LM", tol=1e-14, v0=np.ones(A.shape[0]))
    return np.abs(u[:, 0])


def config3():
    t00 = time.time()
    A = load_graph("hawaii")
    n = A.shape[0]
    rec = {"graph": "hawaii LCC (tests/golden/hawaii.npz)", "n": n, "nnz": int(A.nnz)}
    nrm = ko.normest(A, 1e-2)
    rec["normest_1e-2"] = nrm
    # 1. tr(sinh(A)) by plain Hutchinson: per-probe quadratic forms
    seed, N, m = 3, 256, 30
    _, q = slq_ref.slq_trace(A, N, m, seed=seed, fun="sinh")
    _, q8 = ko.slq_trace(A, 8, m, seed=seed, fun="sinh")
    rel = float(np.max(np.abs(q8 - q[:8]) / np.abs(q8)))
    assert rel < 1e-10, rel
    rec["slq_sinh"] = {"seed": seed, "probes": N, "m": m, "q": q.tolist(),
                       "numpy_vs_c_first8_max_rel": rel,
                       "estimate": float(q.mean()),
                       "stderr": float(q.std(ddof=1) / np.sqrt(N))}
    print("slq", q.mean(), f"{time.time() - t00:.1f}s", flush=True)
    # 2. Hutch++ (mc_trace structure) with the Lanczos-sinh Afun
    t0 = time.time()
    tr, res, it = ko.trace_exp_lanczos(A, m=m, tol=1e-4, maxit=1000, seed=seed, fun="sinh")
    rec["mc_trace_lanczos_sinh"] = {"seed": seed, "m": m, "tol": 1e-4, "maxit": 1000,
                                    "tr": tr, "res": res, "it": it}
    print("mc_trace", tr, res, it, f"{time.time() - t0:.1f}s", flush=True)
    # 3. Omega from centrality + function_multiple_entries(cosh)
    c = centrality(A)
    from krylov_robustness_amd.greedy import find_top_edges
    E = find_top_edges(A, c, 100, "min")
    tol_df = 1e-6 * np.cosh(nrm)
    t0 = time.time()
    temp, fit = ko.function_multiple_entries(A, E, "cosh", tol_df, 100)
    print("fme", fit, f"{time.time() - t0:.1f}s", flush=True)
    ind = np.argsort(-temp, kind="stable")[:30]
    Om = E[ind]
    dfA = temp[ind]
    srt = np.sort(temp)[::-1]
    rec["fme_cosh"] = {"E": E.tolist(), "tol": tol_df, "it": 100, "entries": temp.tolist(),
                       "iter": int(fit),
                       "rank30_gap_rel": float((srt[29] - srt[30]) / srt[29])}
    rng = np.random.default_rng(11)
    w = np.array([A[i - 1, j - 1] for i, j in Om])
    X = rng.uniform(-0.5, 1.0, size=30) * w
    if X.sum() > 10:
        X *= 10 / X.sum()
    tol = 1e-6 * np.sinh(nrm)
    t0 = time.time()
    f, gr = ko.fun_and_grad_krylov_fun(X, A, Om, "sinh", "cosh", dfA, tol, 100)
    print("fg", f, f"{time.time() - t0:.1f}s", flush=True)
    U, B = ko.lowrank_from_edges(X, Om, n)
    xm, itf, lk = ko.trace_fun_update(A, U, B, tol * np.sinh(nrm), 100, 0, "sinh")
    rec["fun_and_grad"] = {"Omega": Om.tolist(), "dfA": dfA.tolist(), "X": X.tolist(), "tol": tol,
                           "it": 100, "f": f, "gr": gr.tolist(), "rank": int(U.shape[1]),
                           "trace_fun_update": {"tol": tol * np.sinh(nrm), "Xm": xm, "iter": int(itf),
                                                "lucky": bool(lk)}}
    # exact objective (dense fp64 eigvalsh of A + U B U'; tr sinh(A) from hawaii_values.json)
    t0 = time.time()
    hv = json.load(open(os.path.join(HERE, "hawaii_values.json")))
    M = A.toarray()
    M += U @ B @ U.T
    M = (M + M.T) / 2
    d2 = np.linalg.eigvalsh(M)
    del M
    exact_tr_update = float(np.sum(np.sinh(d2)) - hv["exact_tr_sinh"])
    rec["fun_and_grad"]["exact_f"] = -exact_tr_update
    print("exact", -exact_tr_update, f"{time.time() - t0:.1f}s", flush=True)
    rec["exact_tr_sinh"] = hv["exact_tr_sinh"]
    rec["seconds"] = time.time() - t00
    with open(os.path.join(HERE, "config3_values.json"), "w") as fh:
        json.dump(rec, fh, indent=1)


def config5():
    t00 = time.time()
    A = load_graph("india")
    k = 50
    Q = int(min(A.nnz // 2 - k, 250))
    c = centrality(A)
    nrm = ko.normest(A, 1e-2)
    tol = 1e-6 * np.exp(nrm)
    edges, rob, An = ko.greedy_krylov(A, k, Q, c, "min", tol, 100, miobi="break")
    print("greedy", rob, f"{time.time() - t00:.1f}s", flush=True)
    # per-step variations: the same loop one step at a time (greedy_krylov.m:80-93)
    steps = []
    S = A.copy()
    from krylov_robustness_amd.greedy import find_top_edges
    top = find_top_edges(S, c, Q + k, "min")
    for j in range(k):
        e, r, S = ko.krylov_miobi(S, 1, top[:Q], tol, 100)
        steps.append(r)
        assert tuple(e[0]) == tuple(edges[j])
        hit = [h for h in range(len(top)) if tuple(top[h]) == tuple(e[0])]
        top = np.delete(top, hit[0], axis=0)
    rec = {"graph": "voltage India (A / max(A))", "n": int(A.shape[0]), "nnz": int(A.nnz),
           "k": k, "Q": Q, "order": "min", "miobi": "break", "it": 100,
           "normest_1e-2": nrm, "tol": tol, "centrality": c.tolist(),
           "edges": np.asarray(edges).tolist(), "rob": float(rob), "step_variation": steps,
           "A_new_nnz": int(An.nnz), "A_new_digest": csc_digest(An),
           "seconds": time.time() - t00}
    with open(os.path.join(HERE, "config5_values.json"), "w") as fh:
        json.dump(rec, fh, indent=1)


if __name__ == "__main__":
    if "--config5" in sys.argv:
        config5()
    if "--config3" in sys.argv:
        config3()

"""Generate the committed golden fixtures (run in the build container only).

Reads the reference's own datasets from /root/reference (MAT v5 via scipy),
prepares each graph the way the reference's test drivers do, and stores
  * graphs.npz   -- CSR arrays of the prepared graphs (data, not source)
  * values.json  -- exact dense answers (the reference's known-answer
                    identities) and oracle outputs on fixed seeds.
Usage:  python tests/golden/make_golden.py
The GPU box never runs this: /root/reference does not exist there.
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np
import scipy.io as sio
import scipy.sparse as sp
import scipy.sparse.csgraph as csg

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, ROOT)
from oracle import krylov_oracle as ko  # noqa: E402

REF = "/root/reference"


def unweighted(A):
    """test_unweighted_break.m:45-52: spones(A+A'), drop the diagonal, keep
    the largest connected component."""
    A = sp.csr_matrix(A, dtype=np.float64)
    A = ((A + A.T) != 0).astype(np.float64).tocsr()
    A.setdiag(0)
    A.eliminate_zeros()
    _, lab = csg.connected_components(A, directed=False)
    big = np.argmax(np.bincount(lab))
    ind = np.flatnonzero(lab == big)
    return A[ind][:, ind].tocsr()


def weighted_voltage(A):
    """test_weighted_exp_lbfgs.m:34-36: A = A / max(A(:))."""
    A = sp.csr_matrix(A, dtype=np.float64)
    return (A / A.max()).tocsr()


def load_graphs():
    g = {}
    d = sio.loadmat(os.path.join(REF, "MIOBI Codes", "dt_oregon.mat"))
    g["oregon_A0"] = unweighted(d["A0"])
    g["oregon_A6"] = unweighted(d["A6"])
    for name in ["Anaheim", "Rome"]:
        P = sio.loadmat(os.path.join(REF, "datasets_paper", "Transport", name + ".mat"))["Problem"]
        g[name.lower()] = unweighted(P["A"][0, 0])
    v = sio.loadmat(os.path.join(REF, "datasets_paper", "voltage_adjacencies_average_2.mat"))
    for name in ["Denmark", "Austria", "India"]:
        g[name.lower()] = weighted_voltage(v[name])
    return g


def save_csr(path, graphs):
    arrays = {}
    for k, A in graphs.items():
        A = A.tocsr()
        A.sort_indices()
        arrays[k + "__indptr"] = A.indptr.astype(np.int64)
        arrays[k + "__indices"] = A.indices.astype(np.int32)
        arrays[k + "__data"] = A.data.astype(np.float64)
        arrays[k + "__n"] = np.array([A.shape[0]], dtype=np.int64)
    np.savez_compressed(path, **arrays)


def main_hawaii():
    """Config 3's graph: Transport Hawaii, unweighted LCC, in
    its own file so graphs.npz stays byte-stable."""
    P = sio.loadmat(os.path.join(REF, "datasets_paper", "Transport", "Hawaii.mat"))["Problem"]
    A = unweighted(P["A"][0, 0])
    save_csr(os.path.join(HERE, "hawaii.npz"), {"hawaii": A})
    print("hawaii", A.shape[0], A.nnz)


V73 = ["Drugs", "as_735", "CollegeMsg"]


def _sha(a):
    import hashlib
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def main_v73():
    """The three MAT v7.3 (HDF5) datasets of datasets_paper/Misc (SURVEY.md
    §8f row 4), read with the package's own reader:
      * v73_values.json -- digests of the raw Problem.A (shape, nnz, sum,
        sha256 of the CSC arrays) that pin the reader, the CollegeMsg
        temporal-edge cross-check, and exact spectra of the prepared graphs;
        an oracle greedy_krylov 'make' selection on CollegeMsg
      * v73_graphs.npz -- the prepared graphs (test_unweighted_make.m:41-52)
    """
    from krylov_robustness_amd import datasets as ds
    graphs, vals = {}, {"_doc": "raw_* pin the MAT v7.3 reader; exact_* dense "
                                "eigvalsh of the prepared graph; oracle_* from "
                                "oracle/krylov_oracle.py"}
    for name in V73:
        path = os.path.join(REF, "datasets_paper", "Misc", name + ".mat")
        t0 = time.time()
        P = ds.load_variable(path, "Problem")
        R = sp.csc_matrix(P["A"])
        rec = {"raw_shape": list(R.shape), "raw_nnz": int(R.nnz), "raw_sum": float(R.sum()),
               "raw_sha_indptr": _sha(R.indptr.astype(np.int64)),
               "raw_sha_indices": _sha(R.indices.astype(np.int64)),
               "raw_sha_data": _sha(R.data.astype(np.float64)),
               "name": P.get("name")}
        if name == "CollegeMsg":
            te = np.asarray(P["aux"]["temporal_edges"])
            rec["temporal_edges"] = [int(te.shape[0]), int(te.shape[1])]
        A = ds.prepare_unweighted(P["A"])
        graphs[name.lower()] = A
        d = np.linalg.eigvalsh(A.toarray())
        rec.update({"n": int(A.shape[0]), "nnz": int(A.nnz), "lambda_max": float(d.max()),
                    "exact_tr_exp": float(np.sum(np.exp(d))),
                    "exact_tr_sinh": float(np.sum(np.sinh(d))),
                    "exact_tr_cosh": float(np.sum(np.cosh(d)))})
        vals[name.lower()] = rec
        print(name, rec["n"], rec["nnz"], f"{time.time() - t0:.1f}s", flush=True)
    # greedy_krylov 'make' on CollegeMsg (test_unweighted_make.m:70-76 with a
    # smaller budget): eigenvector centrality from a dense eigh
    A = graphs["collegemsg"]
    w, V = np.linalg.eigh(A.toarray())
    cen = np.abs(V[:, -1])
    t0 = time.time()
    k, Q = 3, 40
    edges, rob, _ = ko.greedy_krylov(A, k, Q, cen, "min", 1e-6 * np.exp(w[-1]), 100,
                                     miobi="make")
    vals["collegemsg"]["oracle_greedy_make"] = {
        "k": k, "Q": Q, "order": "min", "tol": 1e-6 * float(np.exp(w[-1])), "it": 100,
        "centrality": "abs(leading eigenvector), dense eigh",
        "edges": np.asarray(edges).tolist(), "rob": float(rob)}
    print("greedy", np.asarray(edges).tolist(), rob, f"{time.time() - t0:.1f}s")
    save_csr(os.path.join(HERE, "v73_graphs.npz"), graphs)
    with open(os.path.join(HERE, "v73_values.json"), "w") as f:
        json.dump(vals, f, indent=1)


def main():
    if "--hawaii" in sys.argv:
        return main_hawaii()
    if "--v73" in sys.argv:
        return main_v73()
    graphs = load_graphs()
    arrays = {}
    for k, A in graphs.items():
        A = A.tocsr()
        A.sort_indices()
        arrays[k + "__indptr"] = A.indptr.astype(np.int64)
        arrays[k + "__indices"] = A.indices.astype(np.int32)
        arrays[k + "__data"] = A.data.astype(np.float64)
        arrays[k + "__n"] = np.array([A.shape[0]], dtype=np.int64)
    np.savez_compressed(os.path.join(HERE, "graphs.npz"), **arrays)

    vals = {"_doc": "exact = known-answer identities of the reference; oracle_* = "
                    "oracle/krylov_oracle.py on the stated seeds"}
    for k, A in graphs.items():
        t0 = time.time()
        n = A.shape[0]
        rec = {"n": int(n), "nnz": int(A.nnz)}
        d = np.linalg.eigvalsh(A.toarray())                 # exact spectrum
        rec["lambda_max"] = float(d.max())
        rec["exact_tr_exp"] = float(np.sum(np.exp(d)))       # test_weighted_exp_lbfgs.m:41
        rec["exact_tr_sinh"] = float(np.sum(np.sinh(d)))     # test_weighted_sinh_lbfgs.m:50
        rec["exact_tr_cosh"] = float(np.sum(np.cosh(d)))
        # SLQ per-probe quadratic forms (seed 7, probes 0..15, m = 20)
        if n <= 4000:
            _, q = ko.slq_trace(A, 16, 20, seed=7, fun="exp")
            rec["oracle_slq_exp_seed7_m20"] = q.tolist()
            _, q = ko.slq_trace(A, 16, 20, seed=7, fun="sinh")
            rec["oracle_slq_sinh_seed7_m20"] = q.tolist()
        # trace_fun_update on the first 3 existing edges (krylov_miobi.m:77-99 U, B)
        if n <= 4000:
            I, J = sp.triu(A, 1).nonzero()
            cases = []
            for h in range(3):
                i, j = int(I[h]) + 1, int(J[h]) + 1
                U = np.zeros((n, 2)); U[i - 1, 0] = 1; U[j - 1, 1] = 1
                B = -np.array([[0.0, 1.0], [1.0, 0.0]])
                xm, it, lucky = ko.trace_fun_update(A, U, B, 1e-12, min(100, n), 0, "exp")
                ex = ko.exact_trace_update(A, U, B, "exp")
                cases.append({"edge": [i, j], "oracle": xm, "iter": int(it), "exact": ex})
            rec["trace_fun_update_break"] = cases
        vals[k] = rec
        print(k, n, A.nnz, f"{time.time() - t0:.1f}s", flush=True)
    with open(os.path.join(HERE, "values.json"), "w") as f:
        json.dump(vals, f, indent=1)


if __name__ == "__main__":
    main()

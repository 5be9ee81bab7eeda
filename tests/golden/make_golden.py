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


def main():
    if "--hawaii" in sys.argv:
        return main_hawaii()
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

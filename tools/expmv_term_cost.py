"""Device time per Taylor term of expmv on 10 columns: dt_oregon A6 (config 1,
power law, hub degree 1,519) vs graphs of the same n and nnz without hubs
(Erdos-Renyi) and with the hub rows' degrees capped (same graph minus the
edges past degree 64 of every hub).  One JSON line per graph."""
import json
import os
import sys
import time

import torch  # noqa: F401
import numpy as np
import scipy.sparse as sp

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import krylov_robustness_amd as kra  # noqa: E402
from krylov_robustness_amd import graphs  # noqa: E402
from conftest import load_graph  # noqa: E402

A6 = load_graph("oregon_A6").tocsr()
n, nnz = A6.shape[0], A6.nnz
er = graphs.erdos_renyi(n, nnz // 2, seed=3).tocsr()


def capped(A, cap):
    A = sp.triu(A, 1).tocoo()
    deg = np.zeros(A.shape[0], dtype=np.int64)
    keep = np.zeros(A.nnz, dtype=bool)
    for k in np.argsort(np.random.default_rng(0).random(A.nnz)):
        i, j = A.row[k], A.col[k]
        if deg[i] < cap and deg[j] < cap:
            keep[k] = True
            deg[i] += 1
            deg[j] += 1
    U = sp.csr_matrix((A.data[keep], (A.row[keep], A.col[keep])), shape=A.shape)
    return (U + U.T).tocsr()


ctx = kra.Context(0)
b = np.random.default_rng(1).normal(size=(n, 10))
for name, G in (("oregon_A6", A6), ("erdos_renyi_same_n_nnz", er), ("oregon_A6_deg_capped_64", capped(A6, 64))):
    D = kra.DeviceMatrix(G, ctx)
    kra.expmv(1.0, D, b, ctx=ctx)
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        F, s, m, mv = kra.expmv(1.0, D, b, ctx=ctx)
        ts.append(time.perf_counter() - t0)
    t = min(ts)
    print(json.dumps({"graph": name, "n": G.shape[0], "nnz": G.nnz, "max_deg": int(np.diff(G.indptr).max()),
                      "s": s, "m": m, "mv": mv, "ms": round(t * 1e3, 3), "us_per_mv": round(t * 1e6 / max(mv, 1), 2)}),
          flush=True)

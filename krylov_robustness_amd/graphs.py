"""Seeded synthetic graphs for the benchmark configs.

Host-side input generation only (NumPy): the GPU box regenerates the graphs
from the seed instead of shipping them.  All graphs are symmetric, unit
weight, with no self loops, as the reference's tests prepare them
(test_unweighted_break.m:45-47: spones(A + A'), diagonal removed).
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp


def _sym_csr_from_pairs(i, j, n):
    """Undirected unique pairs (i < j) -> symmetric CSR with unit weights."""
    rows = np.concatenate([i, j])
    cols = np.concatenate([j, i])
    key = rows.astype(np.int64) * n + cols
    key.sort()
    rows = (key // n).astype(np.int64)
    cols = (key % n).astype(np.int32)
    indptr = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(np.bincount(rows, minlength=n), out=indptr[1:])
    data = np.ones(cols.size, dtype=np.float64)
    return sp.csr_matrix((data, cols, indptr), shape=(n, n))


def _unique_pairs(i, j, n):
    lo = np.minimum(i, j).astype(np.int64)
    hi = np.maximum(i, j).astype(np.int64)
    keep = lo != hi
    key = np.unique(lo[keep] * n + hi[keep])
    return key


def erdos_renyi(n: int = 100_000, npairs: int = 500_000, seed: int = 0):
    """Config 2: `npairs` uniform (i, j), symmetrised, diagonal dropped."""
    rng = np.random.default_rng(seed)
    i = rng.integers(0, n, npairs)
    j = rng.integers(0, n, npairs)
    key = _unique_pairs(i, j, n)
    return _sym_csr_from_pairs(key // n, key % n, n)


def chung_lu(n: int = 1_000_000, nnz: int = 10_000_000, gamma: float = 2.5,
             max_degree: float | None = None, seed: int = 0, permute: bool = True):
    """Config 4: Chung-Lu graph with power-law expected degrees
    d_i ~ (i + i0)^(-1/(gamma-1)), scaled to sum(d) = nnz, with the offset i0
    chosen so the largest expected degree is the structural cutoff
    sqrt(nnz) (unless `max_degree` is given).  Exactly nnz/2 distinct
    undirected edges are drawn (endpoints independent, P(i) ~ d_i), so the
    symmetric CSR has exactly `nnz` entries.  `permute` relabels nodes with a
    seeded random permutation so that hubs are not clustered at low indices."""
    rng = np.random.default_rng(seed)
    expo = 1.0 / (gamma - 1.0)
    dmax = float(max_degree) if max_degree else float(np.sqrt(nnz))
    idx = np.arange(n, dtype=np.float64)

    def top(i0):
        w = (idx + i0) ** (-expo)
        return nnz * w[0] / w.sum()

    lo, hi = 1e-6, float(n)
    for _ in range(200):                       # bisection on i0: top(i0) = dmax
        mid = np.sqrt(lo * hi)
        if top(mid) > dmax:
            lo = mid
        else:
            hi = mid
    w = (idx + hi) ** (-expo)
    cdf = np.cumsum(w)
    cdf /= cdf[-1]
    target = nnz // 2
    keys = np.empty(0, dtype=np.int64)
    batch = int(target * 1.05) + 1024
    while keys.size < target:
        a = np.searchsorted(cdf, rng.random(batch), side="right")
        b = np.searchsorted(cdf, rng.random(batch), side="right")
        a = np.minimum(a, n - 1)
        b = np.minimum(b, n - 1)
        keys = np.unique(np.concatenate([keys, _unique_pairs(a, b, n)]))
        batch = int((target - keys.size) * 1.3) + 1024
    # keep a seeded random subset of exactly `target` edges
    keys = rng.permutation(keys)[:target]
    i = keys // n
    j = keys % n
    if permute:
        perm = rng.permutation(n)
        i, j = perm[i], perm[j]
    return _sym_csr_from_pairs(np.minimum(i, j), np.maximum(i, j), n)


def symmetric_weights(A, seed: int = 1, low: float = 0.5, high: float = 1.5):
    """Seeded fp64 weights on a symmetric pattern: w_ij = w_ji uniform in
    [low, high), drawn per undirected edge in (row, col) order of the upper
    triangle.  The weighted drivers' A (Tests/test_weighted_exp_lbfgs.m, a
    weighted symmetric adjacency) at the size of a synthetic pattern: every
    stored value differs from 1, so the 12 B/nnz CSR path (values read) runs."""
    rng = np.random.default_rng(seed)
    U = sp.triu(sp.csr_matrix(A), k=1).tocoo()
    order = np.lexsort((U.col, U.row))
    r, c = U.row[order], U.col[order]
    w = rng.uniform(low, high, r.size)
    W = sp.coo_matrix((np.concatenate([w, w]), (np.concatenate([r, c]), np.concatenate([c, r]))),
                      shape=A.shape).tocsr()
    W.sort_indices()
    return W

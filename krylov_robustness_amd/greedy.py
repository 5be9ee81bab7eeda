"""Greedy edge selection over the device path: krylov_miobi.m / greedy_krylov.m.

``krylov_miobi`` scores every candidate edge of a greedy step with the batched
device evaluation (kt_trace_fun_update_pairs: one block-2 Lanczos run per
candidate, all candidates advanced by one SpMM per step) and edits A on the
device (kt_matrix_set_pairs).  ``greedy_krylov`` is the reference's outer loop
(greedy_krylov.m:64-93) with the search-space heuristics find_top_edges.m /
find_top_missing_edges.m restated on the host: they are ordering/combinatorics
on node centralities, not bandwidth work.

Indices follow the reference: edges are 1-based (i, j) rows with
E(:, 1) >= E(:, 2) for krylov_miobi's candidate lists.
"""
from __future__ import annotations

import ctypes as C
import warnings
from typing import Optional

import numpy as np

from . import _lib
from .core import Context, DeviceMatrix, _dev, _dptr, _fun_code, normest


def _i64(a):
    a = np.ascontiguousarray(np.asarray(a, dtype=np.int64))
    return a, a.ctypes.data_as(C.POINTER(C.c_int64))


def trace_fun_update_pairs(A, E, B, tol=1e-12, it=None, fun="exp", b_self=None,
                           ctx: Optional[Context] = None):
    """Xm[h] = trace_fun_update(A, U_h, B, tol, it, 0, fun) for every candidate
    edge h of E (q x 2, 1-based), U_h = [e_E(h,1), e_E(h,2)] as built in
    krylov_miobi.m:76-98 (a self-loop candidate uses U = e_i and B = b_self).
    Returns (Xm, iter, lucky) arrays."""
    D = _dev(A, ctx)
    E = np.asarray(E, dtype=np.int64).reshape(-1, 2)
    q = E.shape[0]
    ei, pi = _i64(E[:, 0] - 1)
    ej, pj = _i64(E[:, 1] - 1)
    Bm = np.asfortranarray(np.asarray(B, dtype=np.float64).reshape(2, 2))
    if b_self is None:
        b_self = float(Bm[0, 1])
    xm = np.zeros(q)
    itr = np.zeros(q, dtype=np.int32)
    lk = np.zeros(q, dtype=np.int32)
    _lib.check(_lib.load().kt_trace_fun_update_pairs(
        D.handle, q, pi, pj, _dptr(Bm), float(b_self), float(tol), int(it or 0), _fun_code(fun),
        _dptr(xm), itr.ctypes.data_as(C.POINTER(C.c_int)), lk.ctypes.data_as(C.POINTER(C.c_int))))
    return xm, itr, lk


def krylov_miobi(A, k, E=None, tol=1e-12, it=None, poles=np.inf, debug=0, miobi="break",
                 rescale=1.0, ctx: Optional[Context] = None):
    """[edges, rob, A_new] = krylov_miobi(A, k, E, tol, it, poles, debug, miobi, rescale)
    (krylov_miobi.m:1).  A may be a DeviceMatrix (edited in place and returned)
    or a matrix (uploaded; the returned DeviceMatrix holds A_new)."""
    if miobi not in ("break", "make"):
        raise _lib.KrylovError(_lib.KT_ERR_ARG, "KRYLOV_MIOBI:: not supported option for miobi")
    D = _dev(A, ctx)
    if E is None or len(E) == 0:  # :42-46  all edges with E(:,1) >= E(:,2)
        S = D.to_scipy().tocoo()
        keep = S.row >= S.col
        E = np.stack([S.row[keep], S.col[keep]], axis=1) + 1
        E = E[np.lexsort((E[:, 0], E[:, 1]))]  # MATLAB find(): column-major order
    E = np.asarray(E, dtype=np.int64).reshape(-1, 2)
    nE = E.shape[0]
    ei, pi = _i64(E[:, 0] - 1)
    ej, pj = _i64(E[:, 1] - 1)
    cap = max(min(int(k), nE), 1)
    si = np.zeros(cap, dtype=np.int64)
    sj = np.zeros(cap, dtype=np.int64)
    rob = C.c_double()
    ns = C.c_int64()
    _lib.check(_lib.load().kt_krylov_miobi(
        D.handle, int(k), nE, pi, pj, float(tol), int(it or 0), 1 if miobi == "make" else 0,
        float(rescale), si.ctypes.data_as(C.POINTER(C.c_int64)),
        sj.ctypes.data_as(C.POINTER(C.c_int64)), C.byref(rob), C.byref(ns)))
    m = int(ns.value)
    edges = np.stack([si[:m] + 1, sj[:m] + 1], axis=1)
    return edges, float(rob.value), D


def select_extreme(xm, make):
    """krylov_miobi.m:112-124: strict comparison, the first extreme wins.
    Returns (index, value); index -1 if no candidate compares (all NaN)."""
    best, bv = -1, (-np.inf if make else np.inf)
    for h, v in enumerate(np.asarray(xm, dtype=np.float64)):
        if (v > bv) if make else (v < bv):
            best, bv = h, float(v)
    return best, bv


def miobi_loop(k, E, make, score, edit):
    """Host loop of krylov_miobi.m:70-139 over injectable scoring / editing:
    score(E) -> the trace variation of every candidate row of E (1-based),
    edit(edge, value) applies A(i,j) = A(j,i) = value.  Returns (edges, rob)."""
    E = np.asarray(E, dtype=np.int64).reshape(-1, 2).copy()
    edges, rob = [], 0.0
    for _ in range(min(int(k), E.shape[0])):
        xm = score(E)
        best, bv = select_extreme(xm, make)
        if best < 0:
            raise _lib.KrylovError(_lib.KT_ERR_ARG, "KRYLOV_MIOBI:: no finite candidate score")
        chosen = E[best].copy()
        E = np.delete(E, best, axis=0)               # :127
        edit(chosen, 1.0 if make else 0.0)           # :129-135
        edges.append(chosen)
        rob += bv
    return np.array(edges, dtype=np.int64).reshape(-1, 2), rob


def krylov_miobi_sharded(A, k, E, tol=1e-12, it=None, poles=np.inf, debug=0, miobi="break",
                         rescale=1.0, group=None, ctx: Optional[Context] = None):
    """krylov_miobi with the candidate scoring sharded over the ranks of the
    process group: rank r scores its contiguous slice of E on
    its own GPU (kt_trace_fun_update_pairs), the scores are all-gathered in
    rank order, every rank picks the same extreme candidate and edits its own
    device copy of A.  Same result as krylov_miobi on one GPU."""
    import torch.distributed as dist
    from .dist import allgather_concat, probe_shard
    if miobi not in ("break", "make"):
        raise _lib.KrylovError(_lib.KT_ERR_ARG, "KRYLOV_MIOBI:: not supported option for miobi")
    D = _dev(A, ctx)
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    make = miobi == "make"
    sg = 1.0 if make else -1.0
    B = sg * np.array([[0.0, 1.0], [1.0, 0.0]]) / rescale

    def score(Ecur):
        counts = [probe_shard(len(Ecur), r, world)[1] for r in range(world)]
        off, cnt = probe_shard(len(Ecur), rank, world)
        xm = (trace_fun_update_pairs(D, Ecur[off:off + cnt], B, tol, it, b_self=sg, ctx=ctx)[0]
              if cnt else np.zeros(0))
        return allgather_concat(xm, counts, group)

    def edit(e, value):
        D.set_pairs([e], value)

    edges, rob = miobi_loop(k, E, make, score, edit)
    return edges, rob, D


def _stable_head(key, num):
    """argsort(key, kind="stable")[:num] without sorting the whole key: every
    entry at or below the num-th smallest value, in index order, then a
    stable sort of those (same ties, same order)."""
    if num >= len(key):
        return np.argsort(key, kind="stable")
    th = np.partition(key, num - 1)[num - 1]
    if np.isnan(th):  # NaN keys sort last in argsort: take the full sort
        return np.argsort(key, kind="stable")[:num]
    cand = np.flatnonzero(key <= th)
    return cand[np.argsort(key[cand], kind="stable")][:num]


def find_top_edges(A, centrality, num, order="mult"):
    """find_top_edges.m:1-40: the top `num` existing edges (1-based, i > j)."""
    import scipy.sparse as sp
    L = A if sp.isspmatrix_csc(A) else sp.csc_matrix(A)
    if not L.has_canonical_format:  # duplicates summed (tril(A) sees sums), sorted
        L = L.copy()
        L.sum_duplicates()
    # find(tril(A, -1)) in column-major order, read straight off the CSC arrays
    J = np.repeat(np.arange(L.shape[1], dtype=np.int64), np.diff(L.indptr))
    keep = (L.indices > J) & (L.data != 0)
    I = L.indices[keep].astype(np.int64)
    J = J[keep]
    c = np.asarray(centrality, dtype=np.float64).ravel()
    if order == "mult":  # :22-25
        key = -(c[I] * c[J])
    elif order == "min":  # :26-37
        # find(sc == v, 1) with sc = sort(c, 'descend'): the first descending
        # position of v is n - (last ascending position of v), i.e.
        # n - searchsorted(ascending, v, 'right') + 1 (1-based), once per node
        nc = len(c)
        rank = (nc - np.searchsorted(np.sort(c), c, side="right") + 1).astype(np.float64)
        c1, c2 = rank[I], rank[J]
        mn, mx = np.minimum(c1, c2), np.maximum(c1, c2)
        key = mx * (mx - 1) / 2 + mn
    else:
        return np.stack([I + 1, J + 1], axis=1)
    # :19-21 warns when fewer than num edges exist; E(ind(1:num), :) then
    # indexes floor(num) of them and fails only if those are missing too
    if len(I) < num:
        warnings.warn("FIND_TOP_EDGES:: there are not enough edges in the graph")
    num = int(np.floor(num))
    if len(I) < num:
        raise IndexError("FIND_TOP_EDGES:: there are not enough edges in the graph")
    ind = _stable_head(key, num)
    return np.stack([I[ind] + 1, J[ind] + 1], axis=1)


def find_top_missing_edges(A, centrality, num, order="min"):
    """find_top_missing_edges.m:1-67: the top `num` missing edges (1-based)."""
    import scipy.sparse as sp
    A = sp.csr_matrix(A)
    n = A.shape[0]
    c = np.asarray(centrality, dtype=np.float64).ravel()
    indC = np.argsort(-c, kind="stable")  # [sc, indC] = sort(centrality, 'descend')
    sc = c[indC]
    if order == "min":  # :52-64
        E = []
        j = 1
        while len(E) < num:
            if j >= n:
                raise IndexError("FIND_TOP_MISSING_EDGES:: not enough missing edges")
            col = A[indC[:j], :][:, [indC[j]]].toarray().ravel()
            for t in np.flatnonzero(col == 0):
                E.append((indC[t] + 1, indC[j] + 1))
            j += 1
        return np.array(E[:int(np.floor(num))], dtype=np.int64)  # E(1:num, :) with a fractional num
    if order == "mult":  # :22-51
        if (n * n - A.nnz - n) / 2 <= num:
            raise RuntimeError("FIND_TOP_MISSING_EDGES:: output E is not assigned on this branch "
                               "(find_top_missing_edges.m:23-30 returns before setting E)")
        min_N, ln = 2, 0
        while ln < num:
            ln += int(np.sum(A[indC[:min_N - 1], :][:, [indC[min_N - 1]]].toarray() == 0))
            min_N += 1
        min_N -= 1
        N = int(np.sum(sc[0] * sc > sc[min_N - 1] ** 2))
        S = np.triu(np.outer(c[indC[:N]], c[indC[:N]]))
        lin = np.argsort(-S.ravel(order="F"), kind="stable")
        I, J = lin % N, lin // N
        I, J = indC[I], indC[J]
        E = []
        for a, b in zip(I, J):
            if len(E) >= num:
                break
            if a != b and A[a, b] == 0:
                E.append((a + 1, b + 1))
        return np.array(E, dtype=np.int64).reshape(-1, 2)
    raise ValueError(f"unknown order {order!r}")


def edge2low_rank(E, n, value=-1.0):
    """[U, B] = edge2low_rank(E, n): the low-rank factors of an edge edit,
    A + U B U' (functions/edge2low_rank.m:1-13, value = -1: remove the edges;
    the make drivers' local copy, Tests/test_unweighted_make.m:171-183, uses
    +1: add them).  E: m x 2 1-based node pairs.  U: n x k sparse selector of
    the k distinct nodes (ascending, as unique()), B: k x k dense with
    B(a, b) = B(b, a) = value for every edge."""
    import scipy.sparse as sp
    E = np.asarray(E, dtype=np.int64).reshape(-1, 2)
    t1, t2 = E[:, 0], E[:, 1]
    ut = np.unique(np.concatenate([t1, t2]))
    if ut.size and (ut[0] < 1 or ut[-1] > n):
        raise _lib.KrylovError(_lib.KT_ERR_ARG, "edge2low_rank: node index out of range")
    k = ut.size
    U = sp.csc_matrix((np.ones(k), (ut - 1, np.arange(k))), shape=(int(n), k))
    B = np.zeros((k, k))
    a = np.searchsorted(ut, t1)
    b = np.searchsorted(ut, t2)
    B[a, b] = value
    B[b, a] = value
    return U, B


def compute_centrality(A, kind="eig", ctx: Optional[Context] = None):
    """compute_centrality.m: 'eig' = abs(leading eigenvector) (:15-17), on the
    device when A is a DeviceMatrix (kt_eigs_leading), else scipy eigsh;
    'deg' = column sums (:18-19)."""
    import scipy.sparse as sp
    import scipy.sparse.linalg as sla
    if isinstance(A, DeviceMatrix):
        if kind == "deg":
            return np.asarray(A.to_scipy().sum(axis=0)).ravel()
        from .core import eigs_leading
        return np.abs(eigs_leading(A, ctx=ctx)[1])
    A = sp.csr_matrix(A, dtype=np.float64)
    if kind == "deg":
        return np.asarray(A.sum(axis=0)).ravel()
    _, u = sla.eigsh(A, k=1, which="LM")  # eigs(A, 1): largest magnitude
    return np.abs(u[:, 0])


def _is_symmetric(S):
    """issymmetric(A) for the sorted CSC the device exports: CSR of A equals
    its CSC exactly when A == A' entry for entry (the fast path); anything
    else falls back to the elementwise comparison."""
    R = S.tocsr()
    if (R.has_sorted_indices and np.array_equal(R.indptr, S.indptr)
            and np.array_equal(R.indices, S.indices) and np.array_equal(R.data, S.data)):
        return True
    return not (S != S.T).nnz


def greedy_krylov(A, k, Q=0, centrality=None, order="mult", tol=1e-12, it=None, poles=np.inf,
                  debug=0, miobi="break", rescale=1.0, ctx: Optional[Context] = None):
    """[edges, rob_variation, A_new] = greedy_krylov(A, k, Q, centrality, order, tol, it,
    poles, debug, miobi, rescale)  (greedy_krylov.m:1-100).  Returns A_new as
    the DeviceMatrix the edits were applied to (``.to_scipy()`` for the host copy)."""
    D = _dev(A, ctx)
    S = D.to_scipy()
    if not _is_symmetric(S):  # :27-29
        raise _lib.KrylovError(_lib.KT_ERR_NOT_HERMITIAN, "GREEDY_KRYLOV:: Adjacency matrix should be symmetric")
    if not Q:
        # :42-44 Q = max(sum(A, 1)); top_edges(1:Q, :) indexes floor(Q) rows, so
        # a weighted graph whose largest weighted degree is below 1 gives Q = 0,
        # an empty E, and krylov_miobi then scores every edge (krylov_miobi.m:43-46)
        Q = float(np.asarray(S.sum(axis=0)).max())
    # the ranking is asked for Q + k edges unfloored (find_top_edges.m:19 warns
    # against that count); every index use is 1:Q, i.e. floor(Q) rows
    Qn = Q + k
    Q = int(np.floor(Q))
    if miobi == "break" and S.nnz < 2 * k:  # :54-56
        raise _lib.KrylovError(_lib.KT_ERR_ARG, "GREEDY_KRYLOV:: edges to be removed are more than edges in the network")
    if centrality is None:
        centrality = compute_centrality(D, "eig", ctx=ctx)
    top = (find_top_missing_edges(S, centrality, Qn, order) if miobi == "make"
           else find_top_edges(S, centrality, Qn, order))  # :82 (first step)
    if len(top) >= int(k) > 0 and int(Q) >= 1:
        # the step loop in the library (kt_greedy_krylov_steps): krylov_miobi(A, 1,
        # top(1:Q)) per step, the selected pair dropped from the ranking (:84-89)
        T = np.asarray(top, dtype=np.int64).reshape(-1, 2)
        ti, pi = _i64(T[:, 0] - 1)
        tj, pj = _i64(T[:, 1] - 1)
        si = np.zeros(int(k), dtype=np.int64)
        sj = np.zeros(int(k), dtype=np.int64)
        rb = C.c_double()
        ns = C.c_int64()
        _lib.check(_lib.load().kt_greedy_krylov_steps(
            D.handle, int(k), int(Q), len(T), pi, pj, float(tol), int(it or 0), 1 if miobi == "make" else 0,
            float(rescale), si.ctypes.data_as(C.POINTER(C.c_int64)), sj.ctypes.data_as(C.POINTER(C.c_int64)),
            C.byref(rb), C.byref(ns)))
        m = int(ns.value)
        return np.stack([si[:m] + 1, sj[:m] + 1], axis=1), float(rb.value), D
    edges = np.zeros((0, 2), dtype=np.int64)
    rob = 0.0
    last = None
    for j in range(int(k)):  # :64-93
        if j > 0:  # drop the previously selected edge from the search space
            hit = np.flatnonzero(np.all(top == last, axis=1))
            # :84-86; with no match [1 : ind-1, ind+1 : n] is empty and so is top_edges
            top = np.delete(top, hit[0], axis=0) if len(hit) else top[:0]
        E = top[:Q]
        tmp_edges, tmp_rob, D = krylov_miobi(D, 1, E, tol, it, poles, debug, miobi, rescale)
        edges = np.vstack([edges, tmp_edges])
        rob += tmp_rob
        last = tmp_edges[0] if len(tmp_edges) else None
    return edges, rob, D


def default_greedy_tol(A, rel=1e-6, ctx: Optional[Context] = None):
    """tol = 1e-6 * exp(normest(A)) as the greedy test drivers set it
    (Tests/test_unweighted_break.m:56,74: nrm = exp(normest(A, 1e-2)))."""
    return rel * float(np.exp(normest(A, 1e-2, ctx=ctx)))

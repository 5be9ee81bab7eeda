"""Row -> XCD schedules for run.py (each returns order, xoff)."""
import numpy as np


def _pack(groups, A, key=None):
    deg = np.diff(A.indptr)
    lists = []
    for g in range(8):
        rows = np.where(groups == g)[0]
        if key is not None:
            rows = rows[np.argsort(key[rows], kind="stable")]
        lists.append(rows)
    order = np.concatenate(lists)
    xoff = np.concatenate([[0], np.cumsum([len(l) for l in lists])])
    return order, xoff


def contiguous(A):
    """Each XCD takes one contiguous eighth of the rows (by nnz)."""
    cum = A.indptr[1:]
    g = np.minimum((cum * 8) // (A.nnz + 1), 7)
    return _pack(g, A)


def _balanced_split(order, A, parts=8):
    nz = np.diff(A.indptr)[order]
    cum = np.cumsum(nz)
    g = np.minimum((cum * parts) // (cum[-1] + 1), parts - 1)
    xoff = np.concatenate([[0], np.searchsorted(g, np.arange(1, parts)), [len(order)]])
    return order, xoff


def _primary(A, t0):
    """Per row: its highest-degree neighbour that is not among the top t0
    (hubs-first labels: the smallest column index >= t0), n if none."""
    n = A.shape[0]
    col = A.indices.astype(np.int64)
    col[col < t0] = n
    rows = np.repeat(np.arange(n), np.diff(A.indptr))
    prim = np.full(n, n, dtype=np.int64)
    np.minimum.at(prim, rows, col)
    return prim


def sort_primary_4k(A):
    prim = _primary(A, 4096)
    order = np.argsort(prim, kind="stable")
    return _balanced_split(order, A)


def sort_primary_0(A):
    prim = _primary(A, 0)
    order = np.argsort(prim, kind="stable")
    return _balanced_split(order, A)


def _hgroup(A, t0, k, order_within=None):
    """Columns of degree rank [t0, t0 + 8k) get a home XCD ((c - t0) % 8);
    each row goes to the XCD holding most of its home-set neighbours, under
    a 1 % nnz balance cap (greedy, strongest preference first)."""
    n = A.shape[0]
    deg = np.diff(A.indptr)
    col = A.indices.astype(np.int64)
    rows = np.repeat(np.arange(n), deg)
    inh = (col >= t0) & (col < t0 + 8 * k)
    cnt = np.zeros((n, 8), dtype=np.int32)
    np.add.at(cnt, (rows[inh], (col[inh] - t0) % 8), 1)
    pref = np.argsort(-cnt, axis=1, kind="stable")
    best = cnt.max(axis=1)
    cap = A.nnz / 8 * 1.01
    load = np.zeros(8)
    g = np.full(n, -1, dtype=np.int64)
    for r in np.argsort(-best, kind="stable"):
        for q in pref[r]:
            if load[q] + deg[r] <= cap:
                g[r] = q
                load[q] += deg[r]
                break
        else:
            q = int(np.argmin(load))
            g[r] = q
            load[q] += deg[r]
    lists = []
    for q in range(8):
        rr = np.where(g == q)[0]
        if order_within is not None:
            rr = rr[np.argsort(order_within[rr], kind="stable")]
        lists.append(rr)
    order = np.concatenate(lists)
    xoff = np.concatenate([[0], np.cumsum([len(l) for l in lists])])
    return order, xoff


def hgroup_4k_16k(A):
    return _hgroup(A, 4096, 16384)


def hgroup_4k_32k(A):
    return _hgroup(A, 4096, 32768)


def hgroup_0_64k(A):
    return _hgroup(A, 0, 65536)


def hgroup_4k_16k_prim(A):
    return _hgroup(A, 4096, 16384, _primary(A, 4096))

"""Host-side search-space heuristics of the greedy path (find_top_edges.m,
find_top_missing_edges.m) against the oracle's loop restatements, and the
greedy argument checks that run before any device work.  CPU only."""
import numpy as np
import pytest

from conftest import load_graph
from oracle import krylov_oracle as ko

import krylov_robustness_amd as kra


@pytest.mark.parametrize("name", ["india", "rome", "austria", "anaheim"])
@pytest.mark.parametrize("order", ["mult", "min"])
def test_find_top_edges_matches_oracle(name, order):
    A = load_graph(name)
    c = kra.compute_centrality(A)
    num = min(120, A.nnz // 2)
    np.testing.assert_array_equal(kra.find_top_edges(A, c, num, order),
                                  ko.find_top_edges(A, c, num, order))


def test_find_top_edges_ties_keep_find_order():
    """Equal centralities: MATLAB's stable sort keeps find()'s column-major order."""
    A = load_graph("denmark")
    c = np.ones(A.shape[0])
    E = kra.find_top_edges(A, c, 20, "mult")
    np.testing.assert_array_equal(E, ko.find_top_edges(A, c, 20, "mult"))
    assert np.all(np.diff(E[:, 1]) >= 0)          # columns ascending
    assert np.all(E[:, 0] > E[:, 1])               # tril(A, -1)


@pytest.mark.parametrize("order", ["mult", "min"])
@pytest.mark.parametrize("num", [1, 37, 200, 323])
def test_find_top_edges_partial_sort_ties_zeros_layouts(order, num):
    """The partial stable sort (greedy._stable_head) and the CSC read-off
    against the oracle's full sort: heavily tied centralities (so the cut at
    `num` falls inside a run of equal keys), explicit stored zeros (find()
    skips them), unsorted CSC indices, and CSR / dense inputs."""
    import scipy.sparse as sp
    rng = np.random.default_rng(num)
    n = 60
    M = sp.random(n, n, density=0.2, random_state=rng, format="csr")
    M = ((M + M.T) > 0).astype(np.float64).tolil()
    M.setdiag(0)
    A = sp.csc_matrix(M)
    A.eliminate_zeros()
    c = rng.integers(0, 4, size=n).astype(np.float64)  # 4 distinct values: long tie runs
    ref = ko.find_top_edges(A, c, num, order)
    # one edge stored as explicit zeros in both triangles: find() skips it
    Z = A.copy()
    Z.data = Z.data.copy()
    rows = Z.indices
    cols = np.repeat(np.arange(n), np.diff(Z.indptr))
    k = int(np.flatnonzero(rows > cols)[0])
    i0, j0 = int(rows[k]), int(cols[k])
    Z.data[k] = 0.0
    Z.data[int(np.flatnonzero((rows == j0) & (cols == i0))[0])] = 0.0
    Ze = Z.copy()
    Ze.eliminate_zeros()
    num_z = min(num, sp.tril(Ze, -1).nnz)
    ref_z = ko.find_top_edges(Ze, c, num_z, order)
    U = A.copy()  # reversed (unsorted) row indices within each column
    for k in range(n):
        a, b = U.indptr[k], U.indptr[k + 1]
        U.indices[a:b] = U.indices[a:b][::-1].copy()
        U.data[a:b] = U.data[a:b][::-1].copy()
    U.has_sorted_indices = False
    for X in (A, U, A.tocsr(), A.toarray()):
        np.testing.assert_array_equal(kra.find_top_edges(X, c, num, order), ref)
    assert Z.nnz == A.nnz  # the zeros are stored
    np.testing.assert_array_equal(kra.find_top_edges(Z, c, num_z, order), ref_z)


def test_stable_head_matches_full_sort():
    """greedy._stable_head == argsort(kind="stable")[:num], NaN keys included."""
    from krylov_robustness_amd.greedy import _stable_head
    rng = np.random.default_rng(3)
    for trial in range(20):
        key = rng.integers(0, 5, size=50).astype(np.float64)
        if trial % 4 == 0:
            key[rng.integers(0, 50, size=30)] = np.nan
        for num in (1, 7, 25, 49, 50):
            np.testing.assert_array_equal(_stable_head(key, num), np.argsort(key, kind="stable")[:num])


def test_greedy_symmetry_check():
    """greedy_krylov.m:27-29's issymmetric: the CSR == CSC fast path and the
    elementwise fallback (explicit zeros, unsorted indices) agree with A == A'."""
    import scipy.sparse as sp
    from krylov_robustness_amd.greedy import _is_symmetric
    A = sp.csc_matrix(load_graph("india"))
    assert _is_symmetric(A)
    B = A.tolil()
    B[0, 1] = 2.0
    B[1, 0] = 2.0
    assert _is_symmetric(sp.csc_matrix(B))
    B[0, 2] = 3.0  # one triangle only
    assert not _is_symmetric(sp.csc_matrix(B))
    W = A.copy()  # weights that differ across the diagonal
    W.data = W.data.copy()
    W.data[0] = 5.0
    assert not _is_symmetric(W)
    Z = sp.csc_matrix((np.r_[A.data, 0.0], (np.r_[A.tocoo().row, 0], np.r_[A.tocoo().col, 5])), shape=A.shape)
    assert _is_symmetric(Z)  # an explicit zero in one triangle is still A == A'


def test_find_top_edges_too_few():
    A = load_graph("denmark")
    with pytest.raises(IndexError):
        kra.find_top_edges(A, np.ones(A.shape[0]), A.nnz, "min")


@pytest.mark.parametrize("name", ["india", "rome", "austria"])
def test_find_top_missing_edges_min(name):
    A = load_graph(name)
    c = kra.compute_centrality(A)
    E = kra.find_top_missing_edges(A, c, 80, "min")
    np.testing.assert_array_equal(E, ko.find_top_missing_edges_min(A, c, 80))
    assert all(A[i - 1, j - 1] == 0 and i != j for i, j in E)


def test_find_top_missing_edges_mult_are_missing():
    A = load_graph("austria")
    c = kra.compute_centrality(A)
    E = kra.find_top_missing_edges(A, c, 40, "mult")
    assert len(E) == 40
    assert all(A[i - 1, j - 1] == 0 and i != j for i, j in E)
    s = c[E[:, 0] - 1] * c[E[:, 1] - 1]
    assert np.all(np.diff(s) <= 1e-15)            # descending products


def test_edge2low_rank_matches_edit():
    """edge2low_rank.m:1-13: A + U B U' removes (value -1) / adds (+1) the
    edges, U selects the distinct nodes in ascending order."""
    import scipy.sparse as sp
    from conftest import load_graph
    from krylov_robustness_amd.greedy import edge2low_rank
    A = load_graph("anaheim").tocsr()
    n = A.shape[0]
    I, J = sp.triu(A, 1).nonzero()
    E = np.stack([I[[3, 7, 11]] + 1, J[[3, 7, 11]] + 1], axis=1)
    U, B = edge2low_rank(E, n)
    assert U.shape == (n, len(np.unique(E)))
    assert np.array_equal(sp.find(U)[0], np.unique(E) - 1)
    Ud = U.toarray()
    R = A.toarray() + Ud @ B @ Ud.T
    for i, j in E:
        assert R[i - 1, j - 1] == 0 and R[j - 1, i - 1] == 0
    assert abs(R - R.T).max() == 0
    assert (A.toarray() - R).sum() == 2 * len(E)
    U2, B2 = edge2low_rank(E, n, value=1.0)
    assert np.array_equal(B2, -B)
    # shared endpoint: node appears once in U
    U3, B3 = edge2low_rank([[1, 2], [2, 3]], 5)
    assert U3.shape == (5, 3) and B3[0, 1] == -1 and B3[1, 2] == -1 and B3[0, 2] == 0


def test_find_top_edges_duplicate_entries_summed():
    """A CSC input with duplicate entries: MATLAB sparse sums them, so does the
    ranking (an edge stored as +1 and -1 is absent; one stored as 0.5 + 0.5 is
    present once) -- the same as the canonical matrix."""
    import scipy.sparse as sp
    A = sp.csc_matrix(load_graph("india"))
    n = A.shape[0]
    C = A.tocoo()
    lower = np.flatnonzero(C.row > C.col)
    e0, e1 = lower[0], lower[5]
    i0, j0, i1, j1 = C.row[e0], C.col[e0], C.row[e1], C.col[e1]
    extra_r = np.array([i0, j0, i1, j1])
    extra_c = np.array([j0, i0, j1, i1])
    extra_v = np.array([-1.0, -1.0, 0.0, 0.0])
    Dup = sp.coo_matrix((np.concatenate([C.data, extra_v]),
                         (np.concatenate([C.row, extra_r]), np.concatenate([C.col, extra_c]))),
                        shape=(n, n))
    # a CSC whose column arrays carry the duplicates explicitly
    order = np.lexsort((Dup.row, Dup.col))
    rows, cols, vals = Dup.row[order], Dup.col[order], Dup.data[order]
    indptr = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(np.bincount(cols, minlength=n), out=indptr[1:])
    X = sp.csc_matrix((vals, rows, indptr), shape=(n, n))
    assert X.nnz == A.nnz + 4 and not X.has_canonical_format
    canon = X.copy()
    canon.sum_duplicates()
    canon.eliminate_zeros()
    c = kra.compute_centrality(A)
    for order in ("mult", "min"):
        ref = ko.find_top_edges(canon, c, 60, order)
        np.testing.assert_array_equal(kra.find_top_edges(X, c, 60, order), ref)
        np.testing.assert_array_equal(ko.find_top_edges(X, c, 60, order), ref)
        assert not np.any((ref[:, 0] == i0 + 1) & (ref[:, 1] == j0 + 1))  # summed to 0


def test_find_top_edges_fractional_count():
    """find_top_edges.m:19-21 with num = Q + k fractional (a weighted graph's
    Q = max(sum(A, 1))): fewer than num edges only warns; E(ind(1:num), :)
    takes floor(num) and fails only when even those are missing."""
    A = load_graph("denmark")
    c = kra.compute_centrality(A)
    ne = A.nnz // 2
    with pytest.warns(UserWarning, match="FIND_TOP_EDGES"):
        E = kra.find_top_edges(A, c, ne + 0.5, "mult")
    assert len(E) == ne
    with pytest.warns(UserWarning):
        np.testing.assert_array_equal(E, ko.find_top_edges(A, c, ne + 0.5, "mult"))
    with pytest.raises(IndexError), pytest.warns(UserWarning):
        kra.find_top_edges(A, c, ne + 1.5, "mult")
    np.testing.assert_array_equal(kra.find_top_edges(A, c, 10.7, "min"), ko.find_top_edges(A, c, 10, "min"))

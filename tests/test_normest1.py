"""CPU: the normest1 (t = 1) restatement behind normAm.m:25-26 -- the branch
select_taylor_degree takes when t (A - mu I) has negative entries (a graph
with self loops after expmv's shift, or signed weights).  MATLAB's normest1
is closed: the restatement follows the published
Higham-Tisseur Algorithm 2.4, checked here against SciPy's implementation of
the same algorithm (scipy.sparse.linalg.onenormest, t = 1) and against the
exact 1-norm it must not exceed; expmv through this branch is pinned to the
dense expm."""
import numpy as np
import pytest
import scipy.linalg as sla
import scipy.sparse as sp
from scipy.sparse.linalg import LinearOperator, onenormest

from conftest import load_graph
from oracle import krylov_oracle as ko


def signed_graph(n=200, seed=0):
    """Symmetric sparse matrix with mixed-sign continuous weights (no ties)."""
    rng = np.random.default_rng(seed)
    M = sp.random(n, n, density=0.03, random_state=seed, data_rvs=lambda k: rng.normal(size=k))
    return sp.csr_matrix(M + M.T)


def looped(A, every=7, w=2.0):
    """A with self loops of weight w on every `every`-th node: after the shift
    mu = trace/n the other diagonals are -mu < 0 (normest1 branch)."""
    d = np.zeros(A.shape[0])
    d[::every] = w
    return sp.csr_matrix(A + sp.diags(d))


def _power_ops(B, m):
    def mv(x):
        for _ in range(m):
            x = B @ x
        return x

    def rmv(x):
        for _ in range(m):
            x = B.T @ x
        return x
    return mv, rmv


@pytest.mark.parametrize("seed", [0, 1, 2])
@pytest.mark.parametrize("m", [1, 2, 4])
def test_normest1_matches_scipy_algorithm(seed, m):
    B = signed_graph(seed=seed)
    n = B.shape[0]
    mv, rmv = _power_ops(B, m)
    est, it1, it2 = ko.normest1_t1(mv, rmv, n)
    op = LinearOperator((n, n), matvec=mv, rmatvec=rmv, dtype=np.float64)
    ref = onenormest(op, t=1, itmax=5)
    assert est == pytest.approx(ref, rel=1e-12)
    exact = np.abs(np.linalg.matrix_power(B.toarray(), m)).sum(axis=0).max()
    assert est <= exact * (1 + 1e-12)
    assert est >= 0.3 * exact        # the estimator is typically within a small factor
    assert 1 <= it2 <= 5 and it1 in (it2, it2 + 1)


def test_normest1_small_n_is_exact():
    B = sp.csr_matrix(np.array([[0.0, -2.0, 1.0], [-2.0, 1.0, 0.5], [1.0, 0.5, -3.0]]))
    mv, rmv = _power_ops(B, 3)
    est, _, it2 = ko.normest1_t1(mv, rmv, 3)
    assert est == pytest.approx(np.abs(np.linalg.matrix_power(B.toarray(), 3)).sum(0).max(), rel=1e-14)
    assert it2 == 0


def test_normAm_nonnegative_is_exact_and_counts_m():
    A = load_graph("anaheim")
    c, mv = ko.normAm(A, 3)
    assert c == pytest.approx(np.abs(np.linalg.matrix_power(A.toarray(), 3)).sum(0).max(), rel=1e-14)
    assert mv == 3


@pytest.mark.parametrize("kind", ["loops", "signed"])
def test_expmv_normest1_branch_matches_dense(kind):
    A = looped(load_graph("oregon_A0")) if kind == "loops" else 4.0 * signed_graph(300, seed=5)
    b = np.random.default_rng(1).normal(size=(A.shape[0], 3))
    mu = A.diagonal().sum() / A.shape[0]
    C = A - mu * sp.eye(A.shape[0])
    assert C.min() < 0  # normAm takes the normest1 branch
    M, mvd, alpha, unA = ko.select_taylor_degree(A - mu * sp.eye(A.shape[0], format="csr"), b)
    assert unA == 0 and mvd > 0
    f, s, m, mv = ko.expmv(1.0, A, b)
    ref = sla.expm(A.toarray()) @ b
    # ||A||_1 ~ 200: dense expm's own error is ~1e-11 of the largest entry
    assert np.max(np.abs(f - ref)) / np.max(np.abs(ref)) < 1e-10

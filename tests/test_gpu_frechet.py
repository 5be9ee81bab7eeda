"""GPU parity for multiple_frechet_eval / hessianfcn_{exp,fun} (SURVEY.md §8f
next #3) against the oracle restatement (expm of the 2j x 2j block matrix,
as the reference) and the exact dense Frechet derivative.  Tolerance 1e-9
relative to the largest entry: the device forms the (1,2) block through the
Daleckii-Krein divided differences of the symmetric projections (equal to
the block expm up to rounding); iteration counts must match."""
import numpy as np
import pytest
import scipy.sparse as sp

from conftest import load_graph
from oracle import krylov_oracle as ko

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def kra():
    import krylov_robustness_amd as kra
    return kra


def _omega(A, m, seed):
    S = sp.triu(A, 1).tocoo()
    idx = np.random.default_rng(seed).choice(S.nnz, m, replace=False)
    return np.stack([S.row[idx] + 1, S.col[idx] + 1], axis=1)


def _oracle_entries(A, om, tg, f, tol, it):
    Um, Xm, Vm, row, col, iters = ko.multiple_frechet_eval(A, om, f, tol, it)
    out = np.zeros((len(om), len(tg)))
    for h, (i, j) in enumerate(om):
        a, b = Xm[h].shape
        for t, (p, q) in enumerate(tg):
            out[h, t] = Um[row[i]][p - 1, :a] @ Xm[h] @ Vm[col[j]][q - 1, :b]
    return out, iters


@pytest.mark.parametrize("name", ["austria", "rome", "india"])
@pytest.mark.parametrize("f", ["exp", "cosh", "sinh"])
def test_frechet_entries_match_oracle(kra, gpu_ctx, name, f):
    A = load_graph(name)
    om = _omega(A, 8, 3)
    tg = np.vstack([om, om[:, ::-1], [[om[0, 0], om[0, 0]]]])
    out, it = kra.frechet_entries(A, om, tg, f, 1e-10, 100, ctx=gpu_ctx)
    ref, ito = _oracle_entries(A, om, tg, f, 1e-10, 100)
    assert it == ito
    np.testing.assert_allclose(out, ref, rtol=0, atol=1e-9 * np.abs(ref).max())


def test_frechet_exact_small(kra, gpu_ctx):
    A = load_graph("austria")
    om = _omega(A, 4, 5)
    tg = np.array([[p, q] for p in (1, 7, 30) for q in (2, 99, 140)])
    out, _ = kra.frechet_entries(A, om, tg, "exp", 1e-13, 100, ctx=gpu_ctx)
    for h, (i, j) in enumerate(om):
        D = ko.exact_frechet(A, i, j, "exp")
        ex = np.array([D[p - 1, q - 1] for p, q in tg])
        np.testing.assert_allclose(out[h], ex, rtol=0, atol=1e-10 * np.abs(D).max())


@pytest.mark.parametrize("name,f", [("austria", "exp"), ("rome", "exp"), ("india", "cosh"),
                                    ("india", "sinh")])
def test_hessianfcn_matches_oracle(kra, gpu_ctx, name, f):
    A = load_graph(name)
    om = _omega(A, 10, 7)
    w = np.array([A[i - 1, j - 1] for i, j in om])
    X = np.random.default_rng(2).uniform(-0.5, 1.0, size=len(om)) * w
    H = kra.hessianfcn(X, A, om, f, 1e-10, 100, ctx=gpu_ctx)
    Ho = ko.hessianfcn(X, A, om, f, 1e-10, 100)
    np.testing.assert_allclose(H, Ho, rtol=0, atol=1e-9 * np.abs(Ho).max())
    np.testing.assert_array_equal(H, H.T)


def test_hessian_exp_exact_small(kra, gpu_ctx):
    """hessianfcn_exp vs -2 Df(A + XX + XX')(e_i e_j')(p, q) from dense expm."""
    A = load_graph("austria")
    om = _omega(A, 5, 9)
    X = np.linspace(-0.4, 0.6, 5)
    H = kra.hessianfcn_exp(X, A, om, 1e-13, 100, ctx=gpu_ctx)
    n = A.shape[0]
    XX = sp.csr_matrix((X, (om[:, 0] - 1, om[:, 1] - 1)), shape=(n, n))
    At = A + XX + XX.T
    He = np.zeros((5, 5))
    for j in range(5):
        D = ko.exact_frechet(At, om[j, 0], om[j, 1], "exp")
        for l in range(5):
            He[j, l] = -2 * D[om[l, 0] - 1, om[l, 1] - 1]
    np.testing.assert_allclose(H, He, rtol=0, atol=1e-10 * np.abs(He).max())

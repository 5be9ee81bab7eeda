"""GPU parity for function_multiple_entries: the
device's column-batched Arnoldi vs the oracle restatement on the same
omega.  Tolerance 1e-9 relative to max |X| (the device evaluates f(Gm) e1 by
a symmetric eigendecomposition of the Arnoldi projection, the oracle by
expm/funm of the Hessenberg matrix as MATLAB does; they agree to rounding),
identical iteration counts, and exact dense f(A) entries on small graphs."""
import numpy as np
import pytest
import scipy.linalg as sla

from conftest import load_graph
from oracle import krylov_oracle as ko

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def kra():
    import krylov_robustness_amd as kra
    return kra


def _omega(A, m, seed):
    S = A.tocoo()
    idx = np.random.default_rng(seed).choice(S.nnz, m, replace=False)
    om = np.stack([S.row[idx] + 1, S.col[idx] + 1], axis=1)
    return np.vstack([om, [[om[0, 0], om[0, 0]]]])


@pytest.mark.parametrize("name", ["austria", "rome", "india"])
@pytest.mark.parametrize("f", ["exp", "cosh", "sinh"])
def test_fme_matches_oracle(kra, gpu_ctx, name, f):
    A = load_graph(name)
    om = _omega(A, 24, 1)
    tol = 1e-10
    X, it = kra.function_multiple_entries(kra.DeviceMatrix(A, gpu_ctx), om, f, tol, 100, ctx=gpu_ctx)
    Xo, ito = ko.function_multiple_entries(A, om, f, tol, 100)
    assert it == ito
    np.testing.assert_allclose(X, Xo, rtol=1e-9, atol=1e-9 * np.abs(Xo).max())


def test_fme_exact_small(kra, gpu_ctx):
    A = load_graph("austria")
    om = _omega(A, 30, 2)
    X, _ = kra.function_multiple_entries(A, om, "exp", 1e-13, 100, ctx=gpu_ctx)
    E = sla.expm(A.toarray())
    ex = np.array([E[i - 1, j - 1] for i, j in om])
    np.testing.assert_allclose(X, ex, rtol=1e-10, atol=1e-12 * np.abs(ex).max())


def test_fme_two_column_groups(kra, gpu_ctx):
    """> 128 distinct row indices: two device groups, shared rows, repeated
    entries and shuffled order."""
    A = load_graph("rome")
    S = A.tocoo()
    rng = np.random.default_rng(5)
    idx = rng.choice(S.nnz, 150, replace=False)
    om = np.stack([S.row[idx] + 1, S.col[idx] + 1], axis=1)
    om = np.vstack([om, om[:7], om[3:9, ::-1]])
    X, it = kra.function_multiple_entries(A, om, "exp", 1e-8, 60, ctx=gpu_ctx)
    Xo, ito = ko.function_multiple_entries(A, om, "exp", 1e-8, 60)
    assert it == ito
    np.testing.assert_allclose(X, Xo, rtol=1e-9, atol=1e-9 * np.abs(Xo).max())
    np.testing.assert_array_equal(X[150:157], X[:7])


def test_fme_rejects_rational_poles(kra, gpu_ctx):
    A = load_graph("austria")
    with pytest.raises(kra.KrylovError, match="rational"):
        kra.function_multiple_entries(A, [[1, 2]], "exp", 1e-8, 10, poles=[1.0], ctx=gpu_ctx)


def test_maxit_warnings_stay_warnings(kra, gpu_ctx):
    """The reference's 'Reached maximum number of iterations' warnings
    (function_multiple_entries.m:158-161, trace_fun_update.m:128-130) are
    warnings, not errors, and the results are still returned."""
    A = load_graph("rome")
    with pytest.warns(UserWarning, match="FUNCTION_MULTIPLE_ENTRIES:: Reached maximum"):
        X, it = kra.function_multiple_entries(A, [[1, 2], [5, 5]], "exp", 1e-30, 4, ctx=gpu_ctx)
    assert it == 4 and np.all(np.isfinite(X))
    U = np.zeros((A.shape[0], 2)); U[0, 0] = 1; U[1, 1] = 1
    with pytest.warns(UserWarning, match="TRACE_FUN_UPDATE:: Reached maximum"):
        xm, it, _ = kra.trace_fun_update(A, U, -np.array([[0, 1.0], [1.0, 0]]), 1e-30, 5, ctx=gpu_ctx)
    assert it == 5 and np.isfinite(xm)

"""Device Householder thin QR (kt_tsqr.hip) against LAPACK's dgeqrf/dorgqr
(numpy.linalg.qr, the factorisation MATLAB's qr(w, 0) calls): same signs,
same Q, same R to rounding -- including exactly dependent and zero columns,
where the completion is fixed by dlarfg's tau = 0 branch."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def kra():
    import krylov_robustness_amd as kra
    return kra


@pytest.mark.parametrize("n,bs", [(200, 1), (1000, 2), (5000, 10), (3000, 45), (20000, 64),
                                  (4096, 128), (300, 7)])
def test_qr_matches_lapack(kra, gpu_ctx, n, bs):
    W = np.random.default_rng(n + bs).normal(size=(n, bs))
    Q, R = kra.householder_qr(W, ctx=gpu_ctx)
    Qr, Rr = np.linalg.qr(W)
    np.testing.assert_allclose(R, Rr, rtol=0, atol=1e-12 * np.abs(Rr).max())
    np.testing.assert_allclose(Q, Qr, rtol=0, atol=1e-12)


def test_qr_rank_deficient_completion(kra, gpu_ctx):
    """Exactly zero columns (dlarfg's tau = 0 completion, the leaf-edge case of
    the greedy path) and unit selectors (krylov_miobi's U)."""
    n = 500
    rng = np.random.default_rng(3)
    W = np.zeros((n, 6))
    W[:, 0] = rng.normal(size=n)
    W[:, 2] = 0.0                       # zero column after a dense one
    W[7, 3] = 1.0                       # unit selector
    W[:, 4] = 0.0                       # zero column
    W[123, 5] = -1.0
    Q, R = kra.householder_qr(W, ctx=gpu_ctx)
    Qr, Rr = np.linalg.qr(W)
    np.testing.assert_allclose(R, Rr, rtol=0, atol=1e-12 * np.abs(Rr).max())
    np.testing.assert_allclose(Q, Qr, rtol=0, atol=1e-12)
    np.testing.assert_allclose(Q.T @ Q, np.eye(6), atol=1e-13)

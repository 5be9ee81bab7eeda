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


@pytest.mark.parametrize("n,bs", [(3000, 45), (21774, 25), (10860, 10), (200_000, 16)])
def test_qr_two_launch_form_rank_deficient(kra, gpu_ctx, monkeypatch, n, bs):
    """The two-launch reflector sweep (the default) on a rank-deficient block
    (half the columns repeat earlier ones, as in power-grid Krylov blocks, and
    a zero column): Q orthonormal, Q R = W; on a full-rank block Q and R equal
    LAPACK's."""
    rng = np.random.default_rng(n + 7 * bs)
    W = rng.normal(size=(n, bs))
    W[:, bs // 2:] = W[:, :bs - bs // 2] if bs > 1 else W[:, bs // 2:]
    W[:, -1] = 0.0
    monkeypatch.setenv("KT_TSQR_STEP1", "0")
    Q2, R2 = kra.householder_qr(W, ctx=gpu_ctx)
    np.testing.assert_allclose(Q2.T @ Q2, np.eye(bs), atol=1e-12)
    np.testing.assert_allclose(Q2 @ R2, W, rtol=0, atol=1e-12 * np.abs(W).max())
    Wr = rng.normal(size=(n, bs))
    Qp, Rp = kra.householder_qr(Wr, ctx=gpu_ctx)
    Qr, Rr = np.linalg.qr(Wr)
    np.testing.assert_allclose(Rp, Rr, rtol=0, atol=1e-12 * np.abs(Rr).max())
    np.testing.assert_allclose(Qp, Qr, rtol=0, atol=1e-11)


@pytest.mark.parametrize("form", [("KT_TSQR_STEP1", "1")])
@pytest.mark.parametrize("n,bs", [(3000, 45), (21774, 25), (10860, 10), (3228, 29)])
def test_qr_one_launch_per_column_form(kra, gpu_ctx, monkeypatch, n, bs, form):
    """The one-launch-per-column sweep (KT_TSQR_STEP1=1, k_ts_step1: every
    workgroup sums the previous launch's partials itself) groups the
    reductions by workgroup instead of by 64-row block: on a full-rank block Q and R equal
    the two-launch form's and LAPACK's to rounding; on a rank-deficient one
    (repeated columns, a zero column) R agrees to rounding and Q is
    orthonormal with Q R = W -- the completion directions of the deficient
    columns are rounding-dependent in every implementation, LAPACK's included."""
    rng = np.random.default_rng(n + 3 * bs)
    Wr = rng.normal(size=(n, bs))
    monkeypatch.setenv(*form)
    Q1, R1 = kra.householder_qr(Wr, ctx=gpu_ctx)
    monkeypatch.delenv(form[0])
    Q2, R2 = kra.householder_qr(Wr, ctx=gpu_ctx)
    Qr, Rr = np.linalg.qr(Wr)
    np.testing.assert_allclose(R1, R2, rtol=0, atol=1e-13 * np.abs(R2).max())
    np.testing.assert_allclose(Q1, Q2, rtol=0, atol=1e-13)
    np.testing.assert_allclose(R1, Rr, rtol=0, atol=1e-12 * np.abs(Rr).max())
    np.testing.assert_allclose(Q1, Qr, rtol=0, atol=1e-12)
    monkeypatch.setenv(*form)
    W = Wr.copy()
    W[:, bs // 2:] = W[:, :bs - bs // 2]
    W[:, -1] = 0.0
    Q1, R1 = kra.householder_qr(W, ctx=gpu_ctx)
    monkeypatch.delenv(form[0])
    Q2, R2 = kra.householder_qr(W, ctx=gpu_ctx)
    np.testing.assert_allclose(np.abs(R1), np.abs(R2), rtol=0, atol=1e-12 * np.abs(R2).max())
    np.testing.assert_allclose(Q1.T @ Q1, np.eye(bs), atol=1e-12)
    np.testing.assert_allclose(Q1 @ R1, W, rtol=0, atol=1e-12 * np.abs(W).max())

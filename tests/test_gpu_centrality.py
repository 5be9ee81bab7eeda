"""compute_centrality(A, 'eig') on the device (compute_centrality.m:15-17,
eigs(A, 1)) vs scipy's ARPACK eigsh: leading eigenvalue and |u| agree."""
import numpy as np
import pytest
import scipy.sparse.linalg as sla

from conftest import load_graph

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def kra():
    import krylov_robustness_amd as kra
    return kra


@pytest.mark.parametrize("name", ["austria", "rome", "india", "oregon_A6", "hawaii"])
def test_eigs_leading_matches_arpack(kra, gpu_ctx, name):
    A = load_graph(name)
    lam, u = kra.eigs_leading(kra.DeviceMatrix(A, gpu_ctx), ctx=gpu_ctx)
    w, V = sla.eigsh(A, k=1, which="LA", tol=1e-14)
    assert lam == pytest.approx(w[0], rel=1e-12)
    np.testing.assert_allclose(np.abs(u), np.abs(V[:, 0]), atol=1e-9)
    assert np.linalg.norm(u) == pytest.approx(1.0, rel=1e-13)


def test_device_centrality_drives_greedy(kra, gpu_ctx):
    """greedy_krylov without a centrality argument ranks edges by the device
    eigenvector and selects the same edges as with the host one."""
    A = load_graph("india")
    c_host = kra.compute_centrality(A)
    c_dev = kra.compute_centrality(kra.DeviceMatrix(A, gpu_ctx), ctx=gpu_ctx)
    np.testing.assert_allclose(c_dev, c_host, atol=1e-9)
    e1, r1, _ = kra.greedy_krylov(kra.DeviceMatrix(A, gpu_ctx), 3, 40, None, "min", 1e-6, 100, ctx=gpu_ctx)
    e2, r2, _ = kra.greedy_krylov(kra.DeviceMatrix(A, gpu_ctx), 3, 40, c_host, "min", 1e-6, 100, ctx=gpu_ctx)
    np.testing.assert_array_equal(e1, e2)
    assert r1 == pytest.approx(r2, rel=1e-12)

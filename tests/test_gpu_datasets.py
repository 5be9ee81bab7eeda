"""GPU runs on the reference's MAT v7.3 datasets:
CollegeMsg, Drugs and as_735 prepared as test_unweighted_make.m:41-52 and
committed as tests/golden/v73_graphs.npz.

Tolerances: trace_exp against the exact dense spectrum 1e-3 relative (Monte
Carlo estimator stopped at tol 1e-4; these spectra are dominated by
exp(lambda_1) so the oracle lands within 6e-6); SLQ quadratic forms against
the oracle on the same seeds 1e-10 relative; greedy_krylov 'make' selection
exact, its robustness variation 1e-7 relative (lag-2 stopping, see
test_gpu_greedy.py)."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, load_v73_graph
from oracle import krylov_oracle as ko

pytestmark = pytest.mark.gpu
NAMES = ["drugs", "as_735", "collegemsg"]


@pytest.fixture(scope="module")
def kra():
    import krylov_robustness_amd as kra
    return kra


@pytest.fixture(scope="module")
def vals():
    with open(os.path.join(GOLDEN, "v73_values.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("name", NAMES)
def test_trace_exp_exact(kra, gpu_ctx, vals, name):
    A = load_v73_graph(name)
    tr = kra.trace_exp(kra.DeviceMatrix(A, gpu_ctx), method="lanczos", m=30, seed=0, ctx=gpu_ctx)
    assert tr == pytest.approx(vals[name]["exact_tr_exp"], rel=1e-3)


@pytest.mark.parametrize("name", NAMES)
def test_slq_quadforms_vs_oracle(kra, gpu_ctx, name):
    A = load_v73_graph(name)
    D = kra.DeviceMatrix(A, gpu_ctx)
    for fun in ("exp", "sinh"):
        q = kra.slq_quadforms(D, 16, 30, seed=7, fun=fun, ctx=gpu_ctx)[2]
        _, qo = ko.slq_trace(A, 16, 30, seed=7, fun=fun)
        np.testing.assert_allclose(q, qo, rtol=1e-10, atol=0)


def test_greedy_make_collegemsg(kra, gpu_ctx, vals):
    A = load_v73_graph("collegemsg")
    g = vals["collegemsg"]["oracle_greedy_make"]
    w, V = np.linalg.eigh(A.toarray())
    cen = np.abs(V[:, -1])
    edges, rob, _ = kra.greedy_krylov(kra.DeviceMatrix(A, gpu_ctx), g["k"], g["Q"], cen, g["order"],
                                      g["tol"], g["it"], miobi="make", ctx=gpu_ctx)
    assert np.asarray(edges).tolist() == g["edges"]
    assert rob == pytest.approx(g["rob"], rel=1e-7)


def test_device_centrality_as_735(kra, gpu_ctx):
    """compute_centrality(A, 'eig') on the device against a dense eigh."""
    A = load_v73_graph("as_735")
    c = kra.compute_centrality(kra.DeviceMatrix(A, gpu_ctx), "eig", ctx=gpu_ctx)
    w, V = np.linalg.eigh(A.toarray())
    np.testing.assert_allclose(c, np.abs(V[:, -1]), rtol=0, atol=1e-8)


def test_selected_edges_delta_trace(kra, gpu_ctx, vals):
    """The drivers' check of a selected edge set (test_unweighted_make.m:92-93):
    [U, B] = edge2low_rank(edges, n) (+1: the make drivers' copy, :171-183),
    delta = trace_fun_update(A, full(U), B, tol*nrm) -- against the exact
    tr exp(A + U B U') - tr exp(A) from dense spectra.  tol*nrm = 1e-6 e^48
    on a difference of ~1e20: 1e-5 relative."""
    A = load_v73_graph("collegemsg")
    g = vals["collegemsg"]["oracle_greedy_make"]
    E = np.array(g["edges"])
    U, B = kra.edge2low_rank(E, A.shape[0], value=1.0)
    D = kra.DeviceMatrix(A, gpu_ctx)
    xm, it, lucky = kra.trace_fun_update(D, U, B, g["tol"], 100, ctx=gpu_ctx)
    Ad = A.toarray()
    Ud = U.toarray()
    exact = (np.exp(np.linalg.eigvalsh(Ad + Ud @ B @ Ud.T)).sum()
             - np.exp(np.linalg.eigvalsh(Ad)).sum())
    assert xm == pytest.approx(exact, rel=1e-5)

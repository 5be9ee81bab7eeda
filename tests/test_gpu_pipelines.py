"""GPU: the pipelined drivers equal their serial loops BIT FOR BIT.

fun_update, trace_fun_update, function_multiple_entries and the Frechet
entries overlap step j's host work (projections, eigenproblems, the stop
test) with the device's step j + 1, launched speculatively before step j's
stop decision is known; the fun_update stop test may also decide from power
bounds on ||Xm - Xstop||_2 instead of an eigenvalue solve when the projected
size is >= 96 (kt_krylov.cpp sym_norm2_power_bounds).  Each switch has an
environment variable read per call that restores the serial form
(KT_FU_PIPE, KT_TFU_PIPE, KT_FME_PIPE, KT_FRECHET_PIPE, KT_NORM_POW = 0).  The
cases stop mid-run, hit a lucky breakdown (lanczos_krylov.m:91-93 /
arnoldi_krylov.m:79, complete graph K_200: the block Krylov space of an edge
has dimension 3), reach the iteration cap, and take fun_update's dense
fallback at n/2 basis columns (fun_update.m:85-90); every output (Xm, iter,
lucky, Um, f, gr, entries) must be identical with and without the pipeline."""
import warnings

import numpy as np
import pytest
import scipy.sparse as sp

from conftest import load_graph

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def kra():
    import krylov_robustness_amd as kra
    return kra


def _edge(n, i, j):
    U = np.zeros((n, 2))
    U[i, 0] = U[j, 1] = 1.0
    return U, -np.array([[0.0, 1.0], [1.0, 0.0]])


def _complete(n):
    return sp.csr_matrix(np.ones((n, n)) - np.eye(n))


def _both(monkeypatch, var, fn):
    """fn() with the switch at its default and at 0 (serial)."""
    monkeypatch.delenv(var, raising=False)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        a = fn()
        monkeypatch.setenv(var, "0")
        b = fn()
    monkeypatch.delenv(var, raising=False)
    return a, b


def _same(a, b):
    if isinstance(a, (tuple, list)):
        assert len(a) == len(b)
        for x, y in zip(a, b):
            _same(x, y)
    elif isinstance(a, np.ndarray) or isinstance(b, np.ndarray):
        assert (a is None) == (b is None)
        assert np.array_equal(np.asarray(a), np.asarray(b))
    else:
        assert a == b


CASES = {  # name -> (graph, edge, tol, it)
    "stops": (lambda: load_graph("india"), (11, 40), 1e-10, 100),
    "maxit": (lambda: load_graph("india"), (11, 40), 1e-300, 7),
    "lucky": (lambda: _complete(200), (3, 77), 1e-14, 50),
}


@pytest.mark.parametrize("case", sorted(CASES))
def test_trace_fun_update_pipeline_bit_identical(kra, gpu_ctx, monkeypatch, case):
    mk, (i, j), tol, it = CASES[case]
    A = mk()
    D = kra.DeviceMatrix(A, gpu_ctx)
    L = sp.tril(A, -1).tocoo()
    U, B = _edge(A.shape[0], int(L.row[i]), int(L.col[i])) if case != "lucky" else _edge(A.shape[0], i, j)
    for fun in ("exp", "sinh"):
        a, b = _both(monkeypatch, "KT_TFU_PIPE", lambda: kra.trace_fun_update(D, U, B, tol, it, 0, fun,
                                                                                ctx=gpu_ctx))
        _same(a, b)
        if case == "lucky":
            assert a[2] == 1 and a[1] < 5
        if case == "maxit":
            assert a[1] == it


@pytest.mark.parametrize("case", sorted(CASES) + ["dense_fallback"])
def test_fun_update_pipeline_bit_identical(kra, gpu_ctx, monkeypatch, case):
    if case == "dense_fallback":
        A = load_graph("denmark")  # n = 96: the basis reaches n/2 = 48 columns
        L = sp.tril(A, -1).tocoo()
        U, B = _edge(A.shape[0], int(L.row[2]), int(L.col[2]))
        tol, it = 1e-300, 100
    else:
        mk, (i, j), tol, it = CASES[case]
        A = mk()
        L = sp.tril(A, -1).tocoo()
        U, B = _edge(A.shape[0], int(L.row[i]), int(L.col[i])) if case != "lucky" else _edge(A.shape[0], i, j)
    D = kra.DeviceMatrix(A, gpu_ctx)
    dense0 = gpu_ctx.stat(1)
    a, b = _both(monkeypatch, "KT_FU_PIPE", lambda: kra.fun_update(D, U, B, "exp", tol, it, ctx=gpu_ctx))
    _same(a, b)
    if case == "dense_fallback":
        assert gpu_ctx.stat(1) - dense0 == 2 and a[0].shape[0] == A.shape[0]
    if case == "lucky":
        assert a[2] == 1


def test_fun_update_norm_power_bounds_bit_identical(kra, gpu_ctx, monkeypatch):
    """Projected sizes >= 96 (kNormPowMin): the stop test decides from the
    normalised-squaring bounds where they are decisive; the result equals the
    eigenvalue-only decision (KT_NORM_POW=0)."""
    A = load_graph("rome")
    L = sp.tril(A, -1).tocoo()
    U, B = _edge(A.shape[0], int(L.row[20]), int(L.col[20]))
    sizes = []
    for tol, it in ((1e-13, 80), (1e-9, 80), (1e-300, 60)):
        a, b = _both(monkeypatch, "KT_NORM_POW", lambda: kra.fun_update(A, U, B, "exp", tol, it, ctx=gpu_ctx))
        _same(a, b)
        sizes.append(a[0].shape[0])
    assert max(sizes) >= 96  # the bounds were consulted


def test_fun_and_grad_pipelines_bit_identical(kra, gpu_ctx, monkeypatch):
    A = load_graph("india")
    D = kra.DeviceMatrix(A, gpu_ctx)
    L = sp.tril(A, -1).tocoo()
    idx = np.random.default_rng(1).choice(L.nnz, 20, replace=False)
    Om = np.stack([L.row[idx], L.col[idx]], axis=1).astype(np.float64) + 1
    X = np.random.default_rng(2).uniform(-0.4, 0.4, 20)
    dfA = np.random.default_rng(3).uniform(1, 2, 20)
    for var in ("KT_FU_PIPE", "KT_TFU_PIPE"):
        a, b = _both(monkeypatch, var, lambda: kra.fun_and_grad_krylov_exp(X, D, Om, dfA, 1e-8, 80, ctx=gpu_ctx))
        _same(a, b)
        a, b = _both(monkeypatch, var, lambda: kra.fun_and_grad_krylov_fun(X, D, Om, "sinh", "cosh", dfA, 1e-8, 80,
                                                                           ctx=gpu_ctx))
        _same(a, b)


@pytest.mark.parametrize("tol,it", [(1e-10, 100), (1e-300, 9)])
def test_fme_and_frechet_pipelines_bit_identical(kra, gpu_ctx, monkeypatch, tol, it):
    A = load_graph("austria")
    D = kra.DeviceMatrix(A, gpu_ctx)
    L = sp.tril(A, -1).tocoo()
    om = np.stack([L.row[:12], L.col[:12]], axis=1).astype(np.int64) + 1
    for f in ("exp", "cosh"):
        a, b = _both(monkeypatch, "KT_FME_PIPE", lambda: kra.function_multiple_entries(D, om, f, tol, it,
                                                                                       ctx=gpu_ctx))
        _same(a, b)
        if tol < 1e-100:
            assert a[1] == it
        tg = om[::-1][:5]
        a, b = _both(monkeypatch, "KT_FRECHET_PIPE", lambda: kra.frechet_entries(D, om[:6], tg, f, tol, it,
                                                                                 ctx=gpu_ctx))
        _same(a, b)
    X = np.random.default_rng(4).uniform(0.1, 0.3, 6)
    a, b = _both(monkeypatch, "KT_FRECHET_PIPE",
                 lambda: kra.hessianfcn_exp(X, D, om[:6].astype(np.float64), tol, it, ctx=gpu_ctx))
    _same(a, b)

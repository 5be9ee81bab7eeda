"""CPU: pin the oracle against the reference's known-answer identities and the
committed golden fixtures.  No GPU needed."""
import math

import numpy as np
import pytest
import scipy.linalg as sla
import scipy.sparse as sp

from conftest import GRAPHS, load_graph
from oracle import krylov_oracle as ko
from oracle import slq_ref


def test_rademacher_c_matches_numpy():
    lib = slq_ref.load()
    R = ko.rademacher(17, [0, 5, 123456789], seed=42)
    for c, p in enumerate([0, 5, 123456789]):
        for i in range(17):
            assert R[i, c] == lib.slq_ref_rademacher(42, p, i)
    assert set(np.unique(R)) <= {-1.0, 1.0}


def test_tridiag_quadrature_matches_dense():
    import ctypes as C
    rng = np.random.default_rng(0)
    for m in [1, 2, 5, 20, 30]:
        a = rng.normal(size=m) * 3
        e = rng.random(m - 1) + 0.1 if m > 1 else np.zeros(0)
        T = np.diag(a) + np.diag(e, 1) + np.diag(e, -1)
        ref = sla.expm(T)[0, 0]
        got = slq_ref.load().slq_ref_tridiag_quad(m, a.ctypes.data, e.ctypes.data, 0)
        assert got == pytest.approx(ref, rel=1e-12)
        assert ko.tridiag_quadrature(a, e, "exp") == pytest.approx(ref, rel=1e-12)


@pytest.mark.parametrize("name", GRAPHS)
def test_oracle_slq_matches_golden(name, values):
    rec = values[name]
    A = load_graph(name)
    assert A.shape[0] == rec["n"] and A.nnz == rec["nnz"]
    for fun in ["exp", "sinh"]:
        gold = np.array(rec[f"oracle_slq_{fun}_seed7_m20"])
        _, q_np = ko.slq_trace(A, 16, 20, seed=7, fun=fun)
        _, q_c = slq_ref.slq_trace(A, 16, 20, seed=7, fun=fun)
        np.testing.assert_allclose(q_np, gold, rtol=1e-12)
        np.testing.assert_allclose(q_c, gold, rtol=1e-9)


@pytest.mark.parametrize("name", ["denmark", "austria", "anaheim"])
def test_slq_hutchinson_unbiased_statistically(name, values):
    """Plain Hutchinson over many probes converges to exact sum(exp(eig(A)))
    (test_weighted_exp_lbfgs.m:41) within 5 standard errors."""
    A = load_graph(name)
    N = 4000
    mean, q = slq_ref.slq_trace(A, N, 20, seed=11, fun="exp")
    se = q.std(ddof=1) / math.sqrt(N)
    assert abs(mean - values[name]["exact_tr_exp"]) < 5 * se + 1e-9 * abs(mean)


@pytest.mark.parametrize("name", ["anaheim", "rome", "austria", "india"])
def test_trace_fun_update_pinned_to_exact(name, values):
    """trace_fun_update.m Lanczos path vs the debug==3 truth (:91-102)."""
    for c in values[name]["trace_fun_update_break"]:
        assert c["oracle"] == pytest.approx(c["exact"], rel=1e-9, abs=1e-9)


def test_trace_fun_update_dense_shortcut_exact():
    """n <= 130 takes the dense path (trace_fun_update.m:37-51) == exact."""
    A = load_graph("denmark")
    n = A.shape[0]
    U = np.zeros((n, 2)); U[3, 0] = 1; U[7, 1] = 1
    B = -np.array([[0.0, 1.0], [1.0, 0.0]])
    xm, it, lucky = ko.trace_fun_update(A, U, B)
    assert it == 0 and lucky == 0
    assert xm == pytest.approx(ko.exact_trace_update(A, U, B), rel=1e-13)
    xs, _, _ = ko.trace_fun_update(A, U, B, fun="sinh")
    assert xs == pytest.approx(ko.exact_trace_update(A, U, B, "sinh"), rel=1e-12)


def test_trace_fun_update_generic_handle_pinned():
    """A handle outside fun_update.m's list (trace_fun_update.m:88) in the
    oracle: the Lanczos path agrees with the exact update, and a callable
    equal to sinh gives fun='sinh'."""
    A = load_graph("rome")
    n = A.shape[0]
    U = np.zeros((n, 2)); U[5, 0] = 1; U[40, 1] = 1
    B = -np.array([[0.0, 1.0], [1.0, 0.0]])
    f = lambda x: np.tanh(x) + 0.1 * x ** 3  # noqa: E731
    xf, _, _ = ko.trace_fun_update(A, U, B, 1e-12, 100, 0, f)
    assert xf == pytest.approx(ko.exact_trace_update(A, U, B, f), rel=1e-9, abs=1e-10)
    xs, _, _ = ko.trace_fun_update(A, U, B, 1e-12, 100, 0, lambda x: np.sinh(x))
    xr, _, _ = ko.trace_fun_update(A, U, B, 1e-12, 100, 0, "sinh")
    assert xs == xr


def test_fun_update_arnoldi_vs_dense_expm():
    """fun_and_grad_krylov_exp.m:90-93 debug check: Um Xm Um' ~ expm(A+UBU') - expm(A)."""
    A = load_graph("austria")
    n = A.shape[0]
    U = np.zeros((n, 3)); U[0, 0] = 1; U[10, 1] = 1; U[40, 2] = 1
    B = np.array([[0.0, 0.3, 0.0], [0.3, 0.0, -0.2], [0.0, -0.2, 0.0]])
    Xm, it, lucky, Um = ko.fun_update(A, U, B, "exp", 1e-12, 100)
    XX = sla.expm(A.toarray() + U @ B @ U.T) - sla.expm(A.toarray())
    err = np.linalg.norm(XX - Um @ Xm @ Um.T) / np.linalg.norm(XX)
    assert err < 1e-9


def test_fun_and_grad_exp_frechet_identity():
    """fun_and_grad_krylov_exp.m:90-110: f = -tr(expm(A+D)-expm(A)); gradient
    entry k = -2 tr(L_f(A+D, E_ij)) from the block [A+D E;0 A+D]."""
    A = load_graph("denmark")
    n = A.shape[0]
    I, J = sp.triu(A, 1).nonzero()
    Omega = np.stack([I[:4] + 1, J[:4] + 1], axis=1)
    X = np.array([0.1, -0.05, 0.2, 0.0])
    eA = sla.expm(A.toarray())[Omega[:, 0] - 1, Omega[:, 1] - 1]
    f, gr = ko.fun_and_grad_krylov_exp(X, A, Omega, eA, 1e-12, 100)
    U, B = ko.lowrank_from_edges(X, Omega, n)
    AA = A.toarray() + U @ B @ U.T
    f2 = -np.trace(sla.expm(AA) - sla.expm(A.toarray()))
    assert f == pytest.approx(f2, rel=1e-9)
    gr2 = np.zeros(len(X))
    for k in range(len(X)):
        E = np.zeros((n, n)); E[Omega[k, 0] - 1, Omega[k, 1] - 1] = 1
        BB = np.block([[AA, E], [np.zeros((n, n)), AA]])
        gr2[k] = -2 * np.trace(sla.expm(BB)[:n, n:])
    assert np.linalg.norm(gr - gr2) / np.linalg.norm(gr2) < 1e-5   # reference threshold :106


def test_fun_and_grad_zero_fast_path():
    """X == 0 returns f = 0, gr = -2 eA with no Krylov work (fun_and_grad_krylov_exp.m:30-54)."""
    A = load_graph("denmark")
    Omega = np.array([[1, 2], [3, 4]])
    eA = np.array([0.5, 0.25])
    f, gr = ko.fun_and_grad_krylov_exp(np.zeros(2), A, Omega, eA, 1e-6, 100)
    assert f == 0 and np.array_equal(gr, -2 * eA)


def test_fun_and_grad_rejects_nonhermitian():
    A = sp.csr_matrix(np.array([[0.0, 1.0], [0.0, 0.0]]))
    with pytest.raises(ValueError, match="not Hermitian"):
        ko.fun_and_grad_krylov_exp(np.ones(1), A, np.array([[1, 2]]), np.zeros(1), 1e-6, 10)


def test_expmv_matches_dense():
    A = load_graph("anaheim")
    rng = np.random.default_rng(1)
    b = rng.normal(size=(A.shape[0], 3))
    f, s, m, mv = ko.expmv(1.0, A, b)
    ref = sla.expm(A.toarray()) @ b
    assert np.max(np.abs(f - ref)) / np.max(np.abs(ref)) < 1e-12


def test_trace_exp_reference_composition(values):
    """trace_exp.m: mc_trace(expmv, tol 1e-4, maxit 1000) vs exact."""
    A = load_graph("oregon_A0")
    tr = ko.trace_exp(A, seed=1)
    assert tr == pytest.approx(values["oregon_A0"]["exact_tr_exp"], rel=1e-4)


def test_mc_trace_defaults_one_round():
    """mc_trace.m:20-31,41: default maxit=10 -> K = ceil(10/30) = 1 round."""
    A = load_graph("denmark")
    tr, res, it = ko.mc_trace(A.toarray(), A.shape[0])
    assert it == 1 and res == 1.0
    # with a matrix Afun, trace(Q' A Q) + deflated G term estimates trace(A) = 0;
    # the G term's std is <= sqrt(2/10) ||A||_F (Hutchinson, Rademacher)
    assert abs(tr) < 5 * math.sqrt(2 / 10) * sp.linalg.norm(A)


def test_theta_table_matches_published_constants():
    """theta_taylor.mat (the reference's data file, read by
    select_taylor_degree.m:31) against the theta_m of Al-Mohy & Higham
    (2011), as SciPy's independent expm_multiply carries them (2-3
    significant digits): every tabulated degree m >= 2 agrees within 1 %
    (measured <= 0.63 %, at m = 45).  (m = 1 is eps in the .mat and 2.29e-16
    in SciPy's table; degree 1 is never selected: cost m * ceil(||A|| / theta_m).)"""
    from scipy.sparse.linalg import _expm_multiply as em
    theta = ko.theta_taylor()
    assert len(theta) == 100 and np.all(np.diff(theta) > 0)
    for m, v in em._theta.items():
        if m >= 2:
            assert abs(theta[m - 1] - v) <= 0.01 * v, (m, theta[m - 1], v)


@pytest.mark.parametrize("name", ["oregon_A0", "anaheim", "denmark", "india"])
def test_expmv_matches_scipy_expm_multiply(name):
    """The expmv restatement (expmv.m + select_taylor_degree.m + normAm.m)
    against SciPy's expm_multiply -- an independent implementation of the same
    published algorithm (Al-Mohy & Higham 2011: truncated Taylor with the same
    theta_m, shift mu = trace(A)/n, early termination) -- on the reference's
    graphs: the two agree to rounding (1e-12 relative)."""
    from scipy.sparse.linalg import expm_multiply
    A = load_graph(name).tocsr().astype(np.float64)
    rng = np.random.default_rng(5)
    b = np.sign(rng.normal(size=(A.shape[0], 10)))
    f, s, m, mv = ko.expmv(1.0, A, b)
    ref = expm_multiply(A.tocsc(), b)
    assert np.max(np.abs(f - ref)) / np.max(np.abs(ref)) < 1e-12
    assert s >= 1 and 1 <= m <= 55 and mv >= s * 1


def test_config3_fixture_estimates_within_spectral_bounds():
    """The config-3 fixture's normalisers (tests/golden/config3_values.json,
    the oracle's SLQ over 256 probes and its mc_trace) against the spectrum
    of Hawaii (hawaii_values.json, dense eigvalsh): each Rademacher
    Hutchinson estimate over N probes has sigma <= sqrt(2 ||f(A)||_F^2 / N),
    and mc_trace's error is that of its last round's 10 G probes.  The
    fixture's Frobenius norms are pinned by cosh^2 - sinh^2 = 1 summed over
    the n eigenvalues."""
    import json
    import os
    from conftest import GOLDEN
    with open(os.path.join(GOLDEN, "hawaii_values.json")) as f:
        hv = json.load(f)
    with open(os.path.join(GOLDEN, "config3_values.json")) as f:
        c3 = json.load(f)
    assert hv["frob2_cosh"] - hv["frob2_sinh"] == pytest.approx(hv["n"], rel=1e-9)
    assert hv["exact_tr_sinh"] == pytest.approx(c3["exact_tr_sinh"], rel=1e-12)
    exact, frob2 = c3["exact_tr_sinh"], hv["frob2_sinh"]
    N = c3["slq_sinh"]["probes"]
    assert abs(c3["slq_sinh"]["estimate"] - exact) <= 4 * math.sqrt(2 * frob2 / N)
    assert abs(c3["mc_trace_lanczos_sinh"]["tr"] - exact) <= 4 * math.sqrt(2 * frob2 / 10)

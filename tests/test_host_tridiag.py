"""CPU: the host Gauss quadrature of a probe's Lanczos tridiagonal
(kt_host_tridiag_quad; kt_dense.cpp tridiag_quadrature / tridiag_fun_e1),
the per-probe step after every sweep (trace_fun_update.m:78-84 for a single
vector).  Against an independent dense evaluation -- numpy's eigh of T, then
e1' f(T) e1 and f(T) e1 -- for every function code, sizes 1..60, graded and
clustered spectra, a near-breakdown off-diagonal and a split (zero) one.
f(T) e1 comes from replaying the QL pass's rotations (no eigenvector
matrix), so it is checked entry by entry."""
import ctypes as C

import numpy as np
import pytest

from krylov_robustness_amd import _lib

FUNS = {0: np.exp, 1: np.sinh, 2: np.cosh, 3: np.sin, 4: np.cos, 5: np.log, 6: np.sqrt}


def _quad(alpha, off, fun, want_vec=True):
    lib = _lib.load()
    m = len(alpha)
    a = np.ascontiguousarray(alpha, dtype=np.float64)
    e = np.ascontiguousarray(off if m > 1 else [0.0], dtype=np.float64)
    q = C.c_double(0.0)
    fe1 = np.zeros(m) if want_vec else None
    dp = C.POINTER(C.c_double)
    _lib.check(lib.kt_host_tridiag_quad(m, a.ctypes.data_as(dp), e.ctypes.data_as(dp), fun, C.byref(q),
                                        fe1.ctypes.data_as(dp) if want_vec else None))
    return q.value, fe1


def _dense(alpha, off, fun):
    T = np.diag(alpha) + np.diag(off, 1) + np.diag(off, -1)
    w, V = np.linalg.eigh(T)
    fv = V @ (FUNS[fun](w) * V[0, :])
    return float(fv[0]), fv


def _case(rng, m, kind):
    if kind == "lanczos":          # a Lanczos-like T: diagonal in the spectrum, off-diagonals positive
        return rng.uniform(-3, 8, m), np.abs(rng.normal(1.0, 0.5, m - 1)) + 0.1
    if kind == "clustered":
        return 5.0 + 1e-3 * rng.normal(size=m), np.full(m - 1, 1e-4) + 1e-5 * rng.random(m - 1)
    if kind == "nearbreak":        # one tiny coupling: the quadrature must not see past it
        a, e = rng.uniform(0, 4, m), np.abs(rng.normal(1.0, 0.3, m - 1))
        e[m // 2 - 1] = 1e-14
        return a, e
    if kind == "split":            # an exactly zero coupling (QL deflates there)
        a, e = rng.uniform(0, 4, m), np.abs(rng.normal(1.0, 0.3, m - 1))
        e[m // 3] = 0.0
        return a, e
    raise ValueError(kind)


@pytest.mark.parametrize("m", [1, 2, 3, 7, 20, 30, 60])
@pytest.mark.parametrize("kind", ["lanczos", "clustered", "nearbreak", "split"])
def test_quadrature_and_fe1_match_dense(m, kind):
    if m < 4 and kind in ("nearbreak", "split"):
        pytest.skip("needs a few steps")
    rng = np.random.default_rng(1000 * m + len(kind))
    a, e = _case(rng, m, kind)
    if m == 1:
        e = np.zeros(0)
    for fun in (0, 1, 2, 3, 4):
        q_ref, fv_ref = _dense(a, e, fun)
        scale = np.abs(fv_ref).max()
        q, fv = _quad(a, e, fun)
        q_only, _ = _quad(a, e, fun, want_vec=False)
        assert q == q_only  # the same QL pass with and without the rotation log
        assert abs(q - q_ref) <= 1e-12 * max(abs(q_ref), scale)
        np.testing.assert_allclose(fv, fv_ref, rtol=0, atol=1e-12 * scale)


@pytest.mark.parametrize("fun", [5, 6])
def test_log_sqrt_on_positive_spectrum(fun):
    rng = np.random.default_rng(fun)
    m = 25
    a = rng.uniform(4, 9, m)
    e = np.abs(rng.normal(0.5, 0.2, m - 1))  # Gershgorin: eigenvalues > 4 - 2 * max|e| > 0
    q_ref, fv_ref = _dense(a, e, fun)
    q, fv = _quad(a, e, fun)
    assert q == pytest.approx(q_ref, rel=1e-13)
    np.testing.assert_allclose(fv, fv_ref, rtol=0, atol=1e-12 * np.abs(fv_ref).max())


def test_bad_arguments_are_rejected():
    lib = _lib.load()
    q = C.c_double(0.0)
    a = np.ones(3)
    dp = C.POINTER(C.c_double)
    assert lib.kt_host_tridiag_quad(0, a.ctypes.data_as(dp), a.ctypes.data_as(dp), 0, C.byref(q), None) != 0
    assert lib.kt_host_tridiag_quad(3, a.ctypes.data_as(dp), a.ctypes.data_as(dp), 99, C.byref(q), None) != 0
    assert lib.kt_host_tridiag_quad(3, a.ctypes.data_as(dp), None, 0, C.byref(q), None) != 0

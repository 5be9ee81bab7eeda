"""CPU oracle for the trace(f(A)) hot path -- TEST INFRASTRUCTURE ONLY.

This module is a clean-room NumPy/SciPy restatement of the reference's MATLAB
algorithms (COMPiLELab/krylov_robustness, read at /root/reference/functions).
Every function cites the .m file:line it follows.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
it; the product path (``krylov_robustness_amd``) never does, and fails loudly
when its HIP library is missing instead of falling back here.

Pinning.  The reference is MATLAB-only and neither MATLAB nor Octave exists in
this image, so the reference cannot be executed and ships no golden vectors
(SURVEY.md §4, §8c).  This oracle is therefore pinned against the reference's
own known-answer identities instead (tests/test_oracle_pinning.py):
  * exact tr f(A) = sum f(eig(A))          (Tests/test_weighted_exp_lbfgs.m:41)
  * the dense shortcut of trace_fun_update (functions/trace_fun_update.m:37-51)
  * dense expm(A+UBU')-expm(A) check       (functions/fun_and_grad_krylov_exp.m:90-110)
  * exact trace-difference check           (functions/trace_fun_update.m:91-102)
Bit-level parity with MATLAB's closed built-ins (qr, eig, expm, randn) is
unpinned: MATLAB's RNG stream and LAPACK sign conventions cannot be reproduced,
so probes come from the build-defined counter RNG below.
"""
from __future__ import annotations

import math
import warnings
from dataclasses import dataclass, field
from typing import Callable, Optional

import numpy as np
import scipy.linalg as sla
import scipy.sparse as sp

# ---------------------------------------------------------------------------
# Build-defined counter RNG (SURVEY.md §8c "Probes"): splitmix64, identical in
# numpy, C (oracle/slq_ref.c) and HIP (krylov_robustness_amd/csrc/kt_kernels.hip).
# Replaces MATLAB's sign(randn(n, m)) at mc_trace.m:43-44.
# ---------------------------------------------------------------------------
_GAMMA = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def splitmix64(x):
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = x + _GAMMA
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def probe_key(seed: int, probe: int) -> np.uint64:
    with np.errstate(over="ignore"):
        return splitmix64(splitmix64(np.uint64(seed)) + np.uint64(probe))


def rademacher(n: int, probes, seed: int) -> np.ndarray:
    """n x len(probes) matrix of +-1 with entry (i, p) = sign bit of
    splitmix64(key(seed, probe_p) + i)."""
    probes = np.atleast_1d(np.asarray(probes, dtype=np.uint64))
    rows = np.arange(n, dtype=np.uint64)
    out = np.empty((n, probes.size), dtype=np.float64)
    for c, p in enumerate(probes):
        k = probe_key(seed, int(p))
        with np.errstate(over="ignore"):
            h = splitmix64(k + rows)
        out[:, c] = np.where((h >> np.uint64(63)) == 0, 1.0, -1.0)
    return out


# ---------------------------------------------------------------------------
# scalar functions by handle identity (fun_update.m:43-59)
# ---------------------------------------------------------------------------
FUNS = ("exp", "sinh", "cosh", "sin", "cos", "log", "sqrt")
_SCALAR = {"exp": np.exp, "sinh": np.sinh, "cosh": np.cosh, "sin": np.sin,
           "cos": np.cos, "log": np.log, "sqrt": np.sqrt}


def scalar_fun(name):
    """A fun_update.m:43-59 name, or any elementwise callable (a generic
    handle, trace_fun_update.m:88)."""
    if callable(name):
        return name
    return _SCALAR[name]


def matrix_fun(name: str):
    """fun_update.m:43-59: exp->expm, sinh/cosh->(expm(M)-/+expm(-M))/2,
    sin/cos->funm, log->logm, sqrt->sqrtm."""
    if name == "exp":
        return sla.expm
    if name == "sinh":
        return lambda M: (sla.expm(M) - sla.expm(-M)) / 2
    if name == "cosh":
        return lambda M: (sla.expm(M) + sla.expm(-M)) / 2
    if name == "sin":
        return lambda M: np.real_if_close(sla.funm(M, np.sin))
    if name == "cos":
        return lambda M: np.real_if_close(sla.funm(M, np.cos))
    if name == "log":
        return sla.logm
    if name == "sqrt":
        return sla.sqrtm
    raise ValueError(name)


def _matvec(A, X):
    return A @ X


def _full(A):
    return A.toarray() if sp.issparse(A) else np.asarray(A, dtype=np.float64)


def _qr0(w):
    """MATLAB qr(w, 0): economy Householder QR (LAPACK dgeqrf, as MATLAB)."""
    q, r = np.linalg.qr(w, mode="reduced")
    return q, r


# ---------------------------------------------------------------------------
# Block Lanczos: functions/lanczos_krylov.m
# ---------------------------------------------------------------------------
def _mgs_orthogonalize(V, w):
    """lanczos_krylov.m:109-115 (CGS2: two classical passes)."""
    h = V.T @ w
    w = w - V @ h
    h1 = V.T @ w
    h = h + h1
    w = w - V @ h1
    return w, h


@dataclass
class LanczosState:
    V: np.ndarray          # sliding window (n x bs, then n x 2bs)
    H: np.ndarray          # growing block tridiagonal ((j+1)bs x j bs)
    last: np.ndarray       # params.last (continuation block)
    A: object              # params.A
    lucky: bool = False


def _lanczos_add_inf_pole(V, H, A, w):
    """lanczos_krylov.m:73-101."""
    lucky_tol = 1e-8
    lucky = False
    bs = w.shape[1]
    w = _matvec(A, w)                                  # :81
    r0, c0 = H.shape
    Hn = np.zeros((r0 + bs, c0 + bs))                  # :85
    Hn[:r0, :c0] = H
    H = Hn
    rlo = max(0, H.shape[0] - 3 * bs)                  # :88 max(1,end-3bs+1)
    rhi = H.shape[0] - bs
    w, h = _mgs_orthogonalize(V, w)
    H[rlo:rhi, -bs:] = h
    w, R = _qr0(w)                                     # :90
    H[-bs:, -bs:] = R
    if np.linalg.norm(R, "fro") < lucky_tol:           # :91-93
        lucky = True
    if V.shape[1] == bs:                               # :94-99 window rotation
        V = np.hstack([V, w])
    else:
        V = np.hstack([V[:, bs:2 * bs], w])
    return V, H, w, lucky


def lanczos_krylov_start(A, b) -> LanczosState:
    """lanczos_krylov.m:30-58."""
    if A.shape[0] != A.shape[1]:
        raise ValueError("The matrix A should be square")
    if A.shape[1] != b.shape[0]:
        raise ValueError("The block vector b has wrong number of rows")
    bs = b.shape[1]
    V, _ = _qr0(b)                                     # :48
    H = np.zeros((bs, 0))
    V, H, w, lucky = _lanczos_add_inf_pole(V, H, A, V)  # :52
    return LanczosState(V=V, H=H, last=w, A=A, lucky=lucky)


def lanczos_krylov_extend(st: LanczosState) -> LanczosState:
    """lanczos_krylov.m:60-67."""
    V, H, w, lucky = _lanczos_add_inf_pole(st.V, st.H, st.A, st.last)
    return LanczosState(V=V, H=H, last=w, A=st.A, lucky=lucky)


# ---------------------------------------------------------------------------
# Block Arnoldi: functions/arnoldi_krylov.m
# ---------------------------------------------------------------------------
@dataclass
class ArnoldiState:
    V: np.ndarray
    K: np.ndarray
    H: np.ndarray
    last: np.ndarray
    A: object
    lucky: bool = False


def _arnoldi_add_inf_pole(V, K, H, A, w):
    """arnoldi_krylov.m:78-111."""
    lucky_tol = 1e-12
    lucky = False
    bs = w.shape[1]
    w = _matvec(A, w)                                   # :86
    w, h = _mgs_orthogonalize(V, w)                     # :90 (arnoldi_krylov.m:119-125)
    r0, c0 = H.shape
    Hn = np.zeros((r0 + bs, c0 + bs)); Hn[:r0, :c0] = H; H = Hn
    Kn = np.zeros((r0 + bs, c0 + bs)); Kn[:r0, :c0] = K; K = Kn
    H[:-bs, -bs:] = h                                   # :96
    K[-2 * bs:-bs, -bs:] = np.eye(bs)                   # :97
    w, r = _qr0(w)                                      # :99
    if np.linalg.norm(r, 2) < lucky_tol:                # :100-102
        lucky = True
    hh = V.T @ w                                        # :104-106 reorthogonalize
    w = w - V @ hh
    H[:-bs, -bs:] = H[:-bs, -bs:] + hh @ r
    H[-bs:, -bs:] = r                                   # :108
    V = np.hstack([V, w])                               # :110
    return V, K, H, w, lucky


def arnoldi_krylov_start(A, b) -> ArnoldiState:
    """arnoldi_krylov.m:32-62."""
    if A.shape[0] != A.shape[1]:
        raise ValueError("The matrix A should be square")
    bs = b.shape[1]
    V, _ = _qr0(b)
    H = np.zeros((bs, 0)); K = np.zeros((bs, 0))
    V, K, H, w, lucky = _arnoldi_add_inf_pole(V, K, H, A, V)
    return ArnoldiState(V=V, K=K, H=H, last=w, A=A, lucky=lucky)


def arnoldi_krylov_extend(st: ArnoldiState) -> ArnoldiState:
    """arnoldi_krylov.m:64-72."""
    V, K, H, w, lucky = _arnoldi_add_inf_pole(st.V, st.K, st.H, st.A, st.last)
    return ArnoldiState(V=V, K=K, H=H, last=w, A=st.A, lucky=lucky)


# ---------------------------------------------------------------------------
# trace_fun_update: functions/trace_fun_update.m
# ---------------------------------------------------------------------------
def _trace_diff(d1, d2, fun):
    """trace_fun_update.m:43-47 / :85-89."""
    if isinstance(fun, str) and fun == "exp":
        return float(np.sum(np.exp(d1) * (1 - np.exp(d2 - d1))))
    f = scalar_fun(fun)
    return float(np.sum(f(d1) - f(d2)))


def _ishermitian(B):
    B = np.atleast_2d(B)
    return B.shape[0] == B.shape[1] and np.array_equal(B, B.T)


def trace_fun_update(A, U, B, tol=1e-12, it=None, debug=0, fun="exp", hist=None):
    """[Xm, iter, lucky] = trace_fun_update(A, U, B, tol, it, debug, fun)
    (trace_fun_update.m:1-135).  hist (test aid, not in the reference): a list
    that receives (j, err, Xm) for every lag-2 stop test evaluated."""
    U = np.asarray(U, dtype=np.float64)
    if U.ndim == 1:
        U = U[:, None]
    B = np.atleast_2d(np.asarray(B, dtype=np.float64))
    n = A.shape[0]
    if it is None:
        it = min(100, n)                                  # :25-27
    if U.shape[0] <= 130:                                 # :37-51 dense shortcut
        fA = _full(A)
        fAt = fA + U @ B @ U.T
        fAt = (fAt + fAt.T) / 2
        d1 = np.sort(np.linalg.eigvalsh(fAt))
        d2 = np.sort(np.linalg.eigvalsh(fA))
        return _trace_diff(d1, d2, fun), 0, 0
    rk = U.shape[1]                                       # :54
    herm = _ishermitian(B)                                # :55
    d = 2                                                 # :58
    Xstop = np.zeros(d)
    st = None
    Cm = None
    Xm = 0.0
    lucky = False
    j = 0
    for j in range(1, it + 1):                            # :60
        if j == 1:
            st = lanczos_krylov_start(A, U)               # :64
            Cm = st.V[:, :st.V.shape[1] - rk].T @ U       # :65 (Um(:, 1:end-rk))
            Cm = Cm @ B @ Cm.T                            # :66
        else:
            st = lanczos_krylov_extend(st)                # :68
        lucky = st.lucky
        HA = st.H
        Gm = HA[:HA.shape[0] - rk, :]                     # :72
        nn = Gm.shape[0]
        if nn > Cm.shape[0]:                              # :74-76 zero padding
            Cp = np.zeros((nn, nn)); Cp[:Cm.shape[0], :Cm.shape[1]] = Cm; Cm = Cp
        tGm = Gm + Cm                                     # :77
        if herm:                                          # :78-81
            Gm = (Gm + Gm.T) / 2
            tGm = (tGm + tGm.T) / 2
        d1 = np.sort(np.linalg.eigvals(tGm).real) if not herm else np.sort(np.linalg.eigvalsh(tGm))
        d2 = np.sort(np.linalg.eigvals(Gm).real) if not herm else np.sort(np.linalg.eigvalsh(Gm))
        Xm = _trace_diff(d1, d2, fun)                     # :85-89
        if j <= d:                                        # :104-118 lag-2 stop
            Xstop[j - 1] = Xm
        else:
            err = abs(Xm - Xstop[0])
            if hist is not None:
                hist.append((j, err, Xm))
            if err < tol:
                break
            Xstop = np.array([*Xstop[1:d], Xm])
        if lucky:                                         # :119-124
            break
    iter_ = j
    if iter_ == it:                                       # :128-130
        warnings.warn("TRACE_FUN_UPDATE:: Reached maximum number of iterations")
    return Xm, iter_, lucky


# ---------------------------------------------------------------------------
# fun_update: functions/fun_update.m (Arnoldi branch when nargout == 4)
# ---------------------------------------------------------------------------
def fun_update(A, U, B, fun="exp", tol=1e-12, it=None, debug=0, nargout=4):
    """[Xm, iter, lucky, Um] = fun_update(A, U, B, fun, tol, it, debug)
    (fun_update.m:1-140).  nargout<=3 takes the Lanczos branch (:69-76),
    nargout==4 the Arnoldi branch (:77-91)."""
    U = np.asarray(U, dtype=np.float64)
    if U.ndim == 1:
        U = U[:, None]
    B = np.atleast_2d(np.asarray(B, dtype=np.float64))
    n = A.shape[0]
    if it is None:
        it = min(100, n)
    rk = U.shape[1]
    herm = _ishermitian(B)
    f = matrix_fun(fun)
    d = 2
    Xstop = []
    st = None
    Cm = None
    Xm = None
    lucky = False
    j = 0
    for j in range(1, it + 1):                            # :66
        if nargout <= 3:
            if j == 1:
                st = lanczos_krylov_start(A, U)
                Cm = st.V[:, :st.V.shape[1] - rk].T @ U
                Cm = Cm @ B @ Cm.T
            else:
                st = lanczos_krylov_extend(st)
        else:
            if j == 1:
                st = arnoldi_krylov_start(A, U)           # :79
                Cm = st.V[:, :st.V.shape[1] - rk].T @ U   # :80
                Cm = Cm @ B @ Cm.T                        # :81
            else:
                st = arnoldi_krylov_extend(st)            # :83
            if st.V.shape[1] >= st.V.shape[0] / 2:        # :85-90 dense fallback
                Um = np.eye(U.shape[0])
                fA = _full(A)
                Xm = f(fA + U @ B @ U.T) - f(fA)
                return np.real_if_close(Xm), j, st.lucky, Um
        lucky = st.lucky
        HA = st.H
        Gm = HA[:HA.shape[0] - rk, :]                     # :93
        Gm = (Gm + Gm.T) / 2                              # :94
        nn = Gm.shape[0]
        if nn > Cm.shape[0]:                              # :97-99
            Cp = np.zeros((nn, nn)); Cp[:Cm.shape[0], :Cm.shape[1]] = Cm; Cm = Cp
        if herm:                                          # :100-104
            tGm = Gm + (Cm + Cm.T) / 2
        else:
            tGm = Gm + Cm
        Xm = np.real_if_close(f(tGm) - f(Gm))             # :106
        if j <= d:                                        # :109-126
            Xstop.append(Xm)
        else:
            nn = Xm.shape[0]
            X1 = np.zeros((nn, nn)); X1[:Xstop[0].shape[0], :Xstop[0].shape[1]] = Xstop[0]
            err = np.linalg.norm(Xm - X1, 2)
            if err < tol:
                break
            Xstop = [*Xstop[1:d], Xm]
        if lucky:                                         # :127-130
            warnings.warn("FUN_UPDATE:: Detected lucky breakdown")
            break
    iter_ = j
    if iter_ == it:                                       # :133-135
        warnings.warn("FUN_UPDATE:: Reached maximum number of iterations")
    if Xm.shape[0] > st.V.shape[1]:                       # :137 on the Lanczos branch's window
        raise IndexError(f"fun_update.m:137: index exceeds the {st.V.shape[1]} columns of V")
    Um = st.V[:, :Xm.shape[0]]                            # :137
    return Xm, iter_, lucky, Um


# ---------------------------------------------------------------------------
# normest: MATLAB's normest (2-norm power estimate), called at
# fun_and_grad_krylov_exp.m:26 / fun_and_grad_krylov_fun.m:27 with tol 1e-2.
# MATLAB built-in (unpinned third party); restated from its published algorithm.
# ---------------------------------------------------------------------------
def normest(A, tol=1e-6, maxiter=100):
    x = np.asarray(abs(A).sum(axis=0)).ravel()
    e = np.linalg.norm(x)
    if e == 0:
        return 0.0
    x = x / e
    e0 = 0.0
    cnt = 0
    while abs(e - e0) > tol * e:
        e0 = e
        Ax = A @ x
        if np.count_nonzero(Ax) == 0:
            Ax = np.random.default_rng(0).random(Ax.shape)
        x = A.T @ Ax
        normx = np.linalg.norm(x)
        e = normx / np.linalg.norm(Ax)
        x = x / normx
        cnt += 1
        if cnt > maxiter:
            break
    return float(e)


# ---------------------------------------------------------------------------
# Low-rank factor from edge weights: fun_and_grad_krylov_exp.m:56-73
# ---------------------------------------------------------------------------
def lowrank_from_edges(X, Omega, n):
    """Omega is 1-based (|Omega| x 2), as MATLAB passes it."""
    Omega = np.asarray(Omega, dtype=np.int64)
    X = np.asarray(X, dtype=np.float64).ravel()
    aux = np.unique(Omega.ravel())                        # :57 unique(Omega(:))
    k = aux.size
    iaux = {int(a): i for i, a in enumerate(aux)}         # :59-60
    U = np.zeros((n, k))
    B = np.zeros((k, k))
    for j in range(k):                                    # :65-67
        U[aux[j] - 1, j] = 1.0
    for j in range(Omega.shape[0]):                       # :68-73
        i1 = iaux[int(Omega[j, 0])]
        i2 = iaux[int(Omega[j, 1])]
        B[i1, i2] = X[j]
        B[i2, i1] = X[j]
    return U, B


def _check_hermitian(A, msg):
    if sp.issparse(A):
        d = abs(A - A.T)
        if d.nnz and d.max() != 0:
            raise ValueError(msg)
    elif not np.array_equal(A, A.T):
        raise ValueError(msg)


def fun_and_grad_krylov_exp(X, A, Omega, eA, tol, it, debug=False):
    """[f, gr] = fun_and_grad_krylov_exp(X, A, Omega, eA, tol, it, debug)
    (fun_and_grad_krylov_exp.m:1-113)."""
    _check_hermitian(A, "FUN_AND_GRAD_KRYLOV:: matrix A is not Hermitian")  # :21-23
    Omega = np.asarray(Omega, dtype=np.int64)
    eA = np.asarray(eA, dtype=np.float64).ravel()
    n = A.shape[0]
    nrmA = normest(A, 1e-2)                               # :26
    if np.sum(np.abs(X)) == 0:                            # :30-54
        return 0.0, -2 * eA
    U, B = lowrank_from_edges(X, Omega, n)
    eXm, _, _, Um = fun_update(A, U, B, "exp", tol * math.exp(nrmA), it, False, nargout=4)  # :83
    f = -float(np.trace(eXm))                             # :84
    DeA = np.einsum("ij,jk,ik->i", Um[Omega[:, 0] - 1, :], eXm, Um[Omega[:, 1] - 1, :])  # :85-86
    gr = -2 * (eA + DeA)                                  # :88
    return f, gr


def fun_and_grad_krylov_fun(X, A, Omega, fun, dfun, dfA, tol, it, debug=False, fun_M=None):
    """[f, gr] = fun_and_grad_krylov_fun(X, A, Omega, fun, dfun, dfA, tol, it, debug, fun_M)
    (fun_and_grad_krylov_fun.m:1-71)."""
    _check_hermitian(A, "FUN_AND_GRAD_KRYLOV_FCONNECTIVITY:: matrix A is not Hermitian")  # :22-24
    Omega = np.asarray(Omega, dtype=np.int64)
    dfA = np.asarray(dfA, dtype=np.float64).ravel()
    n = A.shape[0]
    nrmA = normest(A, 1e-2)                               # :27
    if np.sum(np.abs(X)) == 0:                            # :31-35
        return 0.0, -2 * dfA
    U, B = lowrank_from_edges(X, Omega, n)
    dfXm, _, _, Um = fun_update(A, U, B, dfun, tol * scalar_fun(dfun)(nrmA), it, False, nargout=4)  # :64
    f = -trace_fun_update(A, U, B, tol * scalar_fun(fun)(nrmA), it, False, fun)[0]              # :65
    DdfA = np.einsum("ij,jk,ik->i", Um[Omega[:, 0] - 1, :], dfXm, Um[Omega[:, 1] - 1, :])       # :67-68
    gr = -2 * (dfA + DdfA)                                # :70
    return f, gr


# ---------------------------------------------------------------------------
# expmv / select_taylor_degree / normAm (third-party Al-Mohy & Higham code
# vendored in the reference: functions/expmv.m, select_taylor_degree.m, normAm.m)
# ---------------------------------------------------------------------------
_THETA = None


def theta_taylor():
    """theta_taylor.mat (1 x 100 fp64), loaded by select_taylor_degree.m:31.
    Tests load it from a committed fixture; see tests/golden/theta_taylor.npy."""
    global _THETA
    if _THETA is None:
        import os
        here = os.path.dirname(os.path.abspath(__file__))
        p = os.path.join(here, "..", "tests", "golden", "theta_taylor.npy")
        _THETA = np.load(p).ravel()
    return _THETA


def _mysign(y):
    """normest1's mysign: sign with sign(0) = +1."""
    s = np.sign(y)
    s[s == 0] = 1.0
    return s


def normest1_t1(matvec, rmatvec, n):
    """[est, ~, ~, it] = normest1(afun, t = 1) -- the block 1-norm estimator
    of Higham & Tisseur (SIAM J. Matrix Anal. Appl. 21(4), 2000, Algorithm
    2.4) that normAm.m:25 calls with ONE column, so no random start columns
    and no column de-duplication are involved: the iteration is
    deterministic.  MATLAB's normest1 itself is a closed built-in (not in the
    reference); this restates the published algorithm, with
    ties in the ordering of h broken towards the smallest index.  Returns
    (est, it1, it2) -- it2 = the number of transposed products, which
    normAm.m:26 turns into mv = it(2) * t * m.
      n <= 4: the exact norm from the identity's columns (no iteration)."""
    if n <= 4:
        Y = np.column_stack([matvec(e) for e in np.eye(n)])
        return float(np.abs(Y).sum(axis=0).max()), 1, 0
    X = np.ones(n) / n                                    # X = ones(n,t)/n
    itmax = 5
    est_old = 0.0
    ind = -1                                              # index of the unit vector X
    ind_best = -1
    S = np.zeros(n)
    k = 1
    it1 = it2 = 0
    est = 0.0
    while True:
        Y = matvec(X)                                     # (1) Y = A X
        it1 += 1
        est = float(np.abs(Y).sum())
        if est > est_old or k == 2:
            if k >= 2:
                ind_best = ind
        if k >= 2 and est <= est_old:                     # (2) no improvement
            est = est_old
            break
        est_old = est
        S_old = S
        if k > itmax:
            break
        S = _mysign(Y)                                    # (3)
        if abs(float(S_old @ S)) == n:                    # S parallel to S_old
            break
        Z = rmatvec(S)                                    # (4) Z = A' S
        it2 += 1
        h = np.abs(Z)
        hmax = float(h.max())
        if k >= 2 and hmax == h[ind_best]:                # (5)
            break
        ind = int(np.argmax(h))                           # first index of the maximum
        X = np.zeros(n)                                   # X = e_ind
        X[ind] = 1.0
        k += 1
    return est, it1, it2


def normAm(A, m):
    """normAm.m:1-52."""
    n = A.shape[0]
    nonneg = (A.min() >= 0) if sp.issparse(A) else bool(np.all(A >= 0))
    if nonneg:                                            # :17-23
        e = np.ones(n)
        for _ in range(m):
            e = A.T @ e
        return float(np.max(np.abs(e))), m

    # :25-26 [c,v,w,it] = normest1(@afun_power, t = 1); mv = it(2)*t*m
    def mv(x):
        for _ in range(m):
            x = A @ x
        return x

    def rmv(x):
        for _ in range(m):
            x = A.T @ x
        return x
    c, _, it2 = normest1_t1(mv, rmv, n)
    return float(c), it2 * m


def select_taylor_degree(A, b, m_max=55, p_max=8, shift=False, force_estm=False):
    """select_taylor_degree.m:1-68 (prec='double', bal=false)."""
    theta = theta_taylor()
    n = A.shape[0]
    if shift:                                             # :37-40
        mu = A.diagonal().sum() / n
        A = A - mu * sp.eye(n, format="csr")
    mv = 0
    normA = abs(A).sum(axis=0).max() if not force_estm else None   # :42 norm(A,1)
    ncols = b.shape[1] if b.ndim > 1 else 1
    if not force_estm and normA <= 4 * theta[m_max - 1] * p_max * (p_max + 3) / (m_max * ncols):  # :44
        unA = 1
        alpha = normA * np.ones(p_max - 1)
    else:                                                 # :51-61
        unA = 0
        eta = np.zeros(p_max)
        alpha = np.zeros(p_max - 1)
        for p in range(1, p_max + 1):
            c, k = normAm(A, p + 1)
            c = c ** (1.0 / (p + 1))
            mv += k
            eta[p - 1] = c
        for p in range(1, p_max):
            alpha[p - 1] = max(eta[p - 1], eta[p])
    M = np.zeros((m_max, p_max - 1))                      # :63-68
    for p in range(2, p_max + 1):
        for m in range(p * (p - 1) - 1, m_max + 1):
            M[m - 1, p - 2] = alpha[p - 2] / theta[m - 1]
    return M, mv, alpha, unA


def expmv(t, A, b, M=None, shift=True, full_term=False):
    """expmv.m:1-94 with prec='double', bal=false.  Returns (f, s, m, mv)."""
    n = A.shape[0]
    b = np.asarray(b, dtype=np.float64)
    mu = 0.0
    if shift:                                             # :33-36
        mu = float(A.diagonal().sum()) / n
        if mu != 0.0:
            A = A - mu * sp.eye(n, format="csr")
    if M is None:                                         # :39-45
        tt = 1
        M, mvd, alpha, unA = select_taylor_degree(t * A, b, shift=False)
        mv = mvd
    else:
        tt = t
        mv = 0
    tol = 2.0 ** -53                                      # :48
    s = 1
    if t == 0:                                            # :53-68
        m = 0
    else:
        m_max, p = M.shape
        Ud = np.diag(np.arange(1, m_max + 1))
        C = (np.ceil(abs(tt) * M)).T @ Ud
        C[C == 0] = np.inf
        if p > 1:
            colmin = C.min(axis=0)                        # min over p (rows of C)
            m = int(np.argmin(colmin)) + 1
            cost = colmin[m - 1]
        else:
            m = int(np.argmin(C)) + 1
            cost = C.ravel()[m - 1]
        if cost == np.inf:
            cost = 0
        s = max(cost / m, 1)
    s = int(s)
    eta = 1.0
    if shift:                                             # :70
        eta = math.exp(t * mu / s)
    f = b.copy()
    for i in range(s):                                    # :73-92
        c1 = np.max(np.sum(np.abs(b), axis=1)) if b.ndim > 1 else np.max(np.abs(b))  # norm(b, inf)
        for k in range(1, m + 1):
            b = (t / (s * k)) * (A @ b)
            mv += 1
            f = f + b
            c2 = np.max(np.sum(np.abs(b), axis=1)) if b.ndim > 1 else np.max(np.abs(b))
            if not full_term:
                nf = np.max(np.sum(np.abs(f), axis=1)) if f.ndim > 1 else np.max(np.abs(f))
                if c1 + c2 <= tol * nf:
                    break
                c1 = c2
        f = eta * f
        b = f
    return f, s, m, mv


# ---------------------------------------------------------------------------
# mc_trace: functions/mc_trace.m (block Hutchinson with nested deflation)
# ---------------------------------------------------------------------------
def mc_trace(Afun, n, tol=1e-3, maxit=10, isAreal=0, debug=0, seed=0):
    """[tr_new, res, it] = mc_trace(Afun, n, tol, maxit, isAreal, debug)
    (mc_trace.m:1-63).  Probes: S = columns (it-1)*20 + [0,10), G = +10
    of the counter RNG (replaces sign(randn(n, m)) at :43-44)."""
    if not callable(Afun):                                # :32-34
        Amat = Afun
        Afun = lambda x: Amat @ x
    tr = 0.0
    tr_old = 0.0
    m = 10                                                # :36
    K = math.ceil(maxit / (3 * m))                        # :41
    tr_new = 0.0
    res = 1.0
    it = 0
    for it in range(1, K + 1):                            # :42
        base = (it - 1) * 2 * m
        S = rademacher(n, np.arange(base, base + m), seed)          # :43
        G = rademacher(n, np.arange(base + m, base + 2 * m), seed)  # :44
        Q, _ = _qr0(Afun(S))                              # :45
        tr = tr + float(np.trace(Q.T @ Afun(Q)))          # :46
        aux = (lambda Q: (lambda x: x - Q @ (Q.T @ x)))(Q)          # :47
        Afun = (lambda F, P: (lambda x: P(F(P(x)))))(Afun, aux)     # :48
        tr_new = tr + float(np.trace(G.T @ Afun(G))) / m  # :49
        res = abs(tr_new - tr_old) / max(abs(tr_new), abs(tr_old))  # :50
        if res < tol:                                     # :54-56
            break
        tr_old = tr_new
    if isAreal == 1:
        tr_new = float(np.real(tr_new))
    return tr_new, res, it


def trace_exp(A, seed=0):
    """trace_exp.m:1-7: mc_trace(@(x) expmv(1, A, x, [], 'double'), n, 1e-4, 1000, 1)."""
    Afun = lambda x: expmv(1.0, A, x)[0]
    return mc_trace(Afun, A.shape[0], 1e-4, 1000, 1, seed=seed)[0]


# ---------------------------------------------------------------------------
# NEW composition: Lanczos-quadrature Afun for probes.
# Per probe the bs=1 case of lanczos_krylov's add_inf_pole (CGS2 against the
# two-vector window, lanczos_krylov.m:73-115) for m steps; T_m is the
# symmetrised projected matrix (as trace_fun_update.m:78-81 does for Gm);
#   z' f(A) z ~= ||z||^2 * e1' f(T_m) e1 = ||z||^2 sum_k tau_k^2 f(theta_k)
#   f(A) z     ~= ||z|| V_m f(T_m) e1.
# ---------------------------------------------------------------------------
def lanczos_probe_tridiag(A, z, m):
    """Run m single-vector steps of lanczos_krylov from z.
    Returns (alpha[m'], offdiag[m'-1], V (n x m'), lucky) where m' <= m stops
    early on lucky breakdown (lanczos_krylov.m:91-93)."""
    z = np.asarray(z, dtype=np.float64).reshape(-1, 1)
    st = lanczos_krylov_start(A, z)
    Vs = [st.V[:, :1]]
    steps = 1
    while steps < m and not st.lucky:
        st = lanczos_krylov_extend(st)
        Vs.append(st.V[:, :1])
        steps += 1
    H = st.H[:steps, :steps]
    T = (H + H.T) / 2
    alpha = np.diag(T).copy()
    off = np.diag(T, -1).copy()
    return alpha, off, np.hstack(Vs), st.lucky


def tridiag_quadrature(alpha, off, fun="exp"):
    """e1' f(T) e1 for symmetric tridiagonal T (Gauss quadrature)."""
    alpha = np.asarray(alpha, dtype=np.float64)
    if alpha.size == 1:
        return float(scalar_fun(fun)(alpha[0]))
    theta, W = sla.eigh_tridiagonal(alpha, np.asarray(off, dtype=np.float64))
    tau = W[0, :]
    return float(np.sum(tau * tau * scalar_fun(fun)(theta)))


def lanczos_quadform(A, z, m, fun="exp"):
    """z' f(A) z by m-step Lanczos quadrature."""
    z = np.asarray(z, dtype=np.float64).ravel()
    nz2 = float(z @ z)
    if nz2 == 0.0:
        return 0.0
    a, e, _, _ = lanczos_probe_tridiag(A, z, m)
    return nz2 * tridiag_quadrature(a, e, fun)


def lanczos_fmv(A, X, m, fun="exp"):
    """f(A) X ~= per column ||x|| V_m f(T_m) e1 (the Lanczos-f handle)."""
    X = np.asarray(X, dtype=np.float64)
    if X.ndim == 1:
        X = X[:, None]
    Y = np.zeros_like(X)
    for c in range(X.shape[1]):
        x = X[:, c]
        nx = np.linalg.norm(x)
        if nx == 0:
            continue
        a, e, V, _ = lanczos_probe_tridiag(A, x, m)
        if a.size == 1:
            coef = np.array([scalar_fun(fun)(a[0])])
        else:
            theta, W = sla.eigh_tridiagonal(a, e)
            coef = W @ (scalar_fun(fun)(theta) * W[0, :])
        # sign of v1 follows qr(b,0); undo so that V[:,0] ~ x/||x|| direction
        s = np.sign(V[:, 0] @ x) or 1.0
        Y[:, c] = s * nx * (V @ coef)
    return Y


def slq_trace(A, nprobes, m, seed=0, fun="exp", probe_offset=0):
    """Plain Hutchinson with Lanczos quadrature over Rademacher probes
    (configs 2-4).  Returns (trace estimate, per-probe quadratic forms)."""
    n = A.shape[0]
    q = np.zeros(nprobes)
    for p in range(nprobes):
        z = rademacher(n, [probe_offset + p], seed)[:, 0]
        q[p] = lanczos_quadform(A, z, m, fun)
    return float(q.mean()), q


def trace_exp_lanczos(A, m=20, tol=1e-4, maxit=1000, seed=0, fun="exp"):
    """Config 1 composition: mc_trace's structure with Afun = Lanczos-f."""
    Afun = lambda X: lanczos_fmv(A, X, m, fun)
    return mc_trace(Afun, A.shape[0], tol, maxit, 1, seed=seed)


# ---------------------------------------------------------------------------
# exact dense answers (the reference's own known-answer checks)
# ---------------------------------------------------------------------------
def exact_trace_fun(A, fun="exp"):
    """sum(f(eig(full(A)))) -- test_weighted_exp_lbfgs.m:41, test_weighted_sinh_lbfgs.m:50."""
    d = np.linalg.eigvalsh(_full(A))
    return float(np.sum(scalar_fun(fun)(d)))


def exact_trace_update(A, U, B, fun="exp"):
    """trace_fun_update.m:91-102 (debug == 3 truth)."""
    U = np.atleast_2d(U)
    if U.shape[0] == 1:
        U = U.T
    fA = _full(A)
    t1 = np.sort(np.linalg.eigvalsh(fA + U @ np.atleast_2d(B) @ U.T))
    t2 = np.sort(np.linalg.eigvalsh(fA))
    return _trace_diff(t1, t2, fun)


# ---------------------------------------------------------------------------
# greedy edge selection: krylov_miobi.m / greedy_krylov.m (host loop logic)
# ---------------------------------------------------------------------------
def krylov_miobi(A, k, E, tol=1e-12, it=None, poles=np.inf, debug=0, miobi="break", rescale=1.0):
    """krylov_miobi.m:1-142 (E 1-based, E(j,1) >= E(j,2); poles unused there too)."""
    A = sp.csr_matrix(A, dtype=np.float64).copy()
    if E is None or len(E) == 0:                          # :43-46 [tmp1, tmp2] = find(A), tmp1 >= tmp2
        C = sp.csc_matrix(A)
        C.sort_indices()
        cols = np.repeat(np.arange(C.shape[1]), np.diff(C.indptr))   # find(): column-major
        rows = C.indices
        keep = (rows >= cols) & (C.data != 0)
        E = np.stack([rows[keep], cols[keep]], axis=1) + 1
    E = np.asarray(E, dtype=np.int64).reshape(-1, 2).copy()
    n = A.shape[0]
    if it is None:
        it = min(100, n)
    nE = E.shape[0]
    rob = 0.0
    edges = np.zeros((0, 2), dtype=np.int64)
    chosen = np.zeros(2, dtype=np.int64)
    for _ in range(min(k, nE)):                           # :70
        mx = [0, np.inf] if miobi == "break" else [0, -np.inf]
        for h in range(nE):                               # :76
            i, j = int(E[h, 0]), int(E[h, 1])
            sgn = -1.0 if miobi == "break" else 1.0
            if i != j:                                    # :77-87
                B = sgn * np.array([[0.0, 1.0], [1.0, 0.0]]) / rescale
                U = np.zeros((n, 2)); U[i - 1, 0] = 1; U[j - 1, 1] = 1
            else:                                         # :88-98
                B = np.array([[sgn]])
                U = np.zeros((n, 1)); U[i - 1, 0] = 1
            tmp = trace_fun_update(A, U, B, tol, it, debug)[0]   # :99
            if (miobi == "break" and tmp < mx[1]) or (miobi != "break" and tmp > mx[1]):  # :112-124
                mx = [h + 1, tmp]
                chosen = E[h, :].copy()
        E = np.delete(E, mx[0] - 1, axis=0)               # :127
        nE -= 1
        A = A.tolil()
        val = 0.0 if miobi == "break" else 1.0            # :129-135
        A[chosen[0] - 1, chosen[1] - 1] = val
        A[chosen[1] - 1, chosen[0] - 1] = val
        A = A.tocsr(); A.eliminate_zeros()
        edges = np.vstack([edges, chosen])
        rob += mx[1]
    return edges, rob, A


def find_top_edges(A, centrality, num, order="mult"):
    """find_top_edges.m:14-39, written as the reference's loops.  A MATLAB
    sparse matrix holds no duplicate entries (they are summed when it is
    built), so duplicates of a SciPy input are summed first."""
    A = sp.csc_matrix(A, copy=True)
    A.sum_duplicates()
    n = A.shape[0]
    I, J = [], []
    for j in range(n):                                    # find(tril(A,-1)): column-major
        for t in range(A.indptr[j], A.indptr[j + 1]):
            i = A.indices[t]
            if i > j and A.data[t] != 0:
                I.append(i)
                J.append(j)
    order_idx = list(range(len(I)))
    cen = [float(x) for x in np.ravel(centrality)]
    if order == "mult":                                   # :22-25
        c = [cen[I[h]] * cen[J[h]] for h in range(len(I))]
        order_idx = sorted(range(len(I)), key=lambda h: -c[h])        # stable, descending
    elif order == "min":                                  # :26-37
        sc = sorted(cen, reverse=True)
        scores = []
        for h in range(len(I)):
            c1 = sc.index(cen[I[h]]) + 1
            c2 = sc.index(cen[J[h]]) + 1
            mn, mx = min(c1, c2), max(c1, c2)
            scores.append(mx * (mx - 1) / 2 + mn)
        order_idx = sorted(range(len(I)), key=lambda h: scores[h])    # stable, ascending
    if len(I) < num:                                      # :19-21 (a warning)
        warnings.warn("FIND_TOP_EDGES:: there are not enough edges in the graph")
    num = int(math.floor(num))                            # E(ind(1:num), :)
    if len(I) < num:                                      # index exceeds: MATLAB errors
        raise IndexError("FIND_TOP_EDGES:: there are not enough edges in the graph")
    return np.array([[I[h] + 1, J[h] + 1] for h in order_idx[:num]], dtype=np.int64)


def find_top_missing_edges_min(A, centrality, num):
    """find_top_missing_edges.m:52-64 ('min' order), as the reference's loop."""
    A = sp.csr_matrix(A)
    cen = np.ravel(centrality)
    indC = sorted(range(len(cen)), key=lambda i: -cen[i])        # sort(.., 'descend'), stable
    E = []
    j = 1
    while len(E) < num:
        for t in range(j):
            if A[indC[t], indC[j]] == 0:
                E.append([indC[t] + 1, indC[j] + 1])
        j += 1
    return np.array(E[:int(math.floor(num))], dtype=np.int64)  # E(1:num, :)


def greedy_krylov(A, k, Q, centrality, order="mult", tol=1e-12, it=None, poles=np.inf, debug=0,
                  miobi="break", rescale=1.0):
    """greedy_krylov.m:64-93 over krylov_miobi (break: find_top_edges; make:
    find_top_missing_edges with the 'min' order)."""
    edges = np.zeros((0, 2), dtype=np.int64)
    rob = 0.0
    top = None
    tmp_edges = None
    if not Q:                                             # :42-44 Q = max(sum(A, 1))
        Q = float(np.asarray(sp.csr_matrix(A).sum(axis=0)).max())
    Qi = int(np.floor(Q))                                 # 1:Q indexes floor(Q) rows
    for j in range(k):
        if j == 0:
            top = (find_top_edges(A, centrality, Q + k, order) if miobi == "break"
                   else find_top_missing_edges_min(A, centrality, Q + k))  # :69 / :80, unfloored
        else:
            hit = [h for h in range(len(top)) if tuple(top[h]) == tuple(tmp_edges[0])]
            # :84-86 with no match, [1 : ind-1, ind+1 : n] is empty: top_edges empties
            top = np.delete(top, hit[0], axis=0) if hit else top[:0]
        E = top[:Qi]
        tmp_edges, tmp_rob, A = krylov_miobi(A, 1, E, tol, it, poles, debug, miobi, rescale)
        edges = np.vstack([edges, tmp_edges])
        rob += tmp_rob
    return edges, rob, A


# ---------------------------------------------------------------------------
# function_multiple_entries.m (poles = inf)
# ---------------------------------------------------------------------------
def fme_matrix_fun(name: str):
    """function_multiple_entries.m:47-60: exp->expm, sin/cos->funm, log->logm,
    sqrt->sqrtm, anything else funm(M, f) (sinh/cosh here)."""
    if name == "exp":
        return sla.expm
    if name in ("sin", "cos"):
        return lambda M: np.real_if_close(sla.funm(M, scalar_fun(name)))
    if name == "sinh":
        return sla.sinhm
    if name == "cosh":
        return sla.coshm
    if name == "log":
        return sla.logm
    if name == "sqrt":
        return sla.sqrtm
    raise ValueError(name)


def function_multiple_entries(A, omega, f="exp", tol=1e-12, it=None, poles=np.inf, debug=0):
    """[X, iter] = function_multiple_entries(A, omega, f, tol, it, poles, debug)
    (function_multiple_entries.m:1-181); omega is 1-based (k x 2)."""
    omega = np.asarray(omega, dtype=np.int64).reshape(-1, 2)
    n = A.shape[0]
    if it is None:
        it = min(100, n)                                  # :24-26
    k = omega.shape[0]
    I0 = list(dict.fromkeys(omega[:, 0].tolist()))        # unique(.., 'stable')   :42
    row = {t: i for i, t in enumerate(I0)}                # the handle keeps the first I  :44
    fM = fme_matrix_fun(f)
    d = 3                                                 # :63
    Xstop = [[] for _ in range(k)]
    notconverged = list(range(k))
    St = [None] * len(I0)
    Uaux = np.zeros(len(I0))
    Gm = [None] * len(I0)
    Xm = [None] * k
    I = list(I0)
    j = 0
    for j in range(1, it + 1):                            # :84
        for h in I:                                       # :86
            r_ = row[h]
            if j == 1:
                U = np.zeros((n, 1)); U[h - 1, 0] = 1.0
                St[r_] = arnoldi_krylov_start(A, U)
                Uaux[r_] = (St[r_].V.T @ U)[0, 0]         # :94-95
            else:
                St[r_] = arnoldi_krylov_extend(St[r_])
            Gm[r_] = St[r_].H[:-1, :]                     # :106
        stop = True
        for h in list(notconverged):                      # :113
            Xm[h] = fM(Gm[row[omega[h, 0]]])
            if j <= d:
                Xstop[h].append(Xm[h])
                stop = False
            else:
                nn = Xm[h].shape[0]
                old = np.zeros((nn, nn))
                o = Xstop[h][0]
                old[:o.shape[0], :o.shape[1]] = o
                err = np.linalg.norm((Xm[h] - old)[:, 0])
                if err > tol:
                    stop = False
                else:
                    notconverged = [x for x in notconverged if x != h]
                    I = list(dict.fromkeys(omega[notconverged, 0].tolist()))
                Xstop[h] = Xstop[h][1:d] + [Xm[h]]
        if stop:
            break
    X = np.zeros(k)
    for h in range(k):                                    # :163-165
        r_ = row[omega[h, 0]]
        nn = Xm[h].shape[0]
        X[h] = St[r_].V[omega[h, 1] - 1, :nn] @ Xm[h][:, 0] * Uaux[r_]
    return X, j


# ---------------------------------------------------------------------------
# multiple_frechet_eval.m / hessianfcn_exp.m / hessianfcn_fun.m (poles = inf)
# ---------------------------------------------------------------------------
def frechet_matrix_fun(name: str):
    """multiple_frechet_eval.m:60-77."""
    if name == "exp":
        return sla.expm
    if name == "sin":
        return sla.sinm
    if name == "cos":
        return sla.cosm
    if name == "log":
        return sla.logm
    if name == "sqrt":
        return sla.sqrtm
    if name == "sinh":
        return lambda M: (sla.expm(M) - sla.expm(-M)) / 2
    if name == "cosh":
        return lambda M: (sla.expm(M) + sla.expm(-M)) / 2
    raise ValueError(name)


def multiple_frechet_eval(A, omega, f="exp", tol=1e-12, it=None, poles=np.inf, debug=0):
    """[Um, Xm, Vm, row, col, iter] = multiple_frechet_eval(A, omega, f, tol, it, poles, debug)
    (multiple_frechet_eval.m:1-212); omega 1-based.  Returns Um/Vm as lists
    (bases with the last block dropped, :207-212), Xm per entry, and the
    row/col maps as dicts index -> position."""
    omega = np.asarray(omega, dtype=np.int64).reshape(-1, 2)
    n = A.shape[0]
    if it is None:
        it = min(100, n)
    k = omega.shape[0]
    AT = sp.csr_matrix(A).T.tocsr()                       # :55
    I0 = list(dict.fromkeys(omega[:, 0].tolist()))
    J0 = list(dict.fromkeys(omega[:, 1].tolist()))
    row = {t: i for i, t in enumerate(I0)}
    col = {t: i for i, t in enumerate(J0)}
    fM = frechet_matrix_fun(f)
    d = 3
    Xstop = [[] for _ in range(k)]
    notconverged = list(range(k))
    SA = [None] * len(I0); SB = [None] * len(J0)
    Uaux = np.zeros(len(I0)); Vaux = np.zeros(len(J0))
    Gm = [None] * len(I0); Hm = [None] * len(J0)
    Xm = [None] * k
    I, J = list(I0), list(J0)
    j = 0
    for j in range(1, it + 1):
        for h in I:                                       # :99-125
            r_ = row[h]
            if j == 1:
                U = np.zeros((n, 1)); U[h - 1, 0] = 1.0
                SA[r_] = arnoldi_krylov_start(A, U)
                Uaux[r_] = (SA[r_].V.T @ U)[0, 0]
            else:
                SA[r_] = arnoldi_krylov_extend(SA[r_])
            Gm[r_] = SA[r_].H[:-1, :]
        for h in J:                                       # :127-148
            c_ = col[h]
            if j == 1:
                V = np.zeros((n, 1)); V[h - 1, 0] = 1.0
                SB[c_] = arnoldi_krylov_start(AT, V)
                Vaux[c_] = (SB[c_].V.T @ V)[0, 0]
            else:
                SB[c_] = arnoldi_krylov_extend(SB[c_])
            Hm[c_] = SB[c_].H[:-1, :] @ np.linalg.inv(SB[c_].K[:-1, :])
        stop = True
        for h in list(notconverged):                      # :150-196
            G = Gm[row[omega[h, 0]]]
            Hh = Hm[col[omega[h, 1]]]
            Cm = np.zeros((j, j)); Cm[0, 0] = Uaux[row[omega[h, 0]]] * Vaux[col[omega[h, 1]]]
            Fm = np.block([[G, Cm], [np.zeros((Hh.shape[1], G.shape[1])), Hh.T]])
            Fm = fM(Fm)
            Xm[h] = Fm[:G.shape[0], G.shape[1]:]
            if j <= d:
                Xstop[h].append(Xm[h])
                stop = False
            else:
                nn = Xm[h].shape[0]
                old = np.zeros((nn, nn))
                o = Xstop[h][0]
                old[:o.shape[0], :o.shape[1]] = o
                err = np.linalg.norm(Xm[h] - old, 2)
                if err > tol:
                    stop = False
                else:
                    notconverged = [x for x in notconverged if x != h]
                    I = list(dict.fromkeys(omega[notconverged, 0].tolist()))
                    J = list(dict.fromkeys(omega[notconverged, 1].tolist()))
                Xstop[h] = Xstop[h][1:d] + [Xm[h]]
        if stop:
            break
    Um = [s.V[:, :-1] for s in SA]                        # :207-212
    Vm = [s.V[:, :-1] for s in SB]
    return Um, Xm, Vm, row, col, j


def hessianfcn(X, A, Omega, f="exp", tol=1e-12, it=None):
    """hessianfcn_exp.m:1-17 (f = exp) / hessianfcn_fun.m:1-17."""
    Omega = np.asarray(Omega, dtype=np.int64).reshape(-1, 2)
    n = A.shape[0]
    k = Omega.shape[0]
    XX = sp.csr_matrix((np.asarray(X, dtype=np.float64).ravel(), (Omega[:, 0] - 1, Omega[:, 1] - 1)),
                       shape=(n, n))
    XX = XX + XX.T
    At = (sp.csr_matrix(A) + XX).tocsr()
    Um, Xm, Vm, row, col, _ = multiple_frechet_eval(At, Omega, f, tol, it, np.inf, False)
    Hes = np.zeros((k, k))
    for jj in range(k):
        h, kk = Omega[jj]
        a, b = Xm[jj].shape
        for l in range(jj, k):
            Hes[jj, l] = Um[row[h]][Omega[l, 0] - 1, :a] @ Xm[jj] @ Vm[col[kk]][Omega[l, 1] - 1, :b]
        Hes[jj + 1:, jj] = Hes[jj, jj + 1:]
    return -2 * Hes


def exact_frechet(A, i, j, f="exp"):
    """Df(A)(e_i e_j') as the (1,2) block of f([A E; 0 A]) (dense; small n)."""
    n = A.shape[0]
    Ad = _full(A)
    E = np.zeros((n, n)); E[i - 1, j - 1] = 1.0
    F = frechet_matrix_fun(f)(np.block([[Ad, E], [np.zeros((n, n)), Ad]]))
    return F[:n, n:]

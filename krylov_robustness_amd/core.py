"""Host-side mirror of the reference's entry points over the C ABI.

Names, argument meaning and error behaviour follow the MATLAB functions in
/root/reference/functions (cited per function); device work happens in
libkrylov_hip.so.  Nothing here computes on the CPU except argument marshalling.
"""
from __future__ import annotations

import ctypes as C
import os
import warnings
from typing import Optional

import numpy as np

from . import _lib


class Context:
    """One HIP device + stream (kt_context_t)."""

    def __init__(self, device: Optional[int] = None):
        lib = _lib.load()
        if device is None:
            device = 0
        h = C.c_void_p()
        _lib.check(lib.kt_context_create(int(device), C.byref(h)))
        self._h = h
        self.device = device

    @property
    def handle(self):
        return self._h

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            _lib.load().kt_context_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    # ---- profiling (HIP events on the library stream) ----
    def profile(self, enable: bool = True):
        _lib.check(_lib.load().kt_profile_enable(self._h, 1 if enable else 0))

    def profile_reset(self):
        _lib.check(_lib.load().kt_profile_reset(self._h))

    def profile_read(self, kernel: int):
        n = C.c_int64()
        ms = C.c_double()
        _lib.check(_lib.load().kt_profile_read(self._h, kernel, C.byref(n), C.byref(ms)))
        return int(n.value), float(ms.value)

    def profile_read_width(self, kernel: int, width: int):
        """(launches, milliseconds) of `kernel` in sweeps of width P = width."""
        n = C.c_int64()
        ms = C.c_double()
        _lib.check(_lib.load().kt_profile_read_width(self._h, kernel, int(width), C.byref(n), C.byref(ms)))
        return int(n.value), float(ms.value)

    def profile_busy(self, kernel: int) -> float:
        """Milliseconds during which at least one profiled launch of `kernel`
        was in flight (union over the sweep lanes' streams)."""
        ms = C.c_double()
        _lib.check(_lib.load().kt_profile_busy(self._h, kernel, C.byref(ms)))
        return float(ms.value)

    def debug_delay(self, lane: int, microseconds: float):
        """Test hook (kt_debug_delay): keep sweep lane `lane`'s stream busy
        for `microseconds`; returns at once."""
        _lib.check(_lib.load().kt_debug_delay(self._h, int(lane), float(microseconds)))

    def yform_redone(self) -> int:
        """Sweeps of the y-form hot path recomputed by the explicit CGS2 sweep
        (cancellation guard / lucky breakdown), since context creation."""
        return self.stat(0)

    def stat(self, which: int) -> int:
        """kt_context_stat: 0 y-form sweeps redone, 1 fun_update dense
        fallbacks, 2 basis columns of the last fun_update, 3 expmv calls,
        4 Taylor terms those calls executed."""
        v = C.c_int64()
        _lib.check(_lib.load().kt_context_stat(self._h, int(which), C.byref(v)))
        return int(v.value)

    def fun_update_stats(self):
        """(dense fallbacks so far, projected size of the last fun_update)."""
        return self.stat(1), self.stat(2)


_default_ctx: Optional[Context] = None


def default_context() -> Context:
    global _default_ctx
    if _default_ctx is None:
        _default_ctx = Context()
    return _default_ctx


def device_count() -> int:
    c = C.c_int()
    _lib.check(_lib.load().kt_device_count(C.byref(c)))
    return int(c.value)


def _as_csc(A):
    import scipy.sparse as sp
    if not sp.issparse(A):
        A = sp.csc_matrix(np.asarray(A, dtype=np.float64))
    A = A.tocsc()
    A.sort_indices()
    if A.shape[0] != A.shape[1]:
        raise _lib.KrylovError(_lib.KT_ERR_NOT_SQUARE, "The matrix A should be square")
    return A


class DeviceMatrix:
    """Device-resident CSR/CSC of a symmetric A (kt_matrix_t)."""

    def __init__(self, A, ctx: Optional[Context] = None, check_symmetric: bool = False):
        self.ctx = ctx or default_context()
        A = _as_csc(A)
        self.n = A.shape[0]
        self.nnz = A.nnz
        colptr = np.ascontiguousarray(A.indptr, dtype=np.int64)
        rowind = np.ascontiguousarray(A.indices, dtype=np.int64)
        vals = np.ascontiguousarray(A.data, dtype=np.float64)
        h = C.c_void_p()
        lib = _lib.load()
        _lib.check(lib.kt_matrix_create_csc(
            self.ctx.handle, self.n,
            colptr.ctypes.data_as(C.POINTER(C.c_int64)),
            rowind.ctypes.data_as(C.POINTER(C.c_int64)),
            vals.ctypes.data_as(C.POINTER(C.c_double)),
            1 if check_symmetric else 0, C.byref(h)))
        self._h = h

    @property
    def handle(self):
        return self._h

    def info(self):
        """(n, nnz) of the current device matrix (nnz changes with edge edits)."""
        n = C.c_int64()
        nnz = C.c_int64()
        _lib.check(_lib.load().kt_matrix_info(self._h, C.byref(n), C.byref(nnz)))
        return int(n.value), int(nnz.value)

    def to_scipy(self):
        """The matrix as scipy CSC (reflects set_pairs / krylov_miobi edits)."""
        import scipy.sparse as sp
        n, nnz = self.info()
        colptr = np.zeros(n + 1, dtype=np.int64)
        rowind = np.zeros(max(nnz, 1), dtype=np.int64)
        vals = np.zeros(max(nnz, 1))
        _lib.check(_lib.load().kt_matrix_export_csc(
            self._h, colptr.ctypes.data_as(C.POINTER(C.c_int64)),
            rowind.ctypes.data_as(C.POINTER(C.c_int64)), vals.ctypes.data_as(C.POINTER(C.c_double))))
        return sp.csc_matrix((vals[:nnz], rowind[:nnz], colptr), shape=(n, n))

    def set_pairs(self, E, value):
        """A(i,j) = A(j,i) = value for the 1-based pairs E (value 0 deletes)."""
        E = np.asarray(E, dtype=np.int64).reshape(-1, 2)
        ei = np.ascontiguousarray(E[:, 0] - 1)
        ej = np.ascontiguousarray(E[:, 1] - 1)
        _lib.check(_lib.load().kt_matrix_set_pairs(
            self._h, E.shape[0], ei.ctypes.data_as(C.POINTER(C.c_int64)),
            ej.ctypes.data_as(C.POINTER(C.c_int64)), float(value)))
        self.n, self.nnz = self.info()

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            _lib.load().kt_matrix_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


def _dev(A, ctx=None) -> DeviceMatrix:
    return A if isinstance(A, DeviceMatrix) else DeviceMatrix(A, ctx)


def _fun_code(fun) -> int:
    if callable(fun):
        fun = getattr(fun, "__name__", str(fun))
    try:
        return _lib.FUN_CODES[str(fun)]
    except KeyError:
        raise _lib.KrylovError(_lib.KT_ERR_UNSUPPORTED, f"unsupported function handle {fun!r}")


def slq_quadforms(A, nprobes: int, m: int, seed: int = 0, fun="exp", probe_offset: int = 0,
                  block: int = 0, ctx: Optional[Context] = None):
    """Per-probe z_p' f(A) z_p for the global probe range [probe_offset,
    probe_offset + nprobes) by m-step Lanczos quadrature (SURVEY.md §8a a10,
    lanczos_krylov.m:73-115 with bs = 1).  Returns (sum, sum_sq, q[nprobes])."""
    D = _dev(A, ctx)
    q = np.zeros(max(int(nprobes), 1), dtype=np.float64)
    s1 = C.c_double()
    s2 = C.c_double()
    _lib.check(_lib.load().kt_slq_trace(
        D.handle, _fun_code(fun), int(m), int(seed) & 0xFFFFFFFFFFFFFFFF, int(probe_offset),
        int(nprobes), int(block), C.byref(s1), C.byref(s2), q.ctypes.data_as(C.POINTER(C.c_double))))
    return float(s1.value), float(s2.value), q[:nprobes]


def slq_submit(A, nprobes: int, m: int, seed: int = 0, fun="exp", probe_offset: int = 0,
               block: int = 0, ctx: Optional[Context] = None):
    """First half of slq_quadforms (kt_slq_submit): queue the probe sweeps on
    the device and return at once.  Returns a pending handle for
    slq_collect; at most two outstanding per context, collected in order."""
    D = _dev(A, ctx)
    t = C.c_int()
    _lib.check(_lib.load().kt_slq_submit(
        D.handle, _fun_code(fun), int(m), int(seed) & 0xFFFFFFFFFFFFFFFF, int(probe_offset),
        int(nprobes), int(block), C.byref(t)))
    return (D, int(t.value), int(nprobes))


def slq_collect(pending):
    """Second half (kt_slq_collect): wait for that submission's sweeps, host
    quadrature.  Returns what slq_quadforms returns: (sum, sum_sq, q)."""
    D, t, nprobes = pending
    q = np.zeros(max(nprobes, 1), dtype=np.float64)
    s1 = C.c_double()
    s2 = C.c_double()
    _lib.check(_lib.load().kt_slq_collect(D.handle, t, C.byref(s1), C.byref(s2),
                                          q.ctypes.data_as(C.POINTER(C.c_double))))
    return float(s1.value), float(s2.value), q[:nprobes]


def slq_plan(A, nprobes: int, ctx: Optional[Context] = None) -> int:
    """Probes per SpMM sweep that slq_quadforms uses with block=0."""
    D = _dev(A, ctx)
    b = C.c_int()
    _lib.check(_lib.load().kt_slq_plan(D.handle, int(nprobes), C.byref(b)))
    return int(b.value)


def slq_trace(A, nprobes: int, m: int, seed: int = 0, fun="exp", block: int = 0,
              ctx: Optional[Context] = None):
    """Plain-Hutchinson trace(f(A)) estimate with Lanczos quadrature."""
    s1, _, q = slq_quadforms(A, nprobes, m, seed, fun, 0, block, ctx)
    return s1 / max(nprobes, 1), q


# ---------------------------------------------------------------------------
# block-Krylov entry points (reference names and argument order)
# ---------------------------------------------------------------------------
def _dptr(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def _colmajor(a, rows=None):
    import scipy.sparse as sp
    if sp.issparse(a):  # e.g. U of edge2low_rank (the callers pass full(U))
        a = a.toarray()
    a = np.asarray(a, dtype=np.float64)
    if a.ndim == 1:
        a = a[:, None]
    return np.asfortranarray(a)


def normest(A, tol=1e-6, ctx: Optional[Context] = None) -> float:
    """MATLAB normest(A, tol) (2-norm power estimate), as called at
    fun_and_grad_krylov_exp.m:26."""
    D = _dev(A, ctx)
    out = C.c_double()
    _lib.check(_lib.load().kt_normest(D.handle, float(tol), C.byref(out)))
    return float(out.value)


def trace_fun_update(A, U, B, tol=1e-12, it=None, debug=0, fun="exp", ctx: Optional[Context] = None):
    """[Xm, iter, lucky] = trace_fun_update(A, U, B, tol, it, debug, fun)
    (trace_fun_update.m:1)."""
    D = _dev(A, ctx)
    U = _colmajor(U)
    B = _colmajor(np.atleast_2d(B))
    xm = C.c_double()
    itr = C.c_int()
    lk = C.c_int()
    name = getattr(fun, "__name__", fun) if callable(fun) else fun
    if callable(fun) and name not in _lib.FUN_CODES:
        # any elementwise handle (trace_fun_update.m:88 sum(fun(d1) - fun(d2))):
        # evaluated on the host eigenvalue vectors through kt_trace_fun_update_fn.
        # ctypes would print and drop an exception raised in the callback, so
        # it is kept here, reported to the library as a non-zero status (the
        # call aborts with KT_ERR_CALLBACK) and re-raised once the call returns.
        raised = []

        def _f(x, y, count, user):
            try:
                k = int(count)
                xs = np.ctypeslib.as_array(x, shape=(k,))
                fx = np.asarray(fun(xs.copy()), dtype=np.float64)
                if fx.shape != (k,):
                    raise ValueError(f"fun must map a length-{k} vector elementwise, got shape {fx.shape}")
                np.ctypeslib.as_array(y, shape=(k,))[:] = fx
                return 0
            except BaseException as e:  # noqa: BLE001 -- re-raised after the call
                raised.append(e)
                return 1
        cb = _lib.SCALAR_FN(_f)
        st = _lib.load().kt_trace_fun_update_fn(
            D.handle, U.shape[1], _dptr(U), _dptr(B), float(tol), int(it or 0),
            C.cast(cb, C.c_void_p), None, C.byref(xm), C.byref(itr), C.byref(lk))
        if raised:
            raise raised[0]
        _lib.check(st)
    else:
        _lib.check(_lib.load().kt_trace_fun_update(
            D.handle, U.shape[1], _dptr(U), _dptr(B), float(tol), int(it or 0), _fun_code(fun),
            C.byref(xm), C.byref(itr), C.byref(lk)))
    its = int(it) if it else min(100, D.n)
    if lk.value and debug:  # trace_fun_update.m:119-124
        warnings.warn("TRACE_FUN_UPDATE:: Detected lucky breakdown")
    if itr.value == its:  # :128-130
        warnings.warn("TRACE_FUN_UPDATE:: Reached maximum number of iterations")
    return float(xm.value), int(itr.value), int(lk.value)


def fun_update(A, U, B, fun="exp", tol=1e-12, it=None, debug=0, want_um=True,
               ctx: Optional[Context] = None, nargout=4):
    """[Xm, iter, lucky, Um] = fun_update(A, U, B, fun, tol, it, debug)
    (fun_update.m:1).  nargout = 4: the Arnoldi branch (:77-91) every caller
    in the reference uses.  nargout <= 3: the block-Lanczos branch (:69-76,
    kt_fun_update_lanczos), returning (Xm, iter, lucky); as in the reference
    a run that took three or more steps then fails at :137
    (Um(:, 1:size(Xm, 1)) on lanczos_krylov's 2-block window): IndexError."""
    D = _dev(A, ctx)
    U = _colmajor(U)
    B = _colmajor(np.atleast_2d(B))
    rk = U.shape[1]
    its = int(it or min(100, D.n))
    maxc = int(min(D.n, (its + 1) * rk))
    if nargout <= 3:
        Xm = np.zeros(maxc * maxc)
        nc = C.c_int64()
        itr = C.c_int()
        lk = C.c_int()
        _lib.check(_lib.load().kt_fun_update_lanczos(
            D.handle, rk, _dptr(U), _dptr(B), _fun_code(fun), float(tol), int(it or 0), maxc,
            _dptr(Xm), C.byref(nc), C.byref(itr), C.byref(lk)))
        if lk.value:  # fun_update.m:127-130
            warnings.warn("FUN_UPDATE:: Detected lucky breakdown")
        if itr.value == its:  # :133-135
            warnings.warn("FUN_UPDATE:: Reached maximum number of iterations")
        k = int(nc.value)
        if k > 2 * rk:  # :137 indexes the n x 2rk window with 1:size(Xm, 1)
            raise IndexError(f"fun_update.m:137: index exceeds the {2 * rk} columns of the Lanczos window "
                             f"(size(Xm, 1) = {k})")
        return Xm[:k * k].reshape(k, k, order="F"), int(itr.value), int(lk.value)
    Xm = np.zeros(maxc * maxc)
    Um = np.zeros(D.n * maxc) if want_um else None
    nc = C.c_int64()
    itr = C.c_int()
    lk = C.c_int()
    _lib.check(_lib.load().kt_fun_update(
        D.handle, rk, _dptr(U), _dptr(B), _fun_code(fun), float(tol), int(it or 0), maxc,
        _dptr(Xm), C.byref(nc), C.byref(itr), C.byref(lk), _dptr(Um) if want_um else None))
    if lk.value:  # fun_update.m:127-130
        warnings.warn("FUN_UPDATE:: Detected lucky breakdown")
    if itr.value == its:  # :133-135
        warnings.warn("FUN_UPDATE:: Reached maximum number of iterations")
    k = int(nc.value)
    X = Xm[:k * k].reshape(k, k, order="F")
    Umat = Um[:D.n * k].reshape(D.n, k, order="F") if want_um else None
    return X, int(itr.value), int(lk.value), Umat


def _omega(Omega):
    Om = np.asfortranarray(np.asarray(Omega, dtype=np.float64))
    if Om.ndim != 2 or Om.shape[1] != 2:
        raise _lib.KrylovError(_lib.KT_ERR_ARG, "Omega must be |Omega| x 2")
    return Om


def fun_and_grad_krylov_exp(X, A, Omega, eA, tol, it, debug=False, ctx: Optional[Context] = None):
    """[f, gr] = fun_and_grad_krylov_exp(X, A, Omega, eA, tol, it, debug)
    (fun_and_grad_krylov_exp.m:1)."""
    D = _dev(A, ctx)
    Om = _omega(Omega)
    X = np.ascontiguousarray(np.asarray(X, dtype=np.float64).ravel())
    eA = np.ascontiguousarray(np.asarray(eA, dtype=np.float64).ravel())
    gr = np.zeros(Om.shape[0])
    f = C.c_double()
    _lib.check(_lib.load().kt_fun_and_grad_krylov_exp(
        D.handle, Om.shape[0], _dptr(X), _dptr(Om), _dptr(eA), float(tol), int(it or 0),
        C.byref(f), _dptr(gr)))
    return float(f.value), gr


def fun_and_grad_krylov_fun(X, A, Omega, fun, dfun, dfA, tol, it, debug=False, fun_M=None,
                            ctx: Optional[Context] = None):
    """[f, gr] = fun_and_grad_krylov_fun(X, A, Omega, fun, dfun, dfA, tol, it, debug, fun_M)
    (fun_and_grad_krylov_fun.m:1)."""
    D = _dev(A, ctx)
    Om = _omega(Omega)
    X = np.ascontiguousarray(np.asarray(X, dtype=np.float64).ravel())
    dfA = np.ascontiguousarray(np.asarray(dfA, dtype=np.float64).ravel())
    gr = np.zeros(Om.shape[0])
    f = C.c_double()
    _lib.check(_lib.load().kt_fun_and_grad_krylov_fun(
        D.handle, Om.shape[0], _dptr(X), _dptr(Om), _fun_code(fun), _fun_code(dfun), _dptr(dfA),
        float(tol), int(it or 0), C.byref(f), _dptr(gr)))
    return float(f.value), gr


# ---------------------------------------------------------------------------
# mc_trace / trace_exp / expmv
# ---------------------------------------------------------------------------
def mc_trace(Afun, n=None, tol=1e-3, maxit=10, isAreal=0, debug=0, seed=0, fun="exp", m=30,
             A=None, ctx: Optional[Context] = None):
    """[tr, res, it] = mc_trace(Afun, n, tol, maxit, isAreal, debug) (mc_trace.m:1).
    Afun: a matrix / DeviceMatrix (mc_trace.m:32-34), or one of the strings
    "lanczos" (f(A) by m-step Lanczos) / "expmv" (expmv(1, A, .)) with A given."""
    if isinstance(Afun, str):
        kind = _lib.AFUN_CODES[Afun]
        D = _dev(A, ctx)
    else:
        kind = _lib.AFUN_CODES["matrix"]
        D = _dev(Afun, ctx)
    if n is not None and int(n) != D.n:
        raise _lib.KrylovError(_lib.KT_ERR_ARG, "n does not match the matrix")
    tr = C.c_double()
    res = C.c_double()
    it = C.c_int()
    _lib.check(_lib.load().kt_mc_trace(D.handle, kind, _fun_code(fun), int(m), float(tol), int(maxit),
                                       int(isAreal), int(seed) & 0xFFFFFFFFFFFFFFFF, C.byref(tr),
                                       C.byref(res), C.byref(it)))
    return float(tr.value), float(res.value), int(it.value)


def trace_exp(A, method="lanczos", m=30, seed=0, ctx: Optional[Context] = None) -> float:
    """tr = trace_exp(A) (trace_exp.m:1-7): mc_trace(Afun, n, 1e-4, 1000, 1),
    Afun = Lanczos-exp (default, the north-star evaluator) or expmv (the
    reference's own composition)."""
    D = _dev(A, ctx)
    tr = C.c_double()
    _lib.check(_lib.load().kt_trace_exp(D.handle, _lib.AFUN_CODES[method], int(m),
                                        int(seed) & 0xFFFFFFFFFFFFFFFF, C.byref(tr)))
    return float(tr.value)


def expmv(t, A, b, ctx: Optional[Context] = None):
    """[f, s, m, mv] = expmv(t, A, b, [], 'double') (expmv.m:1)."""
    D = _dev(A, ctx)
    B = _colmajor(b)
    F = np.zeros_like(B, order="F")
    s = C.c_int()
    mm = C.c_int()
    mv = C.c_int()
    _lib.check(_lib.load().kt_expmv(D.handle, float(t), B.shape[1], _dptr(B), _dptr(F), C.byref(s),
                                    C.byref(mm), C.byref(mv)))
    return F, int(s.value), int(mm.value), int(mv.value)


def lanczos_fmv(A, X, m=30, fun="exp", ctx: Optional[Context] = None):
    """f(A) X by per-column m-step Lanczos (the Lanczos-f Afun handle)."""
    D = _dev(A, ctx)
    X = _colmajor(X)
    Y = np.zeros_like(X, order="F")
    _lib.check(_lib.load().kt_lanczos_fmv(D.handle, _fun_code(fun), int(m), X.shape[1], _dptr(X),
                                          _dptr(Y)))
    return Y


def function_multiple_entries(A, omega, f="exp", tol=1e-12, it=None, poles=np.inf, debug=0,
                              ctx: Optional[Context] = None):
    """[X, iter] = function_multiple_entries(A, omega, f, tol, it, poles, debug)
    (function_multiple_entries.m:1); omega is (k x 2), 1-based as in MATLAB."""
    if not (np.isscalar(poles) and np.isinf(poles)):
        raise _lib.KrylovError(_lib.KT_ERR_UNSUPPORTED,
                               "FUNCTION_MULTIPLE_ENTRIES::Unsupported rational Krylov yet")
    D = _dev(A, ctx)
    om = np.asarray(omega, dtype=np.int64).reshape(-1, 2)
    oi = np.ascontiguousarray(om[:, 0] - 1)
    oj = np.ascontiguousarray(om[:, 1] - 1)
    X = np.zeros(om.shape[0])
    itr = C.c_int()
    _lib.check(_lib.load().kt_function_multiple_entries(
        D.handle, om.shape[0], oi.ctypes.data_as(C.POINTER(C.c_int64)),
        oj.ctypes.data_as(C.POINTER(C.c_int64)), _fun_code(f), float(tol), int(it or 0),
        _dptr(X), C.byref(itr)))
    if itr.value == (int(it) if it else min(100, D.n)):  # function_multiple_entries.m:158-161
        warnings.warn("FUNCTION_MULTIPLE_ENTRIES:: Reached maximum number of iterations")
    return X, int(itr.value)


def householder_qr(W, ctx: Optional[Context] = None):
    """[Q, R] = qr(W, 0) on the device (kt_householder_qr)."""
    ctx = ctx or default_context()
    W = np.asfortranarray(np.asarray(W, dtype=np.float64))
    n, bs = W.shape
    Q = np.zeros((n, bs), order="F")
    R = np.zeros((bs, bs), order="F")
    _lib.check(_lib.load().kt_householder_qr(ctx.handle, n, bs, _dptr(W), _dptr(Q), _dptr(R)))
    return Q, R


def frechet_entries(A, omega, targets, f="exp", tol=1e-12, it=None, ctx: Optional[Context] = None):
    """out[h, t] = Df(A)(e_i e_j')(p, q) for omega[h] = (i, j) and targets[t] =
    (p, q), all 1-based -- the entries multiple_frechet_eval.m:1 exposes through
    Um{row(i)} * Xm{h} * Vm{col(j)}'.  Returns (out, iter)."""
    D = _dev(A, ctx)
    om = np.asarray(omega, dtype=np.int64).reshape(-1, 2)
    tg = np.asarray(targets, dtype=np.int64).reshape(-1, 2)
    oi, oj = np.ascontiguousarray(om[:, 0] - 1), np.ascontiguousarray(om[:, 1] - 1)
    ti, tj = np.ascontiguousarray(tg[:, 0] - 1), np.ascontiguousarray(tg[:, 1] - 1)
    out = np.zeros((om.shape[0], tg.shape[0]), order="F")
    itr = C.c_int()
    p64 = C.POINTER(C.c_int64)
    _lib.check(_lib.load().kt_frechet_entries(
        D.handle, om.shape[0], oi.ctypes.data_as(p64), oj.ctypes.data_as(p64), _fun_code(f),
        float(tol), int(it or 0), tg.shape[0], ti.ctypes.data_as(p64), tj.ctypes.data_as(p64),
        _dptr(out), C.byref(itr)))
    if itr.value == (int(it) if it else min(100, D.n)):  # multiple_frechet_eval.m:202-204
        warnings.warn("MULTIPLE_FRECHET_EVAL:: Reached maximum number of iterations")
    return out, int(itr.value)


def hessianfcn(X, A, Omega, f="exp", tol=1e-12, it=None, ctx: Optional[Context] = None):
    """Hes = hessianfcn_exp(X, A, Omega, tol, it) / hessianfcn_fun(X, A, Omega, f, tol, it)
    (hessianfcn_exp.m:1, hessianfcn_fun.m:1)."""
    D = _dev(A, ctx)
    Om = _omega(Omega)
    X = np.ascontiguousarray(np.asarray(X, dtype=np.float64).ravel())
    k = Om.shape[0]
    H = np.zeros((k, k), order="F")
    _lib.check(_lib.load().kt_hessianfcn(D.handle, k, _dptr(X), _dptr(Om), _fun_code(f), float(tol),
                                         int(it or 0), _dptr(H)))
    return H


def hessianfcn_exp(X, A, Omega, tol=1e-12, it=None, ctx: Optional[Context] = None):
    """hessianfcn_exp.m:1."""
    return hessianfcn(X, A, Omega, "exp", tol, it, ctx)


def hessianfcn_fun(X, A, Omega, f, tol=1e-12, it=None, ctx: Optional[Context] = None):
    """hessianfcn_fun.m:1."""
    return hessianfcn(X, A, Omega, f, tol, it, ctx)


def eigs_leading(A, tol=0.0, maxit=0, ctx: Optional[Context] = None):
    """[u, lambda] = eigs(A, 1) for symmetric A on the device (kt_eigs_leading);
    returns (lambda, u) with ||u|| = 1, sum(u) >= 0."""
    D = _dev(A, ctx)
    n, _ = D.info()
    v = np.zeros(max(n, 1))
    lam = C.c_double()
    st = C.c_int()
    _lib.check(_lib.load().kt_eigs_leading(D.handle, float(tol), int(maxit), C.byref(lam), _dptr(v),
                                           C.byref(st)))
    return float(lam.value), v[:n]

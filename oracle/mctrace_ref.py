"""ctypes wrapper of oracle/libmctrace_ref.so (TEST INFRASTRUCTURE ONLY):
the C + OpenMP restatement of the reference's own trace_exp composition
(trace_exp.m:5-6 = mc_trace.m with the expmv.m Afun; select_taylor_degree.m,
normAm.m), used as the CPU baseline of bench.py's reference-composition leg."""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_PATH = os.path.join(os.environ.get("KT_ORACLE_DIR") or _HERE, "libmctrace_ref.so")  # (sanitizer builds: tools/sanitize.sh)
_lib = None


class Stats(C.Structure):
    _fields_ = [("calls", C.c_int64), ("terms", C.c_int64), ("mv", C.c_int64),
                ("t_select", C.c_double), ("t_terms", C.c_double), ("t_qr", C.c_double),
                ("t_proj", C.c_double), ("t_total", C.c_double)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(_PATH):
            subprocess.run(["make", "-s", "-C", _HERE], check=True)
        lib = C.CDLL(_PATH)
        P = C.c_void_p
        lib.mct_trace_exp.restype = C.c_int
        lib.mct_trace_exp.argtypes = [C.c_int64, P, P, P, C.c_double, C.c_int, C.c_uint64, P, C.c_int, C.c_int,
                                      C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(C.c_int),
                                      C.POINTER(Stats)]
        lib.mct_expmv_block.restype = C.c_int
        lib.mct_expmv_block.argtypes = [C.c_int64, P, P, P, C.c_double, C.c_int, P, P, P, C.c_int,
                                        C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int),
                                        C.POINTER(Stats)]
        lib.mct_round_host_times.restype = C.c_int
        lib.mct_round_host_times.argtypes = [C.c_int64, C.c_uint64, C.c_int, C.POINTER(C.c_double),
                                             C.POINTER(C.c_double)]
        _lib = lib
    return _lib


def _csr(A):
    import scipy.sparse as sp
    A = sp.csr_matrix(A)
    A.sort_indices()
    if (A != A.T).nnz:
        raise ValueError("mctrace_ref: A must be symmetric")
    if A.diagonal().any() or (A.data < 0).any():
        raise ValueError("mctrace_ref: A - mu I must be nonnegative (normAm.m's exact branch)")
    return (np.ascontiguousarray(A.indptr, dtype=np.int64), np.ascontiguousarray(A.indices, dtype=np.int32),
            np.ascontiguousarray(A.data, dtype=np.float64))


def _theta():
    from oracle import krylov_oracle as ko
    return np.ascontiguousarray(ko.theta_taylor(), dtype=np.float64)


def expmv(t, A, B, nthreads=0):
    """(F, s, m, mv, stats) = expmv(t, A, B, [], 'double') on the n x b block B."""
    rp, ci, va = _csr(A)
    B = np.ascontiguousarray(np.atleast_2d(np.asarray(B, dtype=np.float64).T).T)  # row-major n x b
    if B.shape[0] != A.shape[0]:
        B = B.reshape(A.shape[0], -1)
    n, b = B.shape
    F = np.zeros_like(B)
    th = _theta()
    s, m, mv = C.c_int(), C.c_int(), C.c_int()
    st = Stats()
    rc = load().mct_expmv_block(n, rp.ctypes.data, ci.ctypes.data, va.ctypes.data, float(t), b, B.ctypes.data,
                                F.ctypes.data, th.ctypes.data, int(nthreads), C.byref(s), C.byref(m), C.byref(mv),
                                C.byref(st))
    if rc != 0:
        raise RuntimeError(f"mct_expmv_block failed ({rc})")
    return F, s.value, m.value, mv.value, st.as_dict()


def trace_exp(A, seed=0, tol=1e-4, maxit=1000, nthreads=0, rounds_max=0):
    """(tr, res, it, stats) = mc_trace(@(x) expmv(1, A, x, [], 'double'), n, tol, maxit, 1)
    (trace_exp.m:5-6); rounds_max > 0 stops after that many rounds."""
    rp, ci, va = _csr(A)
    th = _theta()
    tr, res, it = C.c_double(), C.c_double(), C.c_int()
    st = Stats()
    rc = load().mct_trace_exp(A.shape[0], rp.ctypes.data, ci.ctypes.data, va.ctypes.data, float(tol), int(maxit),
                              int(seed) & 0xFFFFFFFFFFFFFFFF, th.ctypes.data, int(nthreads), int(rounds_max),
                              C.byref(tr), C.byref(res), C.byref(it), C.byref(st))
    if rc != 0:
        raise RuntimeError(f"mct_trace_exp failed ({rc})")
    return tr.value, res.value, it.value, st.as_dict()


def round_host_times(n, seed=0, nthreads=0):
    """(seconds of one qr(., 0) of an n x 10 block, of one projection
    X - Q (Q' X)): mc_trace's host work per round (mc_trace.m:45, :47)."""
    a, b = C.c_double(), C.c_double()
    if load().mct_round_host_times(int(n), int(seed), int(nthreads), C.byref(a), C.byref(b)) != 0:
        raise RuntimeError("mct_round_host_times failed")
    return a.value, b.value

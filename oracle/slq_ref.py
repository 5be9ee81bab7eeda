"""ctypes wrapper of oracle/libslq_ref.so (TEST INFRASTRUCTURE ONLY)."""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_PATH = os.path.join(os.environ.get("KT_ORACLE_DIR") or _HERE, "libslq_ref.so")  # (sanitizer builds: tools/sanitize.sh)
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(_PATH):
            build()
        lib = C.CDLL(_PATH)
        lib.slq_ref_trace.restype = C.c_double
        lib.slq_ref_trace.argtypes = [C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int,
                                      C.c_int64, C.c_int, C.c_uint64, C.c_int, C.c_int, C.c_void_p]
        lib.slq_ref_rademacher.restype = C.c_double
        lib.slq_ref_rademacher.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64]
        lib.slq_ref_tridiag_quad.restype = C.c_double
        lib.slq_ref_tridiag_quad.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_int]
        lib.slq_ref_max_threads.restype = C.c_int
        _lib = lib
    return _lib


FUN = {"exp": 0, "sinh": 1, "cosh": 2, "sin": 3, "cos": 4, "log": 5, "sqrt": 6}


def slq_trace(A, nprobes, m, seed=0, fun="exp", probe_offset=0, nthreads=0):
    """Returns (mean of quadforms, quadforms) for probes [offset, offset+nprobes)."""
    import scipy.sparse as sp
    A = sp.csr_matrix(A)
    A.sort_indices()
    rp = np.ascontiguousarray(A.indptr, dtype=np.int64)
    ci = np.ascontiguousarray(A.indices, dtype=np.int32)
    va = np.ascontiguousarray(A.data, dtype=np.float64)
    q = np.zeros(max(nprobes, 1))
    mean = load().slq_ref_trace(A.shape[0], rp.ctypes.data, ci.ctypes.data, va.ctypes.data,
                                int(nprobes), int(probe_offset), int(m), int(seed), FUN[fun],
                                int(nthreads), q.ctypes.data)
    return float(mean), q[:nprobes]


def max_threads():
    return int(load().slq_ref_max_threads())


def unit_quad(A, row0, nrows, m, t=(1.0,), nthreads=0):
    """e_i' exp(t_k A) e_i for rows [row0, row0 + nrows) by m-step Lanczos
    from e_i + Gauss quadrature (slq_ref_unit_quad); returns (nrows, len(t))."""
    import scipy.sparse as sp
    A = sp.csr_matrix(A)
    A.sort_indices()
    rp = np.ascontiguousarray(A.indptr, dtype=np.int64)
    ci = np.ascontiguousarray(A.indices, dtype=np.int32)
    va = np.ascontiguousarray(A.data, dtype=np.float64)
    tv = np.ascontiguousarray(t, dtype=np.float64)
    out = np.zeros((int(nrows), tv.size))
    lib = load()
    lib.slq_ref_unit_quad.restype = None
    lib.slq_ref_unit_quad(C.c_int64(A.shape[0]), C.c_void_p(rp.ctypes.data), C.c_void_p(ci.ctypes.data),
                          C.c_void_p(va.ctypes.data), C.c_int64(int(row0)), C.c_int64(int(nrows)), C.c_int(int(m)),
                          C.c_void_p(tv.ctypes.data), C.c_int(tv.size), C.c_int(int(nthreads)),
                          C.c_void_p(out.ctypes.data))
    return out

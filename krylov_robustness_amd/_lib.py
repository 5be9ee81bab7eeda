"""ctypes binding of libkrylov_hip.so (the C ABI declared in include/krylov_trace.h).

There is no fallback: if the in-tree shared library is missing or cannot be
loaded, every entry point raises ``KrylovLibraryError``.

If the process also uses torch, import torch FIRST: the library's ROCm
dependencies (libamdhip64.so.7, librocblas.so.5, librocsolver.so.0) then bind
to the copies torch already loaded (same SONAMEs) instead of a second runtime.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# KT_LIB: another build of the same library (tools' A/B of compile-time variants)
LIB_PATH = os.environ.get("KT_LIB") or os.path.join(_HERE, "libkrylov_hip.so")


class KrylovLibraryError(RuntimeError):
    pass


class KrylovError(RuntimeError):
    """A non-zero kt_status; .code holds the status, str() the library message."""

    def __init__(self, code: int, msg: str):
        super().__init__(msg)
        self.code = code


# kt_status
(KT_OK, KT_ERR_ARG, KT_ERR_HIP, KT_ERR_NOT_HERMITIAN, KT_ERR_NOT_SQUARE, KT_ERR_ALLOC, KT_ERR_UNSUPPORTED,
 KT_ERR_CALLBACK) = range(8)
# kt_afun (mc_trace.m's Afun kinds)
AFUN_CODES = {"matrix": 0, "lanczos": 1, "expmv": 2}
# kt_fun (fun_update.m:43-59)
FUN_CODES = {"exp": 0, "sinh": 1, "cosh": 2, "sin": 3, "cos": 4, "log": 5, "sqrt": 6}

_ctx_p = C.c_void_p
_mat_p = C.c_void_p
_i64p = C.POINTER(C.c_int64)
_dp = C.POINTER(C.c_double)
_ip = C.POINTER(C.c_int)

# kt_scalar_fn: y[i] = f(x[i]) for an elementwise handle outside kt_fun; 0 = ok
SCALAR_FN = C.CFUNCTYPE(C.c_int, _dp, _dp, C.c_int64, C.c_void_p)
# kt_reduce_fn: in-place sum of `count` doubles across ranks; 0 = ok
REDUCE_FN = C.CFUNCTYPE(C.c_int, _dp, C.c_int64, C.c_void_p)

# (name, restype, argtypes) -- every symbol include/krylov_trace.h declares
SIGNATURES = [
    ("kt_abi_version", C.c_int, []),
    ("kt_last_error", C.c_char_p, []),
    ("kt_device_count", C.c_int, [_ip]),
    ("kt_context_create", C.c_int, [C.c_int, C.POINTER(_ctx_p)]),
    ("kt_context_destroy", C.c_int, [_ctx_p]),
    ("kt_matrix_create_csc", C.c_int, [_ctx_p, C.c_int64, _i64p, _i64p, _dp, C.c_int, C.POINTER(_mat_p)]),
    ("kt_matrix_destroy", C.c_int, [_mat_p]),
    ("kt_matrix_info", C.c_int, [_mat_p, _i64p, _i64p]),
    ("kt_slq_trace", C.c_int, [_mat_p, C.c_int, C.c_int, C.c_uint64, C.c_int64, C.c_int64, C.c_int,
                               _dp, _dp, _dp]),
    ("kt_slq_submit", C.c_int, [_mat_p, C.c_int, C.c_int, C.c_uint64, C.c_int64, C.c_int64, C.c_int, _ip]),
    ("kt_slq_collect", C.c_int, [_mat_p, C.c_int, _dp, _dp, _dp]),
    ("kt_slq_plan", C.c_int, [_mat_p, C.c_int64, _ip]),
    ("kt_normest", C.c_int, [_mat_p, C.c_double, _dp]),
    ("kt_trace_fun_update", C.c_int, [_mat_p, C.c_int64, _dp, _dp, C.c_double, C.c_int, C.c_int,
                                      _dp, _ip, _ip]),
    ("kt_trace_fun_update_fn", C.c_int, [_mat_p, C.c_int64, _dp, _dp, C.c_double, C.c_int,
                                         C.c_void_p, C.c_void_p, _dp, _ip, _ip]),
    ("kt_fun_update", C.c_int, [_mat_p, C.c_int64, _dp, _dp, C.c_int, C.c_double, C.c_int,
                                C.c_int64, _dp, _i64p, _ip, _ip, _dp]),
    ("kt_fun_update_lanczos", C.c_int, [_mat_p, C.c_int64, _dp, _dp, C.c_int, C.c_double, C.c_int,
                                        C.c_int64, _dp, _i64p, _ip, _ip]),
    ("kt_fun_and_grad_krylov_exp", C.c_int, [_mat_p, C.c_int64, _dp, _dp, _dp, C.c_double, C.c_int,
                                             _dp, _dp]),
    ("kt_fun_and_grad_krylov_fun", C.c_int, [_mat_p, C.c_int64, _dp, _dp, C.c_int, C.c_int, _dp,
                                             C.c_double, C.c_int, _dp, _dp]),
    ("kt_mc_trace", C.c_int, [_mat_p, C.c_int, C.c_int, C.c_int, C.c_double, C.c_int, C.c_int,
                              C.c_uint64, _dp, _dp, _ip]),
    ("kt_mc_trace_sharded", C.c_int, [_mat_p, C.c_int, C.c_int, C.c_int, C.c_double, C.c_int, C.c_int,
                                      C.c_uint64, C.c_int, C.c_int, REDUCE_FN, C.c_void_p, _dp, _dp,
                                      _ip]),
    ("kt_trace_exp", C.c_int, [_mat_p, C.c_int, C.c_int, C.c_uint64, _dp]),
    ("kt_expmv", C.c_int, [_mat_p, C.c_double, C.c_int64, _dp, _dp, _ip, _ip, _ip]),
    ("kt_lanczos_fmv", C.c_int, [_mat_p, C.c_int, C.c_int, C.c_int64, _dp, _dp]),
    ("kt_trace_fun_update_pairs", C.c_int, [_mat_p, C.c_int64, _i64p, _i64p, _dp, C.c_double,
                                            C.c_double, C.c_int, C.c_int, _dp, _ip, _ip]),
    ("kt_krylov_miobi", C.c_int, [_mat_p, C.c_int, C.c_int64, _i64p, _i64p, C.c_double, C.c_int,
                                  C.c_int, C.c_double, _i64p, _i64p, _dp, _i64p]),
    ("kt_greedy_krylov_steps", C.c_int, [_mat_p, C.c_int, C.c_int64, C.c_int64, _i64p, _i64p, C.c_double,
                                         C.c_int, C.c_int, C.c_double, _i64p, _i64p, _dp, _i64p]),
    ("kt_matrix_set_pairs", C.c_int, [_mat_p, C.c_int64, _i64p, _i64p, C.c_double]),
    ("kt_matrix_export_csc", C.c_int, [_mat_p, _i64p, _i64p, _dp]),
    ("kt_function_multiple_entries", C.c_int, [_mat_p, C.c_int64, _i64p, _i64p, C.c_int, C.c_double,
                                               C.c_int, _dp, _ip]),
    ("kt_householder_qr", C.c_int, [_ctx_p, C.c_int64, C.c_int64, _dp, _dp, _dp]),
    ("kt_host_sym_eig", C.c_int, [C.c_int, _dp, _dp, _dp]),
    ("kt_host_tridiag_quad", C.c_int, [C.c_int, _dp, _dp, C.c_int, _dp, _dp]),
    ("kt_frechet_entries", C.c_int, [_mat_p, C.c_int64, _i64p, _i64p, C.c_int, C.c_double, C.c_int,
                                     C.c_int64, _i64p, _i64p, _dp, _ip]),
    ("kt_hessianfcn", C.c_int, [_mat_p, C.c_int64, _dp, _dp, C.c_int, C.c_double, C.c_int, _dp]),
    ("kt_eigs_leading", C.c_int, [_mat_p, C.c_double, C.c_int, _dp, _dp, _ip]),
    ("kt_profile_enable", C.c_int, [_ctx_p, C.c_int]),
    ("kt_profile_read", C.c_int, [_ctx_p, C.c_int, _i64p, _dp]),
    ("kt_profile_reset", C.c_int, [_ctx_p]),
    ("kt_profile_busy", C.c_int, [_ctx_p, C.c_int, _dp]),
    ("kt_debug_delay", C.c_int, [_ctx_p, C.c_int, C.c_double]),
    ("kt_profile_read_width", C.c_int, [_ctx_p, C.c_int, C.c_int, _i64p, _dp]),
    ("kt_context_stat", C.c_int, [_ctx_p, C.c_int, _i64p]),
    ("kt_host_threads", C.c_int, []),
]

_lib = None
_lock = threading.Lock()


def load():
    """Load (once) and return the CDLL; raise KrylovLibraryError if unavailable."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise KrylovLibraryError(
                f"{LIB_PATH} not found: build it with `make -C krylov_robustness_amd/csrc` "
                "or __graft_entry__.build() (no CPU fallback exists)")
        try:
            lib = C.CDLL(LIB_PATH)
        except OSError as e:  # pragma: no cover - depends on the box
            raise KrylovLibraryError(f"cannot load {LIB_PATH}: {e}") from e
        for name, res, args in SIGNATURES:
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


def check(status: int):
    if status != KT_OK:
        msg = load().kt_last_error()
        raise KrylovError(status, msg.decode() if msg else f"kt status {status}")


def source_digest() -> str:
    """sha256 (16 hex digits) of the sources libkrylov_hip.so is built from
    (krylov_robustness_amd/csrc/*.hip|*.cpp|*.h, include/krylov_trace.h):
    names the library build a profile was measured on (profiles/traffic.json
    records it; bench.py compares it with the tree it runs from)."""
    import glob
    import hashlib
    h = hashlib.sha256()
    root = os.path.dirname(_HERE)
    files = sorted(glob.glob(os.path.join(_HERE, "csrc", "*.hip")) + glob.glob(os.path.join(_HERE, "csrc", "*.cpp")) +
                   glob.glob(os.path.join(_HERE, "csrc", "*.h"))) + [os.path.join(root, "include", "krylov_trace.h")]
    for f in files:
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]

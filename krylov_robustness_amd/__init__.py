"""krylov_robustness_amd -- MI355X-native trace(f(A)) evaluator.

Drop-in for the Krylov trace / matrix-function hot path of
COMPiLELab/krylov_robustness (trace_exp, mc_trace, trace_fun_update,
fun_update, fun_and_grad_krylov_{exp,fun}).  The compute lives
in libkrylov_hip.so (HIP kernels for gfx950 + C++ host driver, C ABI in
include/krylov_trace.h); this package is the Python mirror of the reference
interface used by tests and bench.py.
"""
from ._lib import KrylovError, KrylovLibraryError, FUN_CODES, LIB_PATH
from .core import (Context, DeviceMatrix, default_context, device_count, expmv,
                   eigs_leading, frechet_entries, function_multiple_entries, hessianfcn, hessianfcn_exp,
                   hessianfcn_fun, householder_qr,
                   fun_and_grad_krylov_exp, fun_and_grad_krylov_fun, fun_update, lanczos_fmv,
                   mc_trace, normest, slq_collect, slq_plan, slq_quadforms, slq_submit, slq_trace, trace_exp,
                   trace_fun_update)
from .greedy import (compute_centrality, default_greedy_tol, edge2low_rank, find_top_edges,
                     find_top_missing_edges, greedy_krylov, krylov_miobi, krylov_miobi_sharded,
                     miobi_loop, select_extreme, trace_fun_update_pairs)
from . import datasets, matv73
from .dist import mc_trace_sharded, trace_exp_sharded
from .datasets import load_problem, load_unweighted, prepare_unweighted, prepare_weighted

__all__ = [
    "KrylovError", "KrylovLibraryError", "FUN_CODES", "LIB_PATH", "Context", "DeviceMatrix",
    "default_context", "device_count", "slq_plan", "slq_quadforms", "slq_submit", "slq_collect", "slq_trace", "normest",
    "trace_fun_update", "fun_update", "fun_and_grad_krylov_exp", "fun_and_grad_krylov_fun",
    "mc_trace", "trace_exp", "expmv", "lanczos_fmv", "trace_fun_update_pairs", "krylov_miobi",
    "greedy_krylov", "find_top_edges", "find_top_missing_edges", "compute_centrality",
    "default_greedy_tol", "krylov_miobi_sharded", "miobi_loop", "select_extreme", "function_multiple_entries", "householder_qr", "frechet_entries",
    "hessianfcn", "hessianfcn_exp", "hessianfcn_fun", "eigs_leading", "datasets", "matv73",
    "load_problem", "load_unweighted", "prepare_unweighted", "prepare_weighted",
    "mc_trace_sharded", "trace_exp_sharded", "edge2low_rank",
]

"""Config 5: where greedy_krylov's wall time goes -- the Python-side set-up
(host copy of A, symmetry check, Q, find_top_edges) vs the library call that
runs the k selection steps (kt_greedy_krylov_steps)."""
import ctypes as C
import os
import sys
import time

import torch  # noqa: F401
import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import krylov_robustness_amd as kra  # noqa: E402
from krylov_robustness_amd import _lib, greedy  # noqa: E402
from conftest import load_graph  # noqa: E402

A = load_graph("india")
ctx = kra.Context(0)
c = kra.compute_centrality(A)
D0 = kra.DeviceMatrix(A, ctx)
tol = kra.default_greedy_tol(D0, ctx=ctx)
k, Q = 50, 250
for rep in range(4):
    D = kra.DeviceMatrix(A, ctx)
    t0 = time.perf_counter()
    S = D.to_scipy()
    t1 = time.perf_counter()
    sym = greedy._is_symmetric(S)
    t2 = time.perf_counter()
    top = greedy.find_top_edges(S, c, Q + k, "min")
    t3 = time.perf_counter()
    T = np.asarray(top, dtype=np.int64).reshape(-1, 2)
    pi = np.ascontiguousarray(T[:, 0] - 1)
    pj = np.ascontiguousarray(T[:, 1] - 1)
    si = np.zeros(k, dtype=np.int64)
    sj = np.zeros(k, dtype=np.int64)
    rb = C.c_double()
    ns = C.c_int64()
    _lib.check(_lib.load().kt_greedy_krylov_steps(
        D.handle, k, Q, len(T), pi.ctypes.data_as(C.POINTER(C.c_int64)), pj.ctypes.data_as(C.POINTER(C.c_int64)),
        float(tol), 100, 0, 1.0, si.ctypes.data_as(C.POINTER(C.c_int64)), sj.ctypes.data_as(C.POINTER(C.c_int64)),
        C.byref(rb), C.byref(ns)))
    t4 = time.perf_counter()
    print(f"to_scipy {1e3*(t1-t0):.2f} ms, symmetry {1e3*(t2-t1):.2f}, find_top_edges {1e3*(t3-t2):.2f}, "
          f"library steps {1e3*(t4-t3):.2f} ms, rob {rb.value:.6f}", flush=True)

"""One trace_exp(A) with the reference's expmv Afun on dt_oregon A6 (for rocprofv3)."""
import os
import sys
import time

import torch  # noqa: F401

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import krylov_robustness_amd as kra  # noqa: E402
from conftest import load_graph  # noqa: E402

A = load_graph(sys.argv[1] if len(sys.argv) > 1 else "oregon_A6")
ctx = kra.Context(0)
D = kra.DeviceMatrix(A, ctx)
kra.trace_exp(D, method="expmv", seed=0, ctx=ctx)
t0 = time.perf_counter()
tr = kra.trace_exp(D, method="expmv", seed=0, ctx=ctx)
print(f"trace_exp expmv {tr:.16e} {time.perf_counter() - t0:.4f} s")

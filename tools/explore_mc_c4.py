"""Exploration: trace_exp.m's own structure (mc_trace + Afun) on the config-4
graph -- time per call, rounds, estimate.  Writes one JSON line per variant."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: F401,E402
import krylov_robustness_amd as kra  # noqa: E402
from krylov_robustness_amd import graphs  # noqa: E402

reps = int(os.environ.get("REPS", "5"))
variants = os.environ.get("VARIANTS", "lanczos30,lanczos20,expmv").split(",")
A = graphs.chung_lu(1_000_000, 10_000_000, gamma=2.5, seed=0)
ctx = kra.Context(0)
D = kra.DeviceMatrix(A, ctx)
for v in variants:
    kind = "expmv" if v == "expmv" else "lanczos"
    m = 30 if kind == "expmv" else int(v[len("lanczos"):])
    t0 = time.perf_counter()
    tr, res, it = kra.mc_trace(kind, None, 1e-4, 1000, 1, 0, seed=0, fun="exp", m=m, A=D, ctx=ctx)
    first = time.perf_counter() - t0
    ts = []
    for r in range(reps):
        t0 = time.perf_counter()
        tr2, res2, it2 = kra.mc_trace(kind, None, 1e-4, 1000, 1, 0, seed=r, fun="exp", m=m, A=D, ctx=ctx)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    print(json.dumps({"variant": v, "tr": tr, "res": res, "it": it, "first_s": first,
                      "ms": [round(t * 1e3, 2) for t in ts], "last": [tr2, res2, it2]}), flush=True)

"""BASELINE.json configs[0]: dt_oregon A6 (n = 10,860, nnz = 46,818),
trace(exp(A)) through mc_trace (functions/mc_trace.m:1-63).  Times on the
device, with the numpy oracle on the same inputs beside it:

  * one mc_trace round with the Lanczos-exp Afun (m = 20; 10 S + 10 Q + 10 G
    = 30 probes, maxit = 30 -> K = 1, mc_trace.m:41),
  * trace_exp as the reference composes it (functions/trace_exp.m:1-7:
    Afun = expmv(1, A, .), tol 1e-4, maxit 1000),
  * trace_exp with the Lanczos-exp Afun (tol 1e-4, maxit 1000),

each against the exact sum(exp(eig(A))) (test_weighted_exp_lbfgs.m:41) from
the golden fixtures.  One JSON line."""
import json
import os
import sys
import time

import torch  # noqa: F401  (torch's ROCm runtime first)

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import krylov_robustness_amd as kra  # noqa: E402
from conftest import load_graph  # noqa: E402
from oracle import krylov_oracle as ko  # noqa: E402


def best(fn, rep=5):
    out, t = None, []
    for _ in range(rep):
        t0 = time.perf_counter()
        out = fn()
        t.append(time.perf_counter() - t0)
    return out, min(t)


def once(fn):
    t0 = time.perf_counter()
    out = fn()
    return out, time.perf_counter() - t0


def main():
    with open(os.path.join(ROOT, "tests", "golden", "values.json")) as f:
        exact = json.load(f)["oregon_A6"]["exact_tr_exp"]
    A = load_graph("oregon_A6")
    ctx = kra.Context(0)
    D = kra.DeviceMatrix(A, ctx)
    n = A.shape[0]
    rel = lambda v: abs(v - exact) / abs(exact)

    (tr1, _, it1), t1 = best(lambda: kra.mc_trace("lanczos", n, 1e-4, 30, 1, seed=0, m=20, A=D, ctx=ctx))
    (tro1, _, ito1), to1 = once(lambda: ko.trace_exp_lanczos(A, m=20, tol=1e-4, maxit=30, seed=0))
    tr2, t2 = best(lambda: kra.trace_exp(D, method="expmv", seed=0, ctx=ctx), rep=3)
    tro2, to2 = once(lambda: ko.trace_exp(A, seed=0))
    tr3, t3 = best(lambda: kra.trace_exp(D, method="lanczos", m=20, seed=0, ctx=ctx), rep=3)
    out = {
        "workload": "dt_oregon A6 trace(exp(A)) via mc_trace (BASELINE configs[0])",
        "n": int(n), "nnz": int(A.nnz), "exact_tr_exp": exact,
        "mc_trace_lanczos_round": {"probes": 30, "m": 20, "rounds": it1, "oracle_rounds": ito1,
                                   "device_s": t1, "oracle_s": to1, "tr": tr1, "oracle_tr": tro1,
                                   "rel_vs_oracle": abs(tr1 - tro1) / abs(tro1), "rel_vs_exact": rel(tr1)},
        "trace_exp_expmv": {"device_s": t2, "oracle_s": to2, "tr": tr2, "oracle_tr": tro2,
                            "rel_vs_oracle": abs(tr2 - tro2) / abs(tro2), "rel_vs_exact": rel(tr2)},
        "trace_exp_lanczos": {"device_s": t3, "tr": tr3, "rel_vs_exact": rel(tr3)},
        "oracle": "numpy/scipy restatement (oracle/krylov_oracle.py), single thread, one run",
    }
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

"""Golden fixture for BASELINE config 4 (the bench workload) at full size:
the seeded Chung-Lu graph graphs.chung_lu(1e6, 1e7, 2.5, seed=0).  Build
container only; the GPU tests and bench.py read the JSON this writes.

  * the top-k spectrum (scipy eigsh, k = 16, tol = 0) and from it
    tr(exp(A)) = sum_i exp(lambda_i): the top-k sum is a lower bound and
    (n - k) exp(lambda_k) bounds the rest (every term is positive and at most
    exp(lambda_k)) -- the value trace_exp.m:5-6 estimates;
  * the C oracle's (oracle/slq_ref.c) per-probe quadratic forms
    q_p = z_p' exp(A) z_p by m = 30 Lanczos steps for one full evaluation,
    probes 0..1023 at the bench's first timed seed (0);
  * the numpy restatement of trace_exp.m with the Lanczos-exp Afun
    (mc_trace.m:42-58 structure, m = 30, tol 1e-4, maxit 1000, seed 0);
  * the same spectrum / forms for the weighted variant
    (graphs.symmetric_weights(A, seed=1), bench.py --weighted): spectrum,
    and the forms of probes 0..7.

  python tests/golden/make_config4_fixture.py [--skip-mc]
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np
import scipy.sparse.linalg as sla

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, ROOT)
from oracle import krylov_oracle as ko  # noqa: E402
from oracle import slq_ref  # noqa: E402
from krylov_robustness_amd import graphs  # noqa: E402

K_EIG = 16


def spectrum(A, label):
    t0 = time.time()
    w = sla.eigsh(A, k=K_EIG, which="LA", tol=0, return_eigenvectors=False)
    lam = np.sort(w)[::-1]
    n = A.shape[0]
    top = float(np.sum(np.exp(lam)))
    tail = float((n - K_EIG) * np.exp(lam[-1]))
    print(f"[{label}] eigsh {time.time() - t0:.1f}s lambda1 {lam[0]:.9f} lambda2 {lam[1]:.6f} "
          f"tr {top:.9e} tail bound {tail:.3e}", flush=True)
    return {"k": K_EIG, "lambda_desc": [float(x) for x in lam], "tr_exp_topk": top,
            "tail_bound": tail, "tr_exp_rel_uncertainty": tail / top,
            "method": "scipy.sparse.linalg.eigsh(A, k=16, which='LA', tol=0); "
                      "tr = sum exp(lambda_topk), 0 <= tr - that <= tail_bound"}


def main():
    skip_mc = "--skip-mc" in sys.argv
    t0 = time.time()
    A = graphs.chung_lu(1_000_000, 10_000_000, gamma=2.5, seed=0)
    print(f"graph {time.time() - t0:.1f}s n={A.shape[0]} nnz={A.nnz}", flush=True)
    rec = {"graph": "graphs.chung_lu(1_000_000, 10_000_000, gamma=2.5, seed=0)",
           "n": int(A.shape[0]), "nnz": int(A.nnz)}
    rec["spectrum"] = spectrum(A, "unit")
    t0 = time.time()
    N, m, seed = 1024, 30, 0
    _, q = slq_ref.slq_trace(A, N, m, seed=seed, fun="exp")
    print(f"slq oracle {N} probes {time.time() - t0:.1f}s mean {q.mean():.6e}", flush=True)
    rec["slq_exp"] = {"seed": seed, "m": m, "nprobes": N, "probe_offset": 0,
                      "q": [float(x) for x in q],
                      "estimate": float(q.mean()),
                      "stderr": float(q.std(ddof=1) / np.sqrt(N))}
    if not skip_mc:
        t0 = time.time()
        tr, res, it = ko.trace_exp_lanczos(A, m=30, tol=1e-4, maxit=1000, seed=0)
        print(f"mc_trace oracle {time.time() - t0:.1f}s tr {tr:.12e} res {res:.3e} it {it}", flush=True)
        rec["mc_trace_lanczos_exp"] = {"seed": 0, "m": 30, "tol": 1e-4, "maxit": 1000,
                                       "tr": tr, "res": res, "it": it}
    W = graphs.symmetric_weights(A, seed=1)
    rec["weighted"] = {"weights": "graphs.symmetric_weights(A, seed=1) (uniform [0.5, 1.5))",
                       "spectrum": spectrum(W, "weighted")}
    _, qw = slq_ref.slq_trace(W, 8, m, seed=seed, fun="exp")
    rec["weighted"]["slq_exp"] = {"seed": seed, "m": m, "nprobes": 8, "probe_offset": 0,
                                  "q": [float(x) for x in qw]}
    with open(os.path.join(HERE, "config4_values.json"), "w") as f:
        json.dump(rec, f, indent=1)
    print("wrote config4_values.json", flush=True)


if __name__ == "__main__":
    main()

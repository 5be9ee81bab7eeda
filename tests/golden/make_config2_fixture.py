"""Golden fixture for BASELINE config 2 at full size: the seeded
Erdos-Renyi graph graphs.erdos_renyi(100_000, 500_000, seed=0) (n = 100k,
nnz ~ 1M, unit weights).  Build container only; GPU tests and bench.py
--config er100k read the JSON this writes.

  * tr(exp(A)) with NO sampling error: the sum over all n rows of the
    diagonal entry e_i' exp(A) e_i, each by m = 30 Lanczos steps from the unit
    vector e_i + Gauss quadrature (oracle/slq_ref.c slq_ref_unit_quad; the
    recurrence of lanczos_krylov.m:30-115 with bs = 1).  On an ER spectrum
    (lambda_1 ~ 11.1) m = 30 nodes leave a quadrature error far below
    rounding; checked here by re-running a sample of rows (the 1,000 highest
    degrees and 1,000 random) at m = 45.
  * ||exp(A)||_F^2 = tr(exp(2A)) from the same runs (t = 2) and sum_i
    exp(A)_ii^2: the exact single-probe variance of the Rademacher Hutchinson
    estimator, 2 (||M||_F^2 - sum_i M_ii^2), so a test can bound an N-probe
    estimate by its true standard error (not a sample estimate);
  * the C oracle's per-probe forms q_p = z_p' exp(A) z_p (m = 30) of the
    bench's timed evaluations, probes 0..127 at seeds 0..4 (bench.py
    --config er100k, seeds 0..K-1);
  * a 8,192-probe C-oracle Hutchinson estimate (seed 1000) as an independent
    cross-check of the diagonal sum.

  python tests/golden/make_config2_fixture.py
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, ROOT)
from oracle import slq_ref  # noqa: E402
from krylov_robustness_amd import graphs  # noqa: E402

M = 30
N = 128


def main():
    t0 = time.time()
    A = graphs.erdos_renyi(100_000, 500_000, seed=0)
    n = A.shape[0]
    deg = np.diff(A.indptr)
    print(f"graph n={n} nnz={A.nnz} isolated={int((deg == 0).sum())} {time.time() - t0:.1f}s", flush=True)
    rec = {"graph": "graphs.erdos_renyi(100_000, 500_000, seed=0)", "n": int(n), "nnz": int(A.nnz),
           "lanczos_m": M}

    # per-probe forms of the bench's timed evaluations
    t0 = time.time()
    rec["slq_exp"] = {"m": M, "nprobes": N, "probe_offset": 0, "seeds": {}}
    for seed in range(5):
        _, q = slq_ref.slq_trace(A, N, M, seed=seed, fun="exp")
        rec["slq_exp"]["seeds"][str(seed)] = {"q": [float(x) for x in q], "estimate": float(q.mean()),
                                              "sample_stderr": float(q.std(ddof=1) / np.sqrt(N))}
    print(f"forms 5 x {N} probes {time.time() - t0:.1f}s", flush=True)

    # the exact diagonal, in chunks (progress lines)
    t0 = time.time()
    diag = np.zeros((n, 2))
    chunk = 5000
    for r0 in range(0, n, chunk):
        r1 = min(n, r0 + chunk)
        diag[r0:r1] = slq_ref.unit_quad(A, r0, r1 - r0, M, (1.0, 2.0))
        print(f"  diag rows {r1}/{n} {time.time() - t0:.0f}s", flush=True)
    d1, d2 = diag[:, 0], diag[:, 1]
    tr = float(np.sum(d1))
    fro2 = float(np.sum(d2))
    sumsq = float(np.sum(d1 * d1))
    var1 = 2.0 * (fro2 - sumsq)
    print(f"tr(exp A) = {tr:.15e}, ||exp A||_F^2 = {fro2:.6e}, var1 = {var1:.6e}, "
          f"stderr(N={N}) = {np.sqrt(var1 / N):.6e} ({np.sqrt(var1 / N) / tr:.3e} rel)", flush=True)

    # quadrature convergence on a sample of rows at m = 45
    rng = np.random.default_rng(0)
    sample = np.unique(np.concatenate([np.argsort(-deg, kind="stable")[:1000],
                                       rng.choice(n, 1000, replace=False)]))
    d45 = np.array([slq_ref.unit_quad(A, int(i), 1, 45, (1.0, 2.0))[0] for i in sample])
    conv = float(np.max(np.abs(d45 - diag[sample]) / np.abs(diag[sample])))
    print(f"m=45 vs m=30 on {sample.size} rows: max rel diff {conv:.3e}", flush=True)

    rec["exact"] = {
        "tr_exp": tr, "fro2_exp": fro2, "sum_diag_sq": sumsq,
        "hutchinson_var_per_probe": var1,
        "hutchinson_stderr_128": float(np.sqrt(var1 / N)),
        "rel_uncertainty": max(conv, 1e-12),
        "m45_sample_rows": int(sample.size), "m45_max_rel_diff": conv,
        "method": "sum over all n rows of e_i' exp(tA) e_i by m = 30 Lanczos from e_i + Gauss "
                  "quadrature (oracle/slq_ref.c slq_ref_unit_quad), t = 1 and 2; Rademacher "
                  "Hutchinson variance per probe = 2 (||M||_F^2 - sum M_ii^2), M = exp(A)"}

    t0 = time.time()
    big = 8192
    mean_big, qb = slq_ref.slq_trace(A, big, M, seed=1000, fun="exp")
    se_big = float(qb.std(ddof=1) / np.sqrt(big))
    print(f"{big}-probe oracle Hutchinson {mean_big:.12e} +- {se_big:.3e} "
          f"({(mean_big - tr) / se_big:+.2f} sigma from the diagonal sum) {time.time() - t0:.1f}s", flush=True)
    rec["hutchinson_8192"] = {"seed": 1000, "m": M, "estimate": float(mean_big), "sample_stderr": se_big,
                              "true_stderr": float(np.sqrt(var1 / big))}
    with open(os.path.join(HERE, "config2_values.json"), "w") as f:
        json.dump(rec, f, indent=1)
    print("wrote config2_values.json", flush=True)


if __name__ == "__main__":
    main()

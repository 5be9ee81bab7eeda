"""Golden fixture for fun_and_grad_krylov_fun over EVERY Omega of a fixed
sweep (not a hand-picked one): voltage India, Omega = 5 consecutive upper
edges starting at offsets 0, 5, 10, ..., 95 (triu(A, 1) in scipy's order),
X ~ U(-0.5, 1), dfA ~ N(0, 1) seeded per offset, tol = 1e-6 f(normest(A, 1e-2)),
it = 100, for (fun, dfun) = (sinh, cosh) and (cosh, sinh)
(Tests/test_weighted_sinh_lbfgs.m / _cosh_ settings).  Stores the oracle's
[f, gr], its trace_fun_update iteration count and the exact objective
-(sum f(eig(A + U B U')) - sum f(eig(A))) (dense eigvalsh) ->
omega_sweep_values.json.  Build container only; the GPU test reads the JSON.
Usage: python tests/golden/make_omega_sweep.py"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np
import scipy.sparse as sp

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from oracle import krylov_oracle as ko  # noqa: E402
from conftest import load_graph  # noqa: E402

OFFSETS = list(range(0, 100, 5))
K = 5


def sweep_inputs(A, offset):
    I, J = sp.triu(A, 1).nonzero()
    Om = np.stack([I[offset:offset + K] + 1, J[offset:offset + K] + 1], axis=1)
    rng = np.random.default_rng(1000 + offset)
    X = rng.uniform(-0.5, 1.0, K)
    dfA = rng.normal(size=K)
    return Om, X, dfA


def main():
    A = load_graph("india")
    n = A.shape[0]
    nrm = ko.normest(A, 1e-2)
    lam0 = np.linalg.eigvalsh(A.toarray())
    out = {"graph": "india", "n": n, "normest_1e-2": nrm, "k": K, "offsets": OFFSETS, "cases": {}}
    t0 = time.time()
    for fun, dfun in (("sinh", "cosh"), ("cosh", "sinh")):
        f_ = ko.scalar_fun(fun)
        tol = 1e-6 * f_(nrm)
        rows = []
        for off in OFFSETS:
            Om, X, dfA = sweep_inputs(A, off)
            fo, gro = ko.fun_and_grad_krylov_fun(X, A, Om, fun, dfun, dfA, tol, 100)
            U, B = ko.lowrank_from_edges(X, Om, n)
            Ad = A.toarray() + U @ B @ U.T
            lam1 = np.linalg.eigvalsh(0.5 * (Ad + Ad.T))
            fx = -(np.sum(f_(lam1)) - np.sum(f_(lam0)))
            rows.append({"offset": off, "Omega": Om.tolist(), "X": X.tolist(), "dfA": dfA.tolist(),
                         "f": fo, "gr": list(map(float, gro)), "exact_f": float(fx)})
            print(f"{fun} offset {off}: oracle {fo:.12e} exact {fx:.12e} "
                  f"rel {abs(fo - fx) / abs(fx):.2e} ({time.time() - t0:.0f} s)", flush=True)
        out["cases"][fun] = {"dfun": dfun, "tol": tol, "tol_f": tol * f_(nrm), "rows": rows}
    with open(os.path.join(HERE, "omega_sweep_values.json"), "w") as fh:
        json.dump(out, fh, indent=0)


if __name__ == "__main__":
    main()

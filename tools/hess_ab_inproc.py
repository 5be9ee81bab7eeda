"""hessianfcn_exp A/B inside ONE process (bench_hessian's workload: voltage India,
|Omega| = 30, tol 1e-8 exp(normest)), modes alternating call by call; reports
whether every mode's Hessian is bit-identical to mode 0's.
Usage: python tools/hess_ab_inproc.py REPS VAR=VAL[,VAR=VAL] ..."""
import os
import sys
import time

import torch  # noqa: F401
import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import krylov_robustness_amd as kra  # noqa: E402
from conftest import load_graph  # noqa: E402

reps = int(sys.argv[1])
modes = [dict(kv.split("=") for kv in m.split(",")) for m in sys.argv[2:]]
A = load_graph("india")
ctx = kra.Context(0)
D = kra.DeviceMatrix(A, ctx)
tol = 1e-8 * np.exp(kra.normest(D, 1e-2, ctx=ctx))
c = kra.compute_centrality(A)
E = kra.find_top_edges(A, c, 100, "min")
temp, _ = kra.function_multiple_entries(D, E, "exp", tol, 100, ctx=ctx)
ind = np.argsort(-temp, kind="stable")[:30]
Om = E[ind]
w = np.asarray(A[Om[:, 0] - 1, Om[:, 1] - 1]).ravel()
X = np.random.default_rng(5).uniform(-0.5, 1.0, size=30) * w
if X.sum() > 10:
    X *= 10 / X.sum()
times = [[] for _ in modes]
outs = [None] * len(modes)
for r in range(reps):
    for i, m in enumerate(modes):
        saved = {k: os.environ.get(k) for k in m}
        os.environ.update(m)
        t0 = time.perf_counter()
        H = kra.hessianfcn_exp(X, D, Om, tol, 100, ctx=ctx)
        times[i].append(time.perf_counter() - t0)
        outs[i] = np.array(H)
        for k, v in saved.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v
for i, m in enumerate(modes):
    t = np.array(times[i][2:]) * 1e3
    print(f"hessianfcn_exp india {m}: median {np.median(t):.3f} ms, min {t.min():.3f} (calls 3..{reps}), "
          f"bit-identical to mode 0: {np.array_equal(outs[i], outs[0])}", flush=True)

"""Config 3 fun_and_grad_krylov_fun A/B inside ONE process: the named env
settings alternate call by call (every setting the libraries read per call),
so box-to-box and process-to-process drift cancels.  Usage:
python tools/fg_ab_inproc.py REPS VAR=VAL[,VAR=VAL] VAR=VAL[,...] ..."""
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
A = load_graph("hawaii")
ctx = kra.Context(0)
D = kra.DeviceMatrix(A, ctx)
nrm = kra.normest(D, 1e-2, ctx=ctx)
c = kra.compute_centrality(A)
E = kra.find_top_edges(A, c, 100, "min")
temp, _ = kra.function_multiple_entries(D, E, "cosh", 1e-6 * np.cosh(nrm), 100, ctx=ctx)
ind = np.argsort(-temp, kind="stable")[:30]
Om, dfA = E[ind], temp[ind]
X = np.random.default_rng(11).uniform(-0.5, 1.0, size=30)
if X.sum() > 10:
    X *= 10 / X.sum()
times = [[] for _ in modes]
fs = [None] * len(modes)
for r in range(reps):
    for i, m in enumerate(modes):
        saved = {k: os.environ.get(k) for k in m}
        os.environ.update(m)
        t0 = time.perf_counter()
        f, gr = kra.fun_and_grad_krylov_fun(X, D, Om, "sinh", "cosh", dfA, 1e-6 * np.sinh(nrm), 100, ctx=ctx)
        times[i].append(time.perf_counter() - t0)
        fs[i] = f
        for k, v in saved.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v
for i, m in enumerate(modes):
    t = np.array(times[i][2:]) * 1e3
    print(f"{m}: median {np.median(t):.3f} ms, min {t.min():.3f}, mean {t.mean():.3f} (calls 3..{reps}), f {fs[i]:.12f}")

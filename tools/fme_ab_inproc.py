"""function_multiple_entries A/B inside ONE process (config 3's call: Hawaii LCC,
100 top 'min' edges, cosh, tol 1e-6 cosh(normest)), modes alternating call by
call; asserts every mode returns bit-identical entries and iteration counts.
Usage: python tools/fme_ab_inproc.py REPS VAR=VAL[,VAR=VAL] ..."""
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
graph = os.environ.get("KT_AB_GRAPH", "hawaii")
A = load_graph(graph)
ctx = kra.Context(0)
D = kra.DeviceMatrix(A, ctx)
nrm = kra.normest(D, 1e-2, ctx=ctx)
c = kra.compute_centrality(A)
E = kra.find_top_edges(A, c, 100, "min")
times = [[] for _ in modes]
outs = [None] * len(modes)
for r in range(reps):
    for i, m in enumerate(modes):
        saved = {k: os.environ.get(k) for k in m}
        os.environ.update(m)
        t0 = time.perf_counter()
        X, it = kra.function_multiple_entries(D, E, "cosh", 1e-6 * np.cosh(nrm), 100, ctx=ctx)
        times[i].append(time.perf_counter() - t0)
        outs[i] = (np.array(X), it)
        for k, v in saved.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v
for i, m in enumerate(modes):
    t = np.array(times[i][2:]) * 1e3
    same = np.array_equal(outs[i][0], outs[0][0]) and outs[i][1] == outs[0][1]
    print(f"{graph} {m}: median {np.median(t):.3f} ms, min {t.min():.3f} (calls 3..{reps}), iter {outs[i][1]}, "
          f"bit-identical to mode 0: {same}", flush=True)

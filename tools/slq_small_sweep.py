"""Config 3's probe pass (Hawaii LCC, 256 probes, m=30, sinh is exp-cost) over probes per
sweep P x sweep lanes, in one process (KT_SLQ_LANES is read per call); median of 15 calls each."""
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

g = sys.argv[1] if len(sys.argv) > 1 else "hawaii"
A = load_graph(g)
ctx = kra.Context(0)
D = kra.DeviceMatrix(A, ctx)
print(g, "n", A.shape[0], "plan P", kra.slq_plan(D, 256, ctx=ctx), flush=True)
ref = None
for P in (16, 32, 64, 128):
    for lanes in (1, 2, 3):
        os.environ["KT_SLQ_LANES"] = str(lanes)
        t = []
        for r in range(17):
            t0 = time.perf_counter()
            s1, s2, q = kra.slq_quadforms(D, 256, 30, seed=7, fun="sinh", block=P, ctx=ctx)
            t.append(time.perf_counter() - t0)
        if ref is None:
            ref = q.copy()
        print(f"P {P:4d} lanes {lanes}: median {1e3 * np.median(t[2:]):.3f} ms  max rel vs first {np.abs(q - ref).max() / np.abs(ref).max():.1e}",
              flush=True)

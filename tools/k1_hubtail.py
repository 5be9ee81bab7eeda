"""Is K1 bounded by its hub-row tail?  K1 (isolated, one lane, P = 16) on the
bench's Chung-Lu graph vs graphs with the same n and nnz but the maximum
degree capped (no / fewer long rows)."""
import os
import sys
import time

import torch  # noqa: F401
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import krylov_robustness_amd as kra  # noqa: E402
from krylov_robustness_amd import graphs  # noqa: E402

os.environ["KT_SLQ_LANES"] = "1"
import numpy as np  # noqa: E402
for cap in [None, 1000, 256, 64]:
    A = graphs.chung_lu(1_000_000, 10_000_000, seed=0, max_degree=cap)
    deg = np.diff(A.indptr)
    ctx = kra.Context(0)
    D = kra.DeviceMatrix(A, ctx)
    kra.slq_quadforms(D, 16, 4, seed=0, block=16, ctx=ctx)
    ctx.profile_reset(); ctx.profile(True)
    kra.slq_quadforms(D, 64, 30, seed=0, block=16, ctx=ctx)
    ctx.profile(False)
    l1, ms1 = ctx.profile_read(0)
    print(f"cap {cap}: max deg {deg.max()} rows>64 {(deg > 64).sum()} nnz {A.nnz}  K1 {ms1 / l1 * 1e3:.1f} us",
          flush=True)
    del D, ctx

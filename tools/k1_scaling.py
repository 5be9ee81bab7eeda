"""K1 cost per gathered nonzero vs graph size (same average degree 10,
Chung-Lu, P = 16): separates Infinity-Cache-resident gathers (small tables)
from HBM-served ones.  Prints one line per n."""
import os
import sys
import time

import torch  # noqa: F401
import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, ROOT)
import krylov_robustness_amd as kra  # noqa: E402
from krylov_robustness_amd import graphs  # noqa: E402

P = int(os.environ.get("P", "16"))
ctx = kra.Context(0)
for n in [125_000, 250_000, 500_000, 1_000_000, 2_000_000]:
    A = graphs.chung_lu(n, 10 * n, seed=0)
    D = kra.DeviceMatrix(A, ctx)
    kra.slq_quadforms(D, P, 4, seed=0, block=P, ctx=ctx)
    ctx.profile_reset(); ctx.profile(True)
    kra.slq_quadforms(D, 4 * P, 30, seed=0, block=P, ctx=ctx)
    ctx.profile(False)
    l1, ms1 = ctx.profile_read(0)
    l2, ms2 = ctx.profile_read(1)
    k1 = ms1 / l1 * 1e3
    k2 = ms2 / l2 * 1e3
    gath = A.nnz * 8 * P
    print(f"n={n:8d} nnz={A.nnz:9d} table={8*n*P/2**20:7.1f} MiB  K1 {k1:8.1f} us  "
          f"gather-rate {gath/k1/1e6:7.0f} GB/s  ns/nnz {k1*1e3/A.nnz:6.3f}  K2 {k2:7.1f} us "
          f"({32*n*P/k2/1e6:6.0f} GB/s)", flush=True)
    D.close()

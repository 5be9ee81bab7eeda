"""Time the y-form pass k_spmm_lanczos<16> alone on the bench workload (Chung-Lu
n = 1M, nnz = 10M, one lane, 4 sweeps x m = 30 steps), with the library named
by KT_LIB -- the normal build or a diagnostic build of the pass
(build/diagN/libkrylov_hip.so, -DKT_KY_DIAG=N: 1 = gathers + own row, 2 =
gathers only, 3 = row streams only; their numbers are wrong by construction,
only the launch durations mean anything).  Prints one JSON line.
Usage: KT_LIB=... python tools/ky_diag.py TAG"""
import json
import os
import sys

os.environ["KT_SLQ_LANES"] = "1"
os.environ["KT_SLQ_YFORM"] = "1"
import torch  # noqa: F401,E402  (torch's HIP runtime first)

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, ROOT)
import krylov_robustness_amd as kra  # noqa: E402
from krylov_robustness_amd import graphs  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else "normal"
A = graphs.chung_lu(1_000_000, 10_000_000, gamma=2.5, seed=0)
ctx = kra.Context(0)
D = kra.DeviceMatrix(A, ctx)
P = 16
m = 30
kra.slq_quadforms(D, 2 * P, m, seed=5, block=P, ctx=ctx)  # warm-up
res = []
for rep in range(3):
    ctx.profile_reset()
    ctx.profile(True)
    kra.slq_quadforms(D, 4 * P, m, seed=777, block=P, ctx=ctx)
    ctx.profile(False)
    l1, ms1 = ctx.profile_read(0)
    res.append(ms1 / l1 * 1e3)
print(json.dumps({"variant": tag, "lib": kra.LIB_PATH, "launches": l1, "avg_launch_us": res,
                  "best_us": min(res)}), flush=True)

"""trace_exp with the expmv Afun (the reference composition, trace_exp.m:5-6)
on the bench graph (config 4: Chung-Lu n = 1M), serial (KT_TWIN=0,
KT_MC_SPEC=0), for a rocprofv3 kernel trace:
  rocprofv3 --kernel-trace --stats -d OUT -o c4 -- python3 tools/expmv_c4.py
Prints the call's time, expmv calls and Taylor terms."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["KT_TWIN"] = "0"
os.environ["KT_MC_SPEC"] = "0"


def main():
    import torch  # noqa: F401
    import krylov_robustness_amd as kra
    from krylov_robustness_amd import graphs
    A = graphs.chung_lu(1_000_000, 10_000_000, gamma=2.5, seed=0)
    ctx = kra.Context(0)
    D = kra.DeviceMatrix(A, ctx)
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    for r in range(reps):
        c0, k0 = ctx.stat(3), ctx.stat(4)
        t0 = time.perf_counter()
        tr, res, it = kra.mc_trace("expmv", None, 1e-4, 1000, 1, 0, seed=r, A=D, ctx=ctx)
        dt = time.perf_counter() - t0
        print(json.dumps({"seed": r, "ms": round(dt * 1e3, 2), "tr": tr, "rounds": it,
                          "expmv_calls": ctx.stat(3) - c0, "taylor_terms": ctx.stat(4) - k0,
                          "us_per_term": round(dt * 1e6 / max(ctx.stat(4) - k0, 1), 1)}), flush=True)


if __name__ == "__main__":
    main()

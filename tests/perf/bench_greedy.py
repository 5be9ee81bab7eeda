"""Config 5 (BASELINE.json configs[4] / SURVEY.md §8d): greedy_krylov on the
India voltage graph, break mode, 'min' order, k = 50, Q = min(nnz/2 - k, 250),
tol = 1e-6 * exp(normest(A, 1e-2)), it = 100 (Tests/test_unweighted_break.m:15-20,
:56, :72-74).  Times the device path end to end and the numpy oracle on a
bounded number of greedy steps (--cpu-steps), prints one JSON line."""
import argparse
import json
import os
import sys
import time

import torch  # noqa: F401  (load torch's ROCm runtime first)
import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import krylov_robustness_amd as kra  # noqa: E402
from conftest import load_graph, load_v73_graph  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--graph", default="india")
    ap.add_argument("--k", type=int, default=50)
    ap.add_argument("--Q", type=int, default=250)
    ap.add_argument("--cpu-steps", type=int, default=2)
    ap.add_argument("--repeat", type=int, default=3)
    ap.add_argument("--miobi", default="break", choices=["break", "make"])
    a = ap.parse_args()
    # the Misc MAT v7.3 graphs (test_unweighted_make.m:41-52 preparation)
    A = load_v73_graph(a.graph) if a.graph in ("drugs", "as_735", "collegemsg") else load_graph(a.graph)
    c = kra.compute_centrality(A)
    ctx = kra.Context(0)
    Q = int(min(A.nnz // 2 - a.k, a.Q))  # test_unweighted_make.m:70
    D0 = kra.DeviceMatrix(A, ctx)
    tol = kra.default_greedy_tol(D0, ctx=ctx)
    kra.greedy_krylov(kra.DeviceMatrix(A, ctx), 1, Q, c, "min", tol, 100, miobi=a.miobi, ctx=ctx)  # warm-up
    times = []
    for _ in range(a.repeat):
        D = kra.DeviceMatrix(A, ctx)
        t0 = time.perf_counter()
        edges, rob, _ = kra.greedy_krylov(D, a.k, Q, c, "min", tol, 100, miobi=a.miobi, ctx=ctx)
        times.append(time.perf_counter() - t0)
    gpu_s = min(times)
    out = {"workload": f"greedy_krylov {a.graph} {a.miobi} k={a.k} Q={Q}", "n": A.shape[0],
           "nnz": A.nnz, "gpu_seconds": gpu_s, "gpu_seconds_all": times,
           "candidate_evals_per_s": a.k * Q / gpu_s, "rob_variation": rob,
           "first_edges": edges[:5].tolist()}
    if a.cpu_steps > 0:
        from oracle import krylov_oracle as ko
        t0 = time.perf_counter()
        eo, ro, _ = ko.greedy_krylov(A, a.cpu_steps, Q, c, "min", tol, 100, miobi=a.miobi)
        cpu = time.perf_counter() - t0
        out.update({"cpu_oracle_steps": a.cpu_steps, "cpu_oracle_seconds": cpu,
                    "cpu_oracle_seconds_per_step": cpu / a.cpu_steps,
                    "cpu_edges_match_prefix": bool(np.array_equal(eo, edges[:a.cpu_steps]))})
    print(json.dumps(out))


if __name__ == "__main__":
    main()

"""Drive l2sim.c on the bench graph (Chung-Lu n = 1M, nnz = 10M, hubs-first
relabelling) with different row -> XCD schedules.  CPU-only modelling tool:
python tools/l2sim/run.py [--n N] [--nnz NNZ]"""
import argparse
import ctypes as C
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))


def load():
    lib = C.CDLL(os.path.join(HERE, "libl2sim.so"))
    lib.simulate.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int,
                             C.c_int, C.c_int, C.c_void_p, C.c_int]
    return lib


def hub_relabel(A):
    deg = np.diff(A.indptr)
    new2old = np.argsort(-deg, kind="stable")
    old2new = np.empty_like(new2old)
    old2new[new2old] = np.arange(A.shape[0])
    B = A[new2old][:, new2old].tocsr()
    B.sort_indices()
    return B


def run(lib, A, order, xoff, P=16, inflight=2048, l2=4 << 20, bypass=0):
    out = np.zeros(6, dtype=np.int64)
    rp = np.ascontiguousarray(A.indptr, dtype=np.int64)
    col = np.ascontiguousarray(A.indices, dtype=np.int32)
    order = np.ascontiguousarray(order, dtype=np.int32)
    xoff = np.ascontiguousarray(xoff, dtype=np.int64)
    lib.simulate(A.shape[0], rp.ctypes.data, col.ctypes.data, order.ctypes.data, xoff.ctypes.data,
                 len(xoff) - 1, 8 * P, l2, inflight, out.ctypes.data, bypass)
    g, gh, s, sh, c, ch = [int(v) for v in out]
    miss_lines = (g - gh) + (s - sh) + (c - ch) / 1.0
    return {"gather_hit": gh / g, "stream_hit": sh / s, "miss_GB": miss_lines * 128 / 1e9,
            "gather_miss_GB": (g - gh) * 128 / 1e9}


def baseline_schedule(A, P=16, bpc=4, ncu=256, long_thresh=64):
    n = A.shape[0]
    deg = np.diff(A.indptr)
    long_rows = np.where(deg > long_thresh)[0]
    long_rows = long_rows[np.argsort(-deg[long_rows], kind="stable")]
    waves = 8
    lblocks = min((len(long_rows) + waves - 1) // waves, ncu * 2)
    gpw = 16  # GeoK1 at P = 16: 4 lanes x 32 B per row
    grid = min((n + 63) // 64, ncu * bpc)
    xcd_rows = [[] for _ in range(8)]
    # long rows: li = blockIdx * WAVES + wave, stride lblocks * WAVES
    for li, r in enumerate(long_rows):
        b = (li // waves) % lblocks
        xcd_rows[b % 8].append((li // (lblocks * waves), r))
    short = np.where(deg <= long_thresh)[0]
    per_round = grid * waves * gpw
    rnd = short // per_round
    sb = (short % per_round) // (waves * gpw)
    x = (sb + lblocks) % 8
    lists = []
    for k in range(8):
        lr = [r for _, r in sorted(xcd_rows[k])]
        sel = short[x == k]
        lists.append(np.concatenate([np.array(lr, dtype=np.int64), sel[np.lexsort((sel, rnd[x == k]))]]))
    order = np.concatenate(lists)
    xoff = np.concatenate([[0], np.cumsum([len(l) for l in lists])])
    return order, xoff


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--nnz", type=int, default=10_000_000)
    ap.add_argument("--inflight", type=int, default=2048)
    ap.add_argument("--schedules", default="baseline")
    ap.add_argument("--bypass", type=int, default=0, help="1: row streams skip L2, 2: CSR skips L2, 3: both")
    args = ap.parse_args()
    from krylov_robustness_amd import graphs
    t0 = time.time()
    A = graphs.chung_lu(args.n, args.nnz, gamma=2.5, seed=0)
    A = hub_relabel(A)
    print(f"graph n={A.shape[0]} nnz={A.nnz} ({time.time() - t0:.1f} s)", flush=True)
    lib = load()
    import schedules
    for name in args.schedules.split(","):
        t0 = time.time()
        order, xoff = baseline_schedule(A) if name == "baseline" else getattr(schedules, name)(A)
        assert np.array_equal(np.sort(order), np.arange(A.shape[0]))
        r = run(lib, A, order, xoff, inflight=args.inflight, bypass=args.bypass)
        loads = [int(A.indptr[order[xoff[k]:xoff[k + 1]] + 1].sum() - A.indptr[order[xoff[k]:xoff[k + 1]]].sum())
                 for k in range(8)]
        print(f"{name:24s} gather hit {r['gather_hit']:.3f}  stream hit {r['stream_hit']:.3f}  "
              f"miss {r['miss_GB']:.3f} GB (gathers {r['gather_miss_GB']:.3f})  nnz/xcd max/mean "
              f"{max(loads) / np.mean(loads):.3f}  ({time.time() - t0:.0f} s)", flush=True)


if __name__ == "__main__":
    main()

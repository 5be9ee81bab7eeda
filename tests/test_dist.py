"""CPU: the N>1 path -- probe sharding + one all-reduce -- with world_size 2 (and 8)
over gloo.  Each rank evaluates its shard with the C oracle (the device call
stands behind the same interface on the GPU box); the reduced estimate must
equal the single-process one."""
import os
import socket

import numpy as np
import pytest

from conftest import load_graph
from krylov_robustness_amd.dist import probe_shard, probe_shard_aligned


def test_probe_shard_covers_range():
    for N in [0, 1, 7, 128, 1024, 1000]:
        for W in [1, 2, 3, 4, 8]:
            seen = []
            for r in range(W):
                o, c = probe_shard(N, r, W)
                seen.extend(range(o, o + c))
            assert seen == list(range(N))


def test_probe_shard_aligned_deals_whole_sweeps():
    """--bitstable's shards: contiguous, covering, and every boundary a
    multiple of the sweep width, so a probe's sweep (its neighbours and the
    sweep's width) is the same at every world size."""
    for N in [0, 1, 7, 128, 1000, 1024]:
        for P in [1, 16, 64]:
            for W in [1, 2, 3, 4, 8]:
                seen = []
                for r in range(W):
                    o, c = probe_shard_aligned(N, P, r, W)
                    assert c >= 0 and (c == 0 or o % P == 0)
                    assert c == 0 or (o + c) % P == 0 or o + c == N
                    seen.extend(range(o, o + c))
                assert seen == list(range(N))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    import torch.distributed as dist
    from oracle import slq_ref
    from krylov_robustness_amd.dist import allreduce_sums
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    A = load_graph("anaheim")
    off, cnt = probe_shard(50, rank, world)
    _, q = slq_ref.slq_trace(A, cnt, 20, seed=5, probe_offset=off, nthreads=1)
    s = allreduce_sums([q.sum(), (q ** 2).sum()])
    if rank == 0:
        out.put(s)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 8])
def test_gloo_world_matches_single(world):
    """world 8 = the driver's 8-GPU node (50 probes: shards of 7, 7, 6 x 6)"""
    import torch.multiprocessing as mp
    from oracle import slq_ref
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    s = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    _, q1 = slq_ref.slq_trace(load_graph("anaheim"), 50, 20, seed=5)
    assert s[0] == pytest.approx(q1.sum(), rel=1e-12)
    assert s[1] == pytest.approx((q1 ** 2).sum(), rel=1e-12)


def _greedy_worker(rank, world, port, out):
    """krylov_miobi with candidates sharded over the ranks:
    each rank scores its slice (here with the oracle's trace_fun_update, the
    device pairs call on the GPU box), scores are all-gathered, every rank
    edits its own copy of A."""
    import numpy as np
    import scipy.sparse as sp
    import torch.distributed as dist
    from oracle import krylov_oracle as ko
    import krylov_robustness_amd as kra
    from krylov_robustness_amd.dist import allgather_concat, probe_shard
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    A = sp.lil_matrix(load_graph("austria"))
    E = kra.find_top_edges(A.tocsr(), kra.compute_centrality(A.tocsr()), 12, "min")
    B = -np.array([[0.0, 1.0], [1.0, 0.0]])
    n = A.shape[0]

    def score(Ecur):
        counts = [probe_shard(len(Ecur), r, world)[1] for r in range(world)]
        off, cnt = probe_shard(len(Ecur), rank, world)
        xm = []
        for i, j in Ecur[off:off + cnt]:
            U = np.zeros((n, 2)); U[i - 1, 0] = 1; U[j - 1, 1] = 1
            xm.append(ko.trace_fun_update(A.tocsr(), U, B, 1e-10, 60)[0])
        return allgather_concat(np.array(xm), counts)

    def edit(e, v):
        A[e[0] - 1, e[1] - 1] = v
        A[e[1] - 1, e[0] - 1] = v

    edges, rob = kra.miobi_loop(3, E, False, score, edit)
    if rank == 0:
        out.put((edges.tolist(), rob))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_sharded_greedy_matches_single():
    import torch.multiprocessing as mp
    from oracle import krylov_oracle as ko
    import krylov_robustness_amd as kra
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_greedy_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    edges, rob = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    A = load_graph("austria")
    E = kra.find_top_edges(A, kra.compute_centrality(A), 12, "min")
    eo, ro, _ = ko.krylov_miobi(A, 3, E, 1e-10, 60, np.inf, 0, "break", 1.0)
    assert edges == eo.tolist()
    assert rob == pytest.approx(ro, rel=1e-12)


def _reduce_worker(rank, world, port, out):
    """kt_reduce_fn plumbing: the ctypes callback mc_trace_sharded hands to
    the library sums its buffer over the gloo group in place."""
    import ctypes as C
    import torch.distributed as dist
    from krylov_robustness_amd.dist import reduce_callback
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cb = reduce_callback()
    buf = (C.c_double * 10)(*[0.0] * 10)
    for c in range(rank, 10, world):  # the round-robin G-column deal
        buf[c] = 1.5 * c + 0.25
    st = cb(buf, 10, None)
    if rank == 0:
        out.put((st, list(buf)))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_reduce_callback():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_reduce_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    st, vals = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
    assert st == 0
    assert vals == [1.5 * c + 0.25 for c in range(10)]


def _reduce_fail_worker(rank, world, port, out):
    """One rank's local part of the reduce fails (test hook): it still joins
    the collective with its error flag set, so EVERY rank returns 1 in the
    same round (no rank is left waiting in all_reduce)."""
    import ctypes as C
    import torch.distributed as dist
    from krylov_robustness_amd.dist import reduce_callback
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cb = reduce_callback(fail_on_rank=1)
    buf = (C.c_double * 10)(*[float(rank)] * 10)
    st = cb(buf, 10, None)
    ok = reduce_callback()  # the group is still usable afterwards
    buf2 = (C.c_double * 3)(*[1.0] * 3)
    st2 = ok(buf2, 3, None)
    out.put((rank, st, list(buf), st2, list(buf2)))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_reduce_callback_failure_reaches_every_rank():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_reduce_fail_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, st, buf, st2, buf2 in res:
        assert st == 1                      # failed on both ranks
        assert buf == [float(rank)] * 10    # the buffer is left untouched
        assert st2 == 0 and buf2 == [2.0] * 3


def _bitstable_worker(rank, world, port, out):
    """bench.py --bitstable's reduction: each rank holds the oracle's forms of
    its contiguous probe shard; dist.bitstable_sums all-gathers them and sums
    in global probe order."""
    import torch.distributed as dist
    from oracle import slq_ref
    from krylov_robustness_amd.dist import bitstable_sums, centred_sums, moment_sums
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    A = load_graph("rome")
    N = 37  # ragged: 37 = 10 + 9 + 9 + 9 at world 4
    counts = [probe_shard(N, r, world)[1] for r in range(world)]
    off, cnt = probe_shard(N, rank, world)
    _, q = slq_ref.slq_trace(A, cnt, 15, seed=3, probe_offset=off, nthreads=1)
    stats = {}
    ms = moment_sums(q[:cnt], stats=stats)
    out.put((rank, (bitstable_sums(q[:cnt], counts), centred_sums(q[:cnt], N), ms, stats["calls"])))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_gloo_bitstable_sums_identical_across_world_sizes(world):
    """Bit-identical (==, not approx) estimate on every rank and equal to the
    single-process ordered sum of the same forms (SURVEY.md §8e option); the
    default one-collective form (moment_sums: all-gather of (count, sum, M2),
    Chan's pairwise combination in rank order; ONE collective per
    evaluation) and the two-all-reduce centred form agree to rounding, and
    every rank's moment_sums result is the same bits."""
    import torch.multiprocessing as mp
    from oracle import slq_ref
    from krylov_robustness_amd.dist import bitstable_sums, ordered_sums
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bitstable_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # the forms of one probe do not depend on the shard it was evaluated in
    _, q1 = slq_ref.slq_trace(load_graph("rome"), 37, 15, seed=3, nthreads=1)
    single = bitstable_sums(q1, [37])  # no process group: the local forms, same order
    assert single == ordered_sums(q1)
    for r in range(world):
        assert got[r][0] == single
        # the two-all-reduce form: the same to rounding
        assert got[r][1][0] == pytest.approx(single[0], rel=1e-14)
        assert got[r][1][1] == pytest.approx(single[1], rel=1e-12)
        # bench.py's default: one all-gather, Chan's combination
        assert got[r][3] == 1
        assert got[r][2] == got[0][2]
        assert got[r][2][0] == pytest.approx(single[0], rel=1e-14)
        assert got[r][2][1] == pytest.approx(single[1], rel=1e-12)

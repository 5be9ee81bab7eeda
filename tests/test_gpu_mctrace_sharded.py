"""GPU: mc_trace on `world` ranks (kt_mc_trace_sharded) --
S, Q and tr(Q' Afun Q) replicated, the G-probe columns dealt round-robin and
their quadratic forms all-reduced once per round.

world = 1 must equal kt_mc_trace bit for bit.  world = 2, 3 are run in one
process by one host thread per rank, each with its own context on the same
GPU, joined by an in-process all-reduce.  With the Lanczos Afun each round
queues its Afun columns together (kt_mctrace.cpp mc_trace_batched: the
round's Q and G terms and the next S term, as 16-wide sweeps on several
lanes); a rank's G columns sit in fixed slots beside the replicated columns,
and a column's form does not depend on its neighbours, so every world size
returns the world-1 estimate BIT FOR BIT.
The per-call form (KT_MC_BATCH=0) runs a rank's G columns as a narrower
block (P = 8 or 4 instead of 16), whose reductions round differently: there
the estimate agrees to 1e-12 relative with the same round count.  The expmv
Afun is replicated (its Taylor degree is chosen per block) and never calls
the reduction.  A 2-process gloo run checks the torch.distributed callback
end to end."""
import ctypes as C
import os
import socket
import threading

import numpy as np
import pytest

from conftest import load_graph

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def kra():
    import krylov_robustness_amd as kra
    return kra


class _ThreadReduce:
    """All-reduce (sum) across `world` host threads, one call per round."""

    def __init__(self, world):
        self.world = world
        self.bar = threading.Barrier(world)
        self.bufs = [None] * world
        self.calls = 0
        self.totals = []  # the all-reduced vector of every round (rank 0's view)

    def fn(self, rank):
        from krylov_robustness_amd import _lib

        def cb(buf, count, user):
            arr = np.ctypeslib.as_array(buf, shape=(int(count),))
            self.bufs[rank] = arr.copy()
            self.bar.wait()
            tot = np.zeros(int(count))
            for b in self.bufs:  # fixed rank order
                tot = tot + b
            self.bar.wait()
            arr[:] = tot
            if rank == 0:
                self.calls += 1
                self.totals.append(tot.copy())
            return 0
        return _lib.REDUCE_FN(cb)


def _run_world(kra, A, world, afun, **kw):
    red = _ThreadReduce(world)
    out = [None] * world
    errs = []

    def worker(r):
        try:
            ctx = kra.Context(0)
            D = kra.DeviceMatrix(A, ctx)
            cb = red.fn(r)
            out[r] = kra.mc_trace_sharded(afun, None, A=D, rank=r, world=world, allreduce=cb,
                                          ctx=ctx, **kw)
        except Exception as e:  # pragma: no cover - reported below
            errs.append(e)
            red.bar.abort()

    th = [threading.Thread(target=worker, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not errs, errs
    return out, red.calls


def _run_world_forms(kra, A, world, afun, **kw):
    """As _run_world, plus every round's all-reduced G-form vector."""
    red = _ThreadReduce(world)
    out = [None] * world
    errs = []

    def worker(r):
        try:
            ctx = kra.Context(0)
            D = kra.DeviceMatrix(A, ctx)
            out[r] = kra.mc_trace_sharded(afun, None, A=D, rank=r, world=world, allreduce=red.fn(r),
                                          ctx=ctx, **kw)
        except Exception as e:  # pragma: no cover - reported below
            errs.append(e)
            red.bar.abort()

    th = [threading.Thread(target=worker, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not errs, errs
    return out, red.totals


@pytest.mark.parametrize("afun", ["lanczos", "matrix"])
def test_world1_equals_mc_trace(kra, gpu_ctx, afun):
    A = load_graph("oregon_A0")
    D = kra.DeviceMatrix(A, gpu_ctx)
    kw = dict(tol=1e-3, maxit=90, isAreal=1, seed=3, fun="exp", m=20)
    ref = kra.mc_trace(afun, None, A=D, ctx=gpu_ctx, **kw)
    got = kra.mc_trace_sharded(afun, None, A=D, rank=0, world=1, ctx=gpu_ctx, **kw)
    assert got == ref


@pytest.mark.parametrize("world", [2, 3, 4])
@pytest.mark.parametrize("tol,maxit", [(1e-6, 120), (0.0, 90)])
def test_threads_world_matches_single(kra, gpu_ctx, world, tol, maxit):
    """tol = 0 runs every one of the K = ceil(maxit / 30) rounds, the last
    (it == K, no next S term) included: still bit for bit at every world
    size (the G columns sit in fixed slots, so no sweep width depends on the
    number of columns a rank owns)."""
    A = load_graph("oregon_A0")
    kw = dict(tol=tol, maxit=maxit, isAreal=1, seed=3, fun="exp", m=20)
    ref = kra.mc_trace("lanczos", None, A=kra.DeviceMatrix(A, gpu_ctx), ctx=gpu_ctx, **kw)
    out, calls = _run_world(kra, A, world, "lanczos", **kw)
    for r in out:
        assert r == ref  # every rank, bit for bit
    assert calls == ref[2]  # one all-reduce per round


@pytest.mark.parametrize("world", [2, 3])
def test_threads_world_guard_redo_bit_identical(kra, gpu_ctx, monkeypatch, world):
    """Never computing the S term ahead (KT_MC_AHEAD=0) sends round 1's Q
    columns through y-form sweeps; Q_1's first column is the top eigenvector
    to rounding (exp(A) of this graph is near rank one), a lucky breakdown at
    step 1 that trips the y-form guard.  Only the tripped column takes the
    explicit redo's records, so the replicated Q forms and the G slots stay
    world-independent: bit for bit at every world size, redo included."""
    monkeypatch.setenv("KT_MC_AHEAD", "0")
    A = load_graph("oregon_A0")
    kw = dict(tol=0.0, maxit=60, isAreal=1, seed=3, fun="exp", m=20)
    before = gpu_ctx.stat(0)
    ref = kra.mc_trace("lanczos", None, A=kra.DeviceMatrix(A, gpu_ctx), ctx=gpu_ctx, **kw)
    assert gpu_ctx.stat(0) > before  # the guard redo ran
    out, calls = _run_world(kra, A, world, "lanczos", **kw)
    for r in out:
        assert r == ref
    assert calls == ref[2]


@pytest.mark.parametrize("ahead", ["0", "1"])
def test_threads_world_g_forms_bit_identical(kra, monkeypatch, ahead):
    """The G forms themselves, not only the estimate: on an ER graph (exp(A)
    far from rank one, so the deflated G term is not negligible against the
    trace) every round's all-reduced 10-vector of G quadratic forms is the
    same bits at worlds 1-4 -- G column c sits in slot 2 mb + c of the same
    16-wide sweep whatever the rank count, the other ranks' slots zero.
    KT_MC_AHEAD=0: every round without the S term (the final-round sweep
    plan); 1: every round with it; tol = 0 runs all K rounds."""
    from krylov_robustness_amd import graphs
    monkeypatch.setenv("KT_MC_AHEAD", ahead)
    A = graphs.erdos_renyi(20_000, 100_000, seed=2)
    kw = dict(tol=0.0, maxit=90, isAreal=1, seed=5, fun="exp", m=20)
    ref, g1 = _run_world_forms(kra, A, 1, "lanczos", **kw)
    assert len(g1) == 3 and all(np.all(g != 0) for g in g1)
    gsum = sum(abs(float(np.sum(g))) / 10 for g in g1)
    assert gsum > 1e-6 * abs(ref[0][0])  # the G term moves the estimate
    for world in (2, 3, 4):
        out, gw = _run_world_forms(kra, A, world, "lanczos", **kw)
        assert len(gw) == len(g1)
        for a, b in zip(gw, g1):
            assert np.array_equal(a, b)
        for r in out:
            assert r == ref[0]


@pytest.mark.parametrize("world", [2, 3])
def test_threads_world_per_call_form(kra, gpu_ctx, monkeypatch, world):
    monkeypatch.setenv("KT_MC_BATCH", "0")
    A = load_graph("oregon_A0")
    kw = dict(tol=1e-6, maxit=120, isAreal=1, seed=3, fun="exp", m=20)
    ref = kra.mc_trace("lanczos", None, A=kra.DeviceMatrix(A, gpu_ctx), ctx=gpu_ctx, **kw)
    out, calls = _run_world(kra, A, world, "lanczos", **kw)
    for tr, res, it in out:
        assert tr == out[0][0] and it == out[0][2]  # every rank returns the same estimate
        assert it == ref[2]
        assert tr == pytest.approx(ref[0], rel=1e-12)
    assert calls == ref[2]


def test_threads_expmv_is_replicated(kra, gpu_ctx):
    A = load_graph("oregon_A0")
    kw = dict(tol=1e-4, maxit=60, isAreal=1, seed=1)
    ref = kra.mc_trace("expmv", None, A=kra.DeviceMatrix(A, gpu_ctx), ctx=gpu_ctx, **kw)
    out, calls = _run_world(kra, A, 2, "expmv", **kw)
    assert calls == 0
    for r in out:
        assert r == ref


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _gloo_worker(rank, world, port, q):
    import torch  # noqa: F401
    import torch.distributed as dist
    import krylov_robustness_amd as kra
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    A = load_graph("oregon_A0")
    ctx = kra.Context(0)
    tr = kra.trace_exp_sharded(kra.DeviceMatrix(A, ctx), m=20, seed=2, ctx=ctx)
    q.put((rank, tr))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_two_processes_trace_exp(kra, gpu_ctx):
    import torch.multiprocessing as mp
    A = load_graph("oregon_A0")
    ref = kra.trace_exp(kra.DeviceMatrix(A, gpu_ctx), method="lanczos", m=20, seed=2, ctx=gpu_ctx)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gloo_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=240) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
    assert got[0] == got[1] == ref

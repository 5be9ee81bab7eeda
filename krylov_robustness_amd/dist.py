"""Multi-GPU plumbing: probes shard across ranks (one process per GPU), one
collective per evaluation.

The probe RNG is keyed by the GLOBAL probe index, so the estimate does not
depend on the number of ranks; the only collective of a Hutchinson
evaluation is one all-gather of each rank's (count, sum, centred second
moment) -- 24 bytes per rank -- over RCCL ("nccl" backend) or gloo on CPU,
combined on every rank in rank order (moment_sums).
"""
from __future__ import annotations

import os


def probe_shard(nprobes: int, rank: int, world: int):
    """Contiguous, balanced shard [offset, offset+count) of the global probes."""
    base, rem = divmod(int(nprobes), int(world))
    count = base + (1 if rank < rem else 0)
    offset = rank * base + min(rank, rem)
    return offset, count


def probe_shard_aligned(nprobes: int, block: int, rank: int, world: int):
    """Shard [offset, offset+count) whose boundaries are multiples of the
    sweep width `block`: whole sweeps are dealt (balanced) over the ranks, so
    every probe sits in the same sweep -- same neighbours, same width -- at
    any world size.  Then even a sweep the y-form guard sends back to the
    explicit CGS2 sweep (which recomputes the whole sweep) gives each probe
    the same form everywhere (bench.py --bitstable)."""
    nprobes, block = int(nprobes), max(1, int(block))
    sweeps = (nprobes + block - 1) // block
    s_off, s_cnt = probe_shard(sweeps, rank, world)
    off = min(nprobes, s_off * block)
    return off, min(nprobes, (s_off + s_cnt) * block) - off


def env_rank():
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def _group_ready(force: bool) -> bool:
    """Issue the collective?  Always with more than one rank; at world 1 only
    when `force` is set and a process group exists (exercises RCCL init and
    the collective inside a process that holds libkrylov_hip.so's streams)."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return False
    return dist.get_world_size() > 1 or bool(force)


def allreduce_sums(vals, device=None, force: bool = False):
    """Sum a short list of doubles over the default process group."""
    import torch
    import torch.distributed as dist
    if not _group_ready(force):  # nothing to reduce: no device tensor, no copies, no sync
        return [float(x) for x in vals]
    t = torch.tensor(list(vals), dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return [float(x) for x in t.cpu().tolist()]


def allreduce_max(val: float, device=None, force: bool = False):
    import torch
    import torch.distributed as dist
    if not _group_ready(force):
        return float(val)
    t = torch.tensor([float(val)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def allgather_concat(x, counts, group=None):
    """Concatenate per-rank 1-D float64 arrays in rank order (rank r holds
    counts[r] values).  Pads to max(counts) so one fixed-size all_gather works
    on gloo and RCCL alike; RCCL needs device tensors (current GPU)."""
    import numpy as np
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    m = max(int(max(counts)), 1)
    backend = dist.get_backend(group)
    dev = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")
    t = torch.zeros(m, dtype=torch.float64, device=dev)
    x = np.asarray(x, dtype=np.float64).ravel()
    if x.size:
        t[:x.size] = torch.from_numpy(x).to(dev)
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t, group=group)
    return np.concatenate([p[:int(c)].cpu().numpy() for p, c in zip(parts, counts)])


def ordered_sums(q):
    """(sum q, sum (q - mean)^2) accumulated in index order: the Hutchinson
    estimate's sum and the centred second moment of the forms (two passes:
    sum q^2 - N mean^2 cancels when the spread is small against the mean)."""
    q = [float(v) for v in q]
    s1 = 0.0
    for v in q:
        s1 += v
    mu = s1 / len(q) if q else 0.0
    m2 = 0.0
    for v in q:
        m2 += (v - mu) * (v - mu)
    return s1, m2


def centred_sums(q, nprobes, device=None, force=False):
    """Hutchinson reduction in two all-reduces (rounds 1-5; kept for
    comparison): sum q, then every rank centres its forms on the global mean
    and a second all-reduce sums (q - mean)^2.  Returns (sum q, sum (q -
    mean)^2).  bench.py uses moment_sums (one collective)."""
    s_loc = 0.0
    for v in q:
        s_loc += float(v)
    s1 = allreduce_sums([s_loc], device=device, force=force)[0]
    mu = s1 / nprobes if nprobes else 0.0
    m2_loc = 0.0
    for v in q:
        m2_loc += (float(v) - mu) * (float(v) - mu)
    return s1, allreduce_sums([m2_loc], device=device, force=force)[0]


def local_moments(q):
    """(count, sum q, sum (q - local mean)^2) of one rank's forms, in index
    order (ordered_sums' two passes)."""
    s, m2 = ordered_sums(q)
    return float(len(q)), s, m2


def chan_combine(parts):
    """Combine per-rank (count, sum, M2) triples in the order given (rank
    order) with the pairwise update of Chan, Golub & LeVeque (1979):
    M2_ab = M2_a + M2_b + delta^2 n_a n_b / (n_a + n_b), delta = mean_b -
    mean_a; the sums are added in the same order.  Returns (sum q, M2) --
    the same quantities as ordered_sums over the concatenated forms, equal
    to rounding (bit-equal for a single part)."""
    n, s, m2 = 0.0, 0.0, 0.0
    for nb, sb, m2b in parts:
        nb, sb, m2b = float(nb), float(sb), float(m2b)
        if nb <= 0:
            continue
        if n <= 0:
            n, s, m2 = nb, sb, m2b
            continue
        delta = sb / nb - s / n
        tot = n + nb
        m2 = m2 + m2b + delta * delta * (n * nb / tot)
        s = s + sb
        n = tot
    return s, m2


def moment_sums(q, device=None, force=False, stats=None):
    """Hutchinson reduction over the ranks' probe shards with ONE collective:
    every rank forms (count, sum, M2) of its own forms (local_moments),
    all-gathers the triples (24 bytes per rank) and combines them in rank
    order (chan_combine), so every rank holds the same (sum q, sum (q -
    mean)^2).  Without a process group (or at world 1 without `force`) no
    collective runs and the local triple is the answer.  `stats` (a dict)
    collects the collective's calls and host-side microseconds."""
    import time
    trip = local_moments(q)
    if not _group_ready(force):
        return trip[1], trip[2]
    import torch
    import torch.distributed as dist
    t0 = time.perf_counter()
    world = dist.get_world_size()
    t = torch.tensor(list(trip), dtype=torch.float64, device=device)
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    rows = torch.stack(parts).cpu().tolist()
    if stats is not None:
        stats["calls"] = stats.get("calls", 0) + 1
        stats.setdefault("us", []).append((time.perf_counter() - t0) * 1e6)
    return chan_combine(rows)


def allgather_floats(vals, device=None):
    """Every rank's list of floats (same length), in rank order; the local
    list alone without a process group."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return [[float(v) for v in vals]]
    t = torch.tensor([float(v) for v in vals], dtype=torch.float64, device=device)
    parts = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, t)
    return torch.stack(parts).cpu().tolist()


def bitstable_sums(q, counts, group=None):
    """SURVEY.md §8e's bit-stable reduction: all-gather every rank's per-probe
    forms (rank r holds the counts[r] forms of its contiguous shard, so rank
    order is global probe order) and reduce them in that order on every rank
    (ordered_sums).  The per-probe forms are keyed by the global probe index,
    so the result is bit-identical for any number of ranks, including a single
    process (no group: the local forms, same order)."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        q = allgather_concat(q, counts, group)
    return ordered_sums(q)


def reduce_callback(group=None, fail_on_rank=None):
    """A kt_reduce_fn (include/krylov_trace.h) that sums the buffer over the
    torch.distributed group: device tensors on RCCL ("nccl"), CPU tensors
    on gloo.  Keep the returned object alive for the duration of the call.

    The buffer travels with one extra element, the rank's local error flag:
    a rank whose own part fails (reading the buffer, moving it to the
    device) still joins the collective with that flag set, so every rank
    sees the failure in the same round and returns 1 (the library call then
    fails with KT_ERR_CALLBACK everywhere) instead of the other ranks
    waiting in all_reduce until the process group times out.  Test hook:
    `fail_on_rank` makes that rank's local part fail."""
    import numpy as np
    import torch
    import torch.distributed as dist
    from . import _lib

    def _cb(buf, count, user):
        k = int(count)
        try:
            backend = dist.get_backend(group)
            dev = (torch.device("cuda", torch.cuda.current_device()) if backend == "nccl"
                   else torch.device("cpu"))
        except Exception:  # no usable process group: nothing to join
            return 1
        arr = None
        try:
            if fail_on_rank is not None and dist.get_rank(group) == fail_on_rank:
                raise RuntimeError("injected reduce failure")
            arr = np.ctypeslib.as_array(buf, shape=(k,))
            t = torch.from_numpy(np.append(arr, 0.0)).to(dev)
        except Exception:
            arr = None
            t = torch.zeros(k + 1, dtype=torch.float64, device=dev)
            t[k] = 1.0  # local failure flag
        try:
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
            out = t.cpu().numpy()
        except Exception:
            return 1
        if out[k] != 0.0 or arr is None:
            return 1
        arr[:] = out[:k]
        return 0

    return _lib.REDUCE_FN(_cb)


def mc_trace_sharded(Afun, n=None, tol=1e-3, maxit=10, isAreal=0, debug=0, seed=0, fun="exp",
                     m=30, A=None, rank=None, world=None, allreduce=None, group=None, ctx=None,
                     force=False):
    """[tr, res, it] = mc_trace(...) on `world` GPUs: every
    rank recomputes S, Q and tr(Q' Afun Q) from the shared seed, the G-probe
    columns are dealt round-robin and their quadratic forms summed by one
    all-reduce per round (kt_mc_trace_sharded).  Afun as in core.mc_trace.
    rank / world default to the torch.distributed group; `allreduce` is a
    _lib.REDUCE_FN (default: reduce_callback(group); at world 1 none unless
    `force`, which routes the round sums through the group's all-reduce)."""
    import ctypes as C
    from . import _lib
    from .core import _dev
    if rank is None or world is None:
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            rank, world = dist.get_rank(group), dist.get_world_size(group)
        else:
            rank, world = 0, 1
    if isinstance(Afun, str):
        kind = _lib.AFUN_CODES[Afun]
        D = _dev(A, ctx)
    else:
        kind = _lib.AFUN_CODES["matrix"]
        D = _dev(Afun, ctx)
    if n is not None and int(n) != D.n:
        raise _lib.KrylovError(_lib.KT_ERR_ARG, "n does not match the matrix")
    cb = allreduce if allreduce is not None else (reduce_callback(group) if world > 1 or force
                                                  else _lib.REDUCE_FN(0))
    tr, res, it = C.c_double(), C.c_double(), C.c_int()
    _lib.check(_lib.load().kt_mc_trace_sharded(
        D.handle, kind, _lib.FUN_CODES[fun] if isinstance(fun, str) else int(fun), int(m), float(tol),
        int(maxit), int(isAreal), int(seed) & 0xFFFFFFFFFFFFFFFF, int(rank), int(world), cb, None,
        C.byref(tr), C.byref(res), C.byref(it)))
    return float(tr.value), float(res.value), int(it.value)


def trace_exp_sharded(A, method="lanczos", m=30, seed=0, rank=None, world=None, allreduce=None,
                      group=None, ctx=None):
    """trace_exp.m:1-7 (mc_trace(Afun, n, 1e-4, 1000, 1)) on `world` GPUs."""
    tr, _, _ = mc_trace_sharded(method, None, 1e-4, 1000, 1, 0, seed, "exp", m, A=A, rank=rank,
                                world=world, allreduce=allreduce, group=group, ctx=ctx)
    return tr

"""CPU: the N>1 path -- probe sharding + one all-reduce -- with world_size 2
over gloo.  Each rank evaluates its shard with the C oracle (the device call
stands behind the same interface on the GPU box); the reduced estimate must
equal the single-process one."""
import os
import socket

import numpy as np
import pytest

from conftest import load_graph
from krylov_robustness_amd.dist import probe_shard


def test_probe_shard_covers_range():
    for N in [0, 1, 7, 128, 1024, 1000]:
        for W in [1, 2, 3, 4, 8]:
            seen = []
            for r in range(W):
                o, c = probe_shard(N, r, W)
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


def test_gloo_world2_matches_single():
    import torch.multiprocessing as mp
    from oracle import slq_ref
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    s = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    _, q1 = slq_ref.slq_trace(load_graph("anaheim"), 50, 20, seed=5)
    assert s[0] == pytest.approx(q1.sum(), rel=1e-12)
    assert s[1] == pytest.approx((q1 ** 2).sum(), rel=1e-12)

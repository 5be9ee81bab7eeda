"""Multi-GPU plumbing: probes shard across ranks (one process per GPU), one
all-reduce of the partial sums.

The probe RNG is keyed by the GLOBAL probe index, so the estimate does not
depend on the number of ranks; the only collective is a 2-double sum
(sum q, sum q^2) over RCCL ("nccl" backend) or gloo on CPU.
"""
from __future__ import annotations

import os


def probe_shard(nprobes: int, rank: int, world: int):
    """Contiguous, balanced shard [offset, offset+count) of the global probes."""
    base, rem = divmod(int(nprobes), int(world))
    count = base + (1 if rank < rem else 0)
    offset = rank * base + min(rank, rem)
    return offset, count


def env_rank():
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def allreduce_sums(vals, device=None):
    """Sum a short list of doubles over the default process group."""
    import torch
    import torch.distributed as dist
    t = torch.tensor(list(vals), dtype=torch.float64, device=device)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return [float(x) for x in t.cpu().tolist()]


def allreduce_max(val: float, device=None):
    import torch
    import torch.distributed as dist
    t = torch.tensor([float(val)], dtype=torch.float64, device=device)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())

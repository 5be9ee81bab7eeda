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

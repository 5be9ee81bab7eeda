"""Worker for test_gpu_bench.py::test_mc_trace_sharded_rccl_world1 (launched
by torch.distributed.run with one rank): RCCL process group first (device_id
bound before any library call), then kt_mc_trace_sharded with the round sums
all-reduced through dist.reduce_callback on device tensors, compared with
kt_mc_trace on the same matrix.  Prints one JSON line."""
import json
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    import krylov_robustness_amd as kra
    from krylov_robustness_amd import _lib, dist as kdist
    from conftest import load_graph

    calls = [0]
    inner = kdist.reduce_callback()

    def counting(buf, count, user):  # count the collective calls, then forward
        calls[0] += 1
        return inner(buf, count, user)

    cb = _lib.REDUCE_FN(counting)
    A = load_graph("oregon_A0")
    ctx = kra.Context(local)
    D = kra.DeviceMatrix(A, ctx)
    sharded = kdist.mc_trace_sharded("lanczos", None, 1e-4, 90, 1, 0, 5, "exp", 20, A=D, rank=0,
                                     world=1, allreduce=cb, ctx=ctx)
    single = kra.mc_trace("lanczos", None, 1e-4, 90, 1, 0, seed=5, fun="exp", m=20, A=D, ctx=ctx)
    print(json.dumps({"backend": dist.get_backend(), "callback_calls": calls[0],
                      "sharded": list(sharded), "single": list(single)}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()

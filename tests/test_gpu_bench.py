"""GPU: bench.py keeps the driver's contract -- ONE JSON line on rank 0 with
the metric, whole-job value, roofline (algorithmic + PMC-traffic rates of the
dominant kernel) and cpu_baseline objects -- on a small configuration (the
config-2 graph, 32 probes, m = 5), single process and two torchrun ranks
sharing the GPU over gloo (the N > 1 launch the driver uses, rehearsed)."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

SMALL = ["--config", "er100k", "--nprobes", "32", "--lanczos-m", "5", "--steps", "2", "--warmup", "1"]
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
        "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"}


def _json_lines(out):
    return [json.loads(ln) for ln in out.splitlines() if ln.startswith("{")]


def test_bench_single_process_line():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *SMALL, "--cpu-seconds", "1"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1
    d = lines[0]
    assert KEYS <= set(d)
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["warmup"] == 1
    assert d["value"] > 0 and d["higher_is_better"] is True and d["dtype"] == "f64"
    # ms_per_step is printed to 3 decimals (a 0.5 ms step carries ~1e-3 relative rounding)
    assert d["value"] == pytest.approx(1e3 / d["ms_per_step"], rel=1e-2)
    roof = d["roofline"]
    assert roof["bound"] == "hbm" and roof["unit"] == "GB/s" and roof["peak"] == 8000.0
    assert roof["frac"] == pytest.approx(roof["achieved"] / roof["peak"], rel=1e-3)
    assert roof["avg_launch_us"] > 0
    # the timed-region duration per launch is the union of the launches'
    # intervals over the lanes: no longer than the mean per-launch event time,
    # and the union no longer than the timed wall time
    assert roof["avg_launch_us"] <= roof["timed_region_avg_launch_us_overlapped"] * 1.001
    assert roof["timed_region_busy_ms"] <= d["steps"] * d["ms_per_step"] * 1.01
    assert roof["isolated_pass"]["avg_launch_us"] > 0 and roof["isolated_pass"]["launches"] > 0
    # unit-weight graph: the roofline is priced on the bytes the kernel must
    # move (4 B per nonzero, values never read), SURVEY's 12 B figure beside it
    n, nnz, P = d["config"]["n"], d["config"]["nnz"], d["config"]["probes_per_sweep"]
    assert d["eval_roofline"]["unit_weight_matrix"] is True
    assert roof["algorithmic_bytes_per_launch"] == 4 * nnz + 4 * (n + 1) + 24 * n * P
    assert roof["survey_bytes_per_launch"] == 12 * nnz + 4 * (n + 1) + 24 * n * P
    assert roof["survey_frac"] > roof["frac"]
    # the estimator's standard error from sum q^2
    assert d["trace_stderr"] is not None and 0 < d["trace_stderr"] < abs(d["trace_estimate"])
    cpu = d["cpu_baseline"]
    assert cpu["kind"] == "port" and cpu["value"] > 0 and cpu["cores"] >= 1
    # every CPU the process may use: the affinity mask, capped by the cgroup quota
    sys.path.insert(0, ROOT)
    import bench
    assert cpu["cores"] == bench.cpu_share()[0]
    assert cpu["affinity_cpus"] >= cpu["cores"]
    assert d["yform_redone_sweeps"] == 0
    assert d["collective"] is None  # single process, no torchrun: no process group


def test_bench_two_ranks_one_gpu_gloo():
    env = dict(os.environ, KT_BENCH_ONE_DEVICE="1", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29531", os.path.join(ROOT, "bench.py"),
           "--gpus", "2", *SMALL, "--dist-backend", "gloo", "--no-profile"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1  # rank 0 only
    d = lines[0]
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "probes sharded x2"
    assert d["cpu_baseline"] is None and d["value"] > 0


def test_bench_world1_torchrun_rccl():
    """torchrun with ONE rank and the nccl (RCCL) backend: the process group is
    initialised (device_id bound before any library call) and the per-evaluation
    all-reduce of (sum q, sum q^2) and the max-over-ranks time run through RCCL
    at world 1 -- RCCL init coexisting with libkrylov_hip.so's streams, the
    launch the driver uses at N > 1 minus the peers."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", "29533", os.path.join(ROOT, "bench.py"),
           "--gpus", "1", *SMALL, "--dist-backend", "nccl", "--cpu-seconds", "0"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1
    d = lines[0]
    assert d["n_gpus"] == 1 and d["collective"].startswith("RCCL all_reduce")
    assert d["value"] > 0 and d["roofline"]["avg_launch_us"] > 0
    # same probes, same estimate as the single-process line (the collective is a sum of one)
    r1 = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *SMALL, "--cpu-seconds", "0",
                         "--no-profile"], capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r1.returncode == 0, r1.stderr[-2000:]
    d1 = _json_lines(r1.stdout)[0]
    assert d["trace_estimate"] == d1["trace_estimate"]
    assert d["trace_stderr"] == d1["trace_stderr"]


def test_mc_trace_sharded_rccl_world1():
    """kt_mc_trace_sharded with dist.reduce_callback on device tensors over an
    RCCL group of one rank (tests/rccl_world1_worker.py under torchrun): the
    G-term sums of every round travel through RCCL's all-reduce, and the
    estimate, residual and round count are bit-identical to kt_mc_trace."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", "29535",
           os.path.join(ROOT, "tests", "rccl_world1_worker.py")]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_lines(r.stdout)[-1]
    assert d["backend"] == "nccl" and d["callback_calls"] >= 1
    assert d["sharded"] == d["single"]

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
    # (the union is formed over every launch of the timed region at once, so
    # pipelined evaluations' overlapping launches are not counted twice)
    assert roof["timed_region_busy_ms"] <= roof["timed_region_ms"] + 1e-3
    # (both printed to 3 decimals: half a unit of rounding per step)
    assert roof["timed_region_ms"] <= d["steps"] * (d["ms_per_step"] + 5e-4) * 1.001 + 5e-4
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
    assert roof["busy_within_timed_region"] is True


def _single_line(*extra):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *SMALL, "--cpu-seconds", "0",
                        "--no-profile", *extra], capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    return _json_lines(r.stdout)[0]


def _ranks_line(world, port, *extra):
    """bench.py under torchrun with `world` gloo ranks sharing GPU 0 (the N > 1
    launch the driver uses, rehearsed on one card)."""
    env = dict(os.environ, KT_BENCH_ONE_DEVICE="1", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
           "--gpus", str(world), *SMALL, "--dist-backend", "gloo", "--no-profile", *extra]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1  # rank 0 only
    d = lines[0]
    # a one-device rehearsal counts one GPU; the ranks are the process group's
    assert d["n_gpus"] == 1 and d["launch"]["process_group_world_size"] == world
    assert d["launch"]["one_device_rehearsal"] is True
    assert d["config"]["parallelism"] == f"probes sharded x{world}"
    assert d["cpu_baseline"] is None and d["value"] > 0
    assert d["per_rank_timed_ms"]["ranks"] == world
    assert d["per_rank_timed_ms"]["min"] <= d["per_rank_timed_ms"]["max"]
    return d


def test_bench_two_ranks_one_gpu_gloo():
    """Two ranks: the sharded evaluation gives the single-process estimate and
    standard error (the only difference is the order the two shards' sums are
    added: rel 1e-12), and so does the sharded mc_trace leg (G columns dealt
    over the ranks; S, Q replicated)."""
    d1 = _single_line("--mc-steps", "1")
    d = _ranks_line(2, 29531, "--mc-steps", "1")
    # one collective per evaluation (all-gather of count, sum, M2; Chan's combination)
    c = d["collective"]
    assert c["backend"] == "gloo" and c["op"].startswith("all_gather of each rank's")
    assert c["calls_per_eval"] == 1 and c["us_per_call_mean"] > 0
    assert d["trace_estimate"] == pytest.approx(d1["trace_estimate"], rel=1e-12)
    assert d["trace_stderr"] == pytest.approx(d1["trace_stderr"], rel=1e-12)
    for a, b in zip(d["evaluations"]["estimates"], d1["evaluations"]["estimates"]):
        assert a == pytest.approx(b, rel=1e-12)
    assert d["mc_trace"]["trace_estimate"] == pytest.approx(d1["mc_trace"]["trace_estimate"], rel=1e-12)
    assert d["mc_trace"]["rounds"] == d1["mc_trace"]["rounds"]


def test_bench_four_ranks_one_gpu_gloo():
    d1 = _single_line("--mc-steps", "0")
    d = _ranks_line(4, 29537, "--mc-steps", "0")
    assert d["trace_estimate"] == pytest.approx(d1["trace_estimate"], rel=1e-12)
    assert d["trace_stderr"] == pytest.approx(d1["trace_stderr"], rel=1e-12)


def test_bench_bitstable_identical_over_1_2_4_ranks():
    """--bitstable: every rank all-gathers the per-probe forms
    and sums them in global probe order, so 1, 2 and 4 ranks print the SAME
    estimate and standard error, bit for bit."""
    d1 = _single_line("--mc-steps", "0", "--bitstable")
    d2 = _ranks_line(2, 29539, "--mc-steps", "0", "--bitstable")
    d4 = _ranks_line(4, 29541, "--mc-steps", "0", "--bitstable")
    assert d2["collective"]["op"].startswith("all_gather of the per-probe forms")
    for d in (d2, d4):
        assert d["trace_estimate"] == d1["trace_estimate"]
        assert d["trace_stderr"] == d1["trace_stderr"]
        assert d["evaluations"]["estimates"] == d1["evaluations"]["estimates"]
    # and it agrees with the all-reduce line to rounding
    d0 = _single_line("--mc-steps", "0")
    assert d1["trace_estimate"] == pytest.approx(d0["trace_estimate"], rel=1e-12)


def test_bench_world1_torchrun_rccl():
    """torchrun with ONE rank and the nccl (RCCL) backend: the process group is
    initialised (device_id bound before any library call) and the per-evaluation
    all-gather of (count, sum q, M2) and the max-over-ranks time run through RCCL
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
    assert d["n_gpus"] == 1 and d["collective"]["backend"] == "RCCL"
    assert d["collective"]["calls_per_eval"] == 1
    assert d["value"] > 0 and d["roofline"]["avg_launch_us"] > 0
    # same probes, same estimate as the single-process line (the collective is a sum of one)
    d1 = _single_line()
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


def test_bench_gpus2_self_launches_two_ranks():
    """`python3 bench.py --gpus 2` with no torchrun environment (the way the
    driver may invoke it) starts the two ranks itself as a torchrun child
    process: the process group's world size is 2 (n_gpus counts distinct
    devices: 1 in this one-card rehearsal), and the estimate equals the
    single-process line's to rounding.  Rehearsed on one card: both ranks
    share GPU 0 over gloo."""
    d1 = _single_line("--mc-steps", "0")
    env = dict(os.environ, KT_BENCH_ONE_DEVICE="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "TORCHELASTIC_RUN_ID"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", *SMALL,
                        "--dist-backend", "gloo", "--no-profile", "--mc-steps", "0"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1  # rank 0's line, relayed
    d = lines[0]
    assert d["n_gpus"] == 1 and d["launch"]["process_group_world_size"] == 2
    assert d["launch"]["launcher"] == "torchrun" and d["config"]["parallelism"] == "probes sharded x2"
    assert d["trace_estimate"] == pytest.approx(d1["trace_estimate"], rel=1e-12)
    assert d["trace_stderr"] == pytest.approx(d1["trace_stderr"], rel=1e-12)

#!/usr/bin/env python3
"""bench.py -- trace(exp(A)) evaluations/s on the BASELINE.json metric config.

Workload (BASELINE.json metric / configs[3]): synthetic Chung-Lu scale-free
graph, n = 1,000,000, nnz = 10,000,000 (power law 2.5, unit weights, seeded),
one evaluation = plain Hutchinson over N = 1024 Rademacher probes, each with
m = 30 Lanczos steps + host Gauss quadrature.  A "step" is one evaluation.
Multi-GPU (torchrun, one process per GPU): the 1024 probes of each
evaluation are sharded over the ranks and one RCCL all-reduce of
(sum q, sum q^2) gives the trace -- strong scaling of a fixed evaluation.

Prints ONE JSON line on rank 0 (contract in the task statement).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# MI355X peaks (/opt/skills/guides/MI355X_MICROARCH.md, chip-level parameters)
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None,
                    help="timed evaluations (default 5; 100 with --config er100k, whose evaluations "
                         "take ~5 ms)")
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="sf1m", choices=["sf1m", "er100k"])
    ap.add_argument("--nprobes", type=int, default=None)
    ap.add_argument("--m", "--lanczos-m", dest="m", type=int, default=30)
    ap.add_argument("--block", type=int, default=0, help="probes per SpMM sweep (0 = auto)")
    ap.add_argument("--cpu-seconds", type=float, default=30.0,
                    help="CPU-baseline time budget (rank 0, N=1 only; stops earlier once half an "
                         "evaluation's probes are done); 0 disables")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU-baseline OpenMP threads (0 = every CPU this process may use)")
    ap.add_argument("--lanes", type=int, default=0,
                    help="probe sweeps in flight on separate HIP streams (KT_SLQ_LANES, 1..4; "
                         "0 = the library default: 2 for the y-form pass, 3 for the explicit sweep)")
    ap.add_argument("--explicit", action="store_true",
                    help="explicit K1/K2 CGS2 sweep instead of the y-form pass (KT_SLQ_YFORM=0)")
    ap.add_argument("--weighted", action="store_true",
                    help="seeded fp64 weights on the graph (graphs.symmetric_weights, uniform [0.5, 1.5)): "
                         "the weighted drivers' A, values read (12 B per nonzero)")
    ap.add_argument("--estimator", default="hutchinson", choices=["hutchinson", "mc_trace"],
                    help="headline estimator: plain Hutchinson over N probes (BASELINE configs[3]) or "
                         "trace_exp.m's own mc_trace structure (Lanczos-exp Afun, tol 1e-4, maxit 1000)")
    ap.add_argument("--mc-steps", type=int, default=5,
                    help="timed trace_exp (mc_trace) evaluations reported beside the headline "
                         "(0 = skip that leg unless --estimator mc_trace)")
    ap.add_argument("--ref-cpu-seconds", type=float, default=8.0,
                    help="trace_exp as the reference composes it (mc_trace + expmv Afun): one serial GPU "
                         "run, and the CPU restatements timed on bounded samples of it -- the C/OpenMP one "
                         "on one whole expmv call, the 1-thread SciPy one for this many seconds of Taylor "
                         "terms (rank 0, N=1, config sf1m, beside the mc_trace leg); 0 disables")
    ap.add_argument("--bitstable", action="store_true",
                    help="all-gather the per-probe forms and sum them in global probe order on every "
                         "rank (SURVEY §8e): the estimate is bit-identical for any number of ranks")
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="process-group backend for N > 1 (nccl = RCCL over xGMI; gloo only to "
                         "rehearse the multi-rank path, e.g. several ranks sharing one GPU with "
                         "KT_BENCH_ONE_DEVICE=1)")
    return ap.parse_args()


def make_graph(config, weighted=False):
    from krylov_robustness_amd import graphs
    if config == "sf1m":
        A, N, wl = (graphs.chung_lu(1_000_000, 10_000_000, gamma=2.5, seed=0), 1024,
                    "chung_lu n=1M nnz=10M gamma=2.5 (BASELINE configs[3])")
    else:
        A, N, wl = (graphs.erdos_renyi(100_000, 500_000, seed=0), 128,
                    "erdos_renyi n=100k nnz~1M (BASELINE configs[1])")
    if weighted:
        A = graphs.symmetric_weights(A, seed=1)
        wl += ", weighted: symmetric_weights(seed=1) uniform [0.5, 1.5)"
    return A, N, wl


def reference_trace(config, weighted=False):
    """tr(exp(A)) of the bench graph, or None for graphs without one:
      * sf1m: from its spectrum (tests/golden/config4_values.json, written in
        the build container by tests/golden/make_config4_fixture.py: scipy
        eigsh top 16, every other term bounded by exp(lambda_16));
      * er100k: the sum of all n diagonal entries e_i' exp(A) e_i, each by
        m = 30 Lanczos from e_i + Gauss quadrature (tests/golden/
        config2_values.json, make_config2_fixture.py), with the Rademacher
        Hutchinson estimator's exact standard error."""
    if config == "er100k" and not weighted:
        try:
            with open(os.path.join(ROOT, "tests", "golden", "config2_values.json")) as f:
                ex = json.load(f)["exact"]
        except (OSError, ValueError, KeyError):
            return None
        return {"value": ex["tr_exp"], "rel_uncertainty": ex["rel_uncertainty"],
                "hutchinson_stderr_per_probe": math.sqrt(ex["hutchinson_var_per_probe"]),
                "source": "tests/golden/config2_values.json: sum over all n rows of e_i' exp(A) e_i (m = 30 "
                          "Lanczos from e_i + Gauss quadrature; m = 45 agrees to 7e-14), exact Hutchinson "
                          "variance 2 (||exp A||_F^2 - sum exp(A)_ii^2) per probe"}
    if config != "sf1m":
        return None
    try:
        with open(os.path.join(ROOT, "tests", "golden", "config4_values.json")) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    spec = d["weighted"]["spectrum"] if weighted else d["spectrum"]
    return {"value": spec["tr_exp_topk"], "rel_uncertainty": spec["tr_exp_rel_uncertainty"],
            "lambda1": spec["lambda_desc"][0],
            "source": "tests/golden/config4_values.json: sum exp(lambda_i) over the top 16 "
                      "eigenvalues (scipy eigsh, tol 0), the rest bounded by (n-16) exp(lambda_16)"}


def cpu_share():
    """CPUs this process may actually use: the affinity mask, capped by the
    cgroup CPU quota when one is set (cgroup v2 cpu.max, v1 cfs_quota_us).
    Returns (cpus, detail)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    quota = None
    for path, parse in (("/sys/fs/cgroup/cpu.max", lambda t: t.split()),
                        ("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", None)):
        try:
            with open(path) as f:
                txt = f.read().strip()
        except OSError:
            continue
        if parse is not None:
            q, per = (parse(txt) + ["100000"])[:2]
            if q != "max":
                quota = int(q) / int(per)
        else:
            q = int(txt)
            if q > 0:
                with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                    quota = q / int(f.read().strip())
        break
    cpus = aff if quota is None else max(1, min(aff, int(math.floor(quota + 1e-9))))
    return cpus, {"affinity_cpus": aff, "cgroup_cpu_quota": quota, "host_cpus": os.cpu_count(),
                  "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS")}


def cpu_baseline(A, m, budget_s, nprobes_eval, threads=0):
    """Time the C restatement (oracle/slq_ref.c, OpenMP over probes) on a
    bounded sample of the same workload (at least half an evaluation's probes
    unless the time budget runs out first); extrapolate to evals/s.  Threads:
    every CPU the process may use (cpu_share) unless given."""
    from oracle import slq_ref
    share, detail = cpu_share()
    threads = int(threads) or share
    slq_ref.load()
    done = 0
    t0 = time.perf_counter()
    batch = threads
    target = max(1, nprobes_eval // 2)
    while True:
        slq_ref.slq_trace(A, batch, m, seed=12345, probe_offset=done, nthreads=threads)
        done += batch
        el = time.perf_counter() - t0
        if el >= budget_s or done >= target:
            break
    probes_per_s = done / el
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            model = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), None)
    except OSError:
        pass
    return {"value": probes_per_s / nprobes_eval, "unit": "evals/s", "cores": threads,
            "kind": "port", "cpu_model": model, **detail,
            "sample": f"{done} of the {nprobes_eval} probes of one evaluation (m={m}) in "
                      f"{el:.1f} s with {threads} OpenMP threads (every CPU this process may use: "
                      f"affinity mask capped by the cgroup quota), extrapolated"}


def _kernel_template_args(name):
    """'k_spmm_lanczos<16, 512, 10>' -> ('k_spmm_lanczos', ['16', '512', '10'])."""
    base, _, rest = name.partition("<")
    return base.strip(), [a.strip() for a in rest.rstrip(">").split(",")] if rest else []


def _pmc_traffic(kernel, P, config="sf1m", weighted=False):
    """HBM bytes per launch of the dominant kernel from the committed rocprofv3
    counter summary (profiles/traffic.json, section = the bench workload,
    written by tools/pmc_traffic.py from counter passes of this same bench
    command), or None.  Matches the kernel's name and its first template
    argument (the probe block P) exactly, so P = 1 never picks up P = 16."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        with open(path) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None
    sec = t.get(config + ("_weighted" if weighted else ""))
    if not isinstance(sec, dict):
        return None
    for k, v in sec.items():
        if k.startswith("_"):
            continue
        base, targs = _kernel_template_args(k)
        if base == kernel and targs[:1] == [str(P)] and isinstance(v, dict):
            return v.get("hbm_bytes_per_launch")
    return None


def _pmc_traffic_build(config="sf1m", weighted=False):
    """{csrc digest the section's counters were measured on, whether it is
    this tree's} -- a kernel change since the last PMC pass shows as False."""
    from krylov_robustness_amd._lib import source_digest
    try:
        with open(os.path.join(ROOT, "profiles", "traffic.json")) as f:
            sec = json.load(f).get(config + ("_weighted" if weighted else ""), {})
    except (OSError, ValueError):
        sec = {}
    rec = (sec.get("_build") or {}).get("csrc_sha256") if isinstance(sec, dict) else None
    cur = source_digest()
    return {"traffic_csrc_sha256": rec, "csrc_sha256": cur, "traffic_build_current": rec == cur}


def _metric_name(n, nnz):
    def short(x):
        for unit, div in (("M", 1_000_000), ("k", 1_000)):
            if x >= div and x % (div // 10 or 1) == 0:
                v = x / div
                return f"{v:g}{unit}"
        return str(x)
    # BASELINE.json's metric string, with n / nnz of the graph actually used
    return f"trace(exp(A)) evals/sec + achieved HBM GB/s, n={short(n)} nnz={short(nnz)}, 1/2/4/8 GPU"


def _hutchinson(s1, m2, N):
    """Plain Hutchinson over N probes: estimate = mean q, standard error from
    the sample variance of the N quadratic forms (m2 = sum (q - mean)^2)."""
    tr = s1 / N
    return tr, (math.sqrt(m2 / (N - 1) / N) if N > 1 else None)


def _pooled(sums, N):
    """Hutchinson over the forms of several evaluations of N probes each: the
    pooled mean and its standard error (Chan et al.'s combination of the
    per-evaluation centred moments)."""
    K = len(sums)
    mu = sum(s for s, _ in sums) / (N * K)
    m2 = sum(m for _, m in sums) + sum(N * (s / N - mu) ** 2 for s, _ in sums)
    return mu, (math.sqrt(m2 / (N * K - 1) / (N * K)) if N * K > 1 else None)


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def self_launch_cmd(nproc, argv, port):
    """The torchrun command bench.py runs as a child when asked for --gpus N
    > 1 without a torchrun environment: N ranks, one per GPU, same flags."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *argv]


def launch_guard(args, env=os.environ):
    """Before anything touches a GPU.  Returns None to run in this process,
    or the argv of a torchrun child that runs the N ranks:
      * no torchrun environment and --gpus N > 1: launch N ranks as a CHILD
        process (never exec: this process then only relays its exit status);
      * under torchrun: WORLD_SIZE must equal --gpus (a line that says N GPUs
        must have run on N ranks)."""
    if "WORLD_SIZE" not in env:
        if args.gpus > 1:
            return self_launch_cmd(args.gpus, sys.argv[1:], _free_port())
        return None
    world = int(env["WORLD_SIZE"])
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but torchrun started WORLD_SIZE={world} ranks")
    return None


def main():
    args = parse()
    if args.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    child = launch_guard(args)
    if child is not None:
        import subprocess
        rc = subprocess.run(child).returncode  # stdout/stderr inherited: rank 0's JSON line passes through
        sys.exit(rc)
    if args.steps is None:
        args.steps = 100 if args.config == "er100k" else 5
    if args.lanes == 0:
        args.lanes = 3 if args.explicit else 2
    os.environ["KT_SLQ_LANES"] = str(args.lanes)
    os.environ["KT_SLQ_YFORM"] = "0" if args.explicit else "1"
    import torch  # noqa: F401  -- load torch's HIP runtime first (one runtime per process)
    import torch.distributed as dist

    from krylov_robustness_amd import dist as kdist
    rank, world, local_rank = kdist.env_rank()
    if os.environ.get("KT_BENCH_ONE_DEVICE") == "1":  # rehearsal: every rank on GPU 0
        local_rank = 0
    # a process group whenever torchrun launched us -- at world 1 too, so the
    # RCCL init and the all-reduce run inside the process that holds
    # libkrylov_hip.so's streams exactly as at N > 1
    use_pg = world > 1 or "TORCHELASTIC_RUN_ID" in os.environ
    if use_pg:
        torch.cuda.set_device(local_rank)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world,
                                    device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", local_rank)
    coll_dev = dev if args.dist_backend == "nccl" else torch.device("cpu")  # where the sums meet

    import krylov_robustness_amd as kra
    A, N, wl = make_graph(args.config, args.weighted)
    if args.nprobes:
        N = args.nprobes
    m = args.m
    n, nnz = A.shape[0], A.nnz
    ctx = kra.Context(local_rank)
    D = kra.DeviceMatrix(A, ctx)
    off, cnt = kdist.probe_shard(N, rank, world)
    counts = [kdist.probe_shard(N, r, world)[1] for r in range(world)]
    # --bitstable plans the sweep width on the GLOBAL probe count and deals
    # whole sweeps to the ranks, so every world size runs each probe in the
    # same sweep (a guard redo recomputes a whole sweep)
    P = args.block or kra.slq_plan(D, N if args.bitstable else cnt, ctx=ctx)
    if args.bitstable:
        off, cnt = kdist.probe_shard_aligned(N, P, rank, world)
        counts = [kdist.probe_shard_aligned(N, P, r, world)[1] for r in range(world)]
    ref = reference_trace(args.config, args.weighted) if m >= 20 else None

    def submit(seed):
        return kra.slq_submit(D, cnt, m, seed=seed, probe_offset=off, block=P, ctx=ctx)

    coll_stats = {}

    def finish(pending):
        _, _, q = kra.slq_collect(pending)
        if args.bitstable:  # every rank reduces all N forms in global probe order
            return kdist.bitstable_sums(q, counts)
        # ONE collective per evaluation: all-gather of (count, sum, M2), Chan's
        # combination in rank order
        return kdist.moment_sums(q, device=coll_dev, force=use_pg, stats=coll_stats)

    def step(seed):
        return finish(submit(seed))

    def barrier():
        if use_pg:
            dist.barrier()
        torch.cuda.synchronize(dev)

    run_hutch = args.estimator == "hutchinson"
    extra = {}
    value = ms_per_step = None
    roof = None
    if run_hutch:
        for w in range(args.warmup):
            step(1000 + w)
        coll_stats.clear()
        if not args.no_profile:
            ctx.profile_reset()
            ctx.profile(True)
        barrier()
        t0 = time.perf_counter()
        # evaluations pipelined one deep: evaluation s's sweeps are queued on
        # the device before the host finishes evaluation s-1 (its quadrature
        # and reduction), so the host half hides under device work; every
        # evaluation is complete and reduced inside the timed region
        sums = []
        pending = None
        for s in range(args.steps):
            nxt = submit(s)
            if pending is not None:
                sums.append(finish(pending))
            pending = nxt
        if pending is not None:
            sums.append(finish(pending))
        barrier()
        el = time.perf_counter() - t0
        if not args.no_profile:
            ctx.profile(False)
        el_local = el
        el_max = kdist.allreduce_max(el, device=coll_dev, force=use_pg)
        # every rank's timed region (outside it): the spread says whether a
        # slow N > 1 line is one rank or all of them
        rank_el = [r[0] for r in kdist.allgather_floats([el], device=coll_dev)] if use_pg else [el]
        tr, tr_stderr = _hutchinson(*sums[-1], N)
        k1_overlapped = None
        timed = None
        if not args.no_profile:
            l1, ms1 = ctx.profile_read(0)
            k1_overlapped = round(ms1 / l1 * 1e3, 2) if l1 else None
            # union of the launches' event intervals over the lanes' streams:
            # time with >= 1 dominant launch in flight, overlap counted once
            timed = (l1, ctx.profile_busy(0)) if l1 else None
            # Roofline pass: with several lanes in flight the per-launch event
            # times include the other lanes' kernels, so the dominant kernel's
            # duration is measured on an isolated single-lane pass (4 sweeps of
            # the same P-probe block, m steps each) right after the timed region.
            os.environ["KT_SLQ_LANES"] = "1"
            ctx.profile_reset()
            ctx.profile(True)
            kra.slq_quadforms(D, 4 * P, m, seed=777, probe_offset=0, block=P, ctx=ctx)
            ctx.profile(False)
            os.environ["KT_SLQ_LANES"] = str(args.lanes)

        ms_per_step = el_max * 1e3 / args.steps
        value = args.steps / el_max
        # algorithmic bytes: one launch of the dominant kernel = one
        # Lanczos step of one P-probe sweep: CSR (12 nnz + 4(n+1)) + gather source,
        # previous vector, next vector (8nP each).  The y-form pass
        # (k_spmm_lanczos) moves exactly these streams; the explicit sweep's K1 is
        # charged the whole step although its K2 streams two of them.
        kbase = "k_spmm_dot" if args.explicit else "k_spmm_lanczos"
        kname = f"{kbase}<{P}"
        # SURVEY's per-unit figure charges fp64 values + int32 columns (12 B per
        # nonzero).  A unit-weight matrix (every stored value 1.0, detected when
        # the device matrix is created) never reads the values: its kernels'
        # compulsory CSR bytes are 4 B per nonzero, and that is the figure the
        # roofline fraction uses (the SURVEY figure is kept beside it, labelled).
        unit = bool(A.nnz) and bool(np.all(A.data == 1.0))
        per_nnz = 4 if unit else 12
        k1_bytes_survey = 12 * nnz + 4 * (n + 1) + 24 * n * P
        k1_bytes = per_nnz * nnz + 4 * (n + 1) + 24 * n * P
        sweeps = math.ceil(cnt / P)
        b_eval_rank = m * (sweeps * (per_nnz * nnz + 4 * (n + 1)) + 24 * n * cnt)
        b_eval_rank_survey = m * (sweeps * (12 * nnz + 4 * (n + 1)) + 24 * n * cnt)
        if not args.no_profile:
            l1, ms1 = ctx.profile_read(0)
            l2, ms2 = ctx.profile_read(1)
            if l1 and timed:
                iso_ms = ms1 / l1
                iso_gbs = k1_bytes / (iso_ms * 1e-3) / 1e9
                tl, busy_ms = timed
                # the union of this rank's launches lies inside its own timed
                # region (launches after t0, complete before the closing sync)
                # (GPU event clock vs host clock: a small edge skew is tolerated;
                # anything beyond 0.5 % marks the roofline fields suspect instead
                # of aborting the run)
                busy_ok = busy_ms <= el_local * 1e3 * 1.005
                if not busy_ok:
                    print(f"bench.py: WARNING profiled busy time {busy_ms:.3f} ms exceeds the timed region "
                          f"{el_local * 1e3:.3f} ms", file=sys.stderr)
                k1_ms = busy_ms / tl  # effective duration per launch in the timed region
                achieved = k1_bytes / (k1_ms * 1e-3) / 1e9
                # PMC bytes were profiled per graph (profiles/traffic.json keyed by
                # kernel and, for other graphs than sf1m, by config)
                traffic = _pmc_traffic(kbase, P, args.config, args.weighted)
                roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                        **_pmc_traffic_build(args.config, args.weighted),
                        "kernel": kname + ">", "avg_launch_us": round(k1_ms * 1e3, 2),
                        "launches": tl, "algorithmic_bytes_per_launch": k1_bytes,
                        "algorithmic_bytes_basis": ("unit-weight matrix: 4 nnz (int32 columns; values "
                                                    "never read) + 4 (n+1) + 24 n P" if unit else
                                                    "12 nnz + 4 (n+1) + 24 n P"),
                        "survey_bytes_per_launch": k1_bytes_survey,
                        "survey_frac": round(k1_bytes_survey / (k1_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                        "measured": "HIP events around every launch of the kernel in the timed region, "
                                    "on each sweep lane's stream; avg_launch_us = union of their intervals "
                                    "(time with >= 1 launch in flight, lane overlap counted once) / launches",
                        "timed_region_busy_ms": round(busy_ms, 3),
                        "busy_within_timed_region": busy_ok,
                        "timed_region_ms": round(el_local * 1e3, 3),
                        "timed_region_avg_launch_us_overlapped": k1_overlapped,
                        "isolated_pass": {"avg_launch_us": round(iso_ms * 1e3, 2), "launches": l1,
                                          "achieved": round(iso_gbs, 1),
                                          "frac": round(iso_gbs / HBM_PEAK_GBS, 4),
                                          "measured": "HIP events on a single-lane pass (4 sweeps x m "
                                                      "steps) after the timed region: the kernel alone"}}
                if traffic:  # memory-side rate: PMC bytes per launch over the same durations
                    tgbs = traffic / (k1_ms * 1e-3) / 1e9
                    roof["traffic_GBs"] = round(tgbs, 1)
                    roof["traffic_frac"] = round(tgbs / HBM_PEAK_GBS, 4)
                    roof["isolated_pass"]["traffic_GBs"] = round(traffic / (iso_ms * 1e-3) / 1e9, 1)
                if l2:
                    extra["k2_update_avg_us"] = round(ms2 / l2 * 1e3, 2)
                l3, ms3 = ctx.profile_read(2)
                if l3:
                    extra["start_pass_avg_us"] = round(ms3 / l3 * 1e3, 2)
        extra["sweep"] = "explicit K1/K2 CGS2" if args.explicit else "y-form single pass"
        extra["yform_redone_sweeps"] = ctx.yform_redone()
        eval_gbs = b_eval_rank / (ms_per_step * 1e-3) / 1e9
        extra["eval_roofline"] = {"B_eval_bytes_per_rank": b_eval_rank, "achieved_GBs_per_rank":
                                  round(eval_gbs, 1), "frac": round(eval_gbs / HBM_PEAK_GBS, 4),
                                  "B_eval_bytes_per_rank_survey": b_eval_rank_survey,
                                  "unit_weight_matrix": unit}
        coll = None
        if use_pg:
            us = coll_stats.get("us", [])
            coll = {"backend": "RCCL" if args.dist_backend == "nccl" else "gloo",
                    "op": ("all_gather of the per-probe forms, summed in global probe order" if args.bitstable
                           else "all_gather of each rank's (count, sum q, sum (q - shard mean)^2), combined "
                                "in rank order by Chan's pairwise formula"),
                    "calls_per_eval": (len(us) / args.steps) if not args.bitstable else 1,
                    "us_per_call_mean": round(sum(us) / len(us), 1) if us else None,
                    "us_per_call_max": round(max(us), 1) if us else None,
                    "measured": "host perf_counter around the collective and the read-back of its result "
                                "(inside the timed region), this rank"}
        extra["collective"] = coll
        extra["per_rank_timed_ms"] = {"min": round(min(rank_el) * 1e3, 3), "max": round(max(rank_el) * 1e3, 3),
                                      "ranks": len(rank_el)}
        extra["trace_estimate"] = tr
        extra["trace_stderr"] = tr_stderr
        extra["trace_stderr_basis"] = (f"sample standard deviation of the {N} per-probe quadratic "
                                       f"forms / sqrt({N}) (plain Hutchinson), last timed evaluation")
        ests = [_hutchinson(a, b, N)[0] for a, b in sums]
        pooled, pooled_se = _pooled(sums, N)
        extra["evaluations"] = {"seeds": f"0..{args.steps - 1}", "estimates": ests,
                                "pooled_estimate": pooled, "pooled_stderr": pooled_se,
                                "pooled_basis": f"all {N * len(sums)} forms of the timed evaluations"}
        if ref:
            extra["reference_trace"] = ref
            extra["rel_err"] = (tr - ref["value"]) / ref["value"]
            extra["err_in_stderr"] = (tr - ref["value"]) / tr_stderr if tr_stderr else None
            if "hutchinson_stderr_per_probe" in ref:  # the estimator's true standard error
                extra["err_in_true_stderr"] = (tr - ref["value"]) / (ref["hutchinson_stderr_per_probe"] /
                                                                     math.sqrt(N))
            extra["evaluations"]["rel_err"] = [(e - ref["value"]) / ref["value"] for e in ests]
            extra["evaluations"]["pooled_rel_err"] = (pooled - ref["value"]) / ref["value"]

    # ---- trace_exp.m's own estimator: mc_trace with the Lanczos-exp Afun ----
    mc = None
    mc_steps = args.mc_steps if run_hutch else max(args.mc_steps, 1)
    if args.estimator == "mc_trace" and args.steps:
        mc_steps = args.steps
    if mc_steps > 0:
        mc = _mc_trace_leg(args, kra, kdist, D, ctx, m, mc_steps, use_pg, barrier, coll_dev, world, ref,
                           n, nnz, A)
        if rank == 0 and world == 1 and args.ref_cpu_seconds > 0 and args.config == "sf1m":
            mc["reference_composition"] = _reference_composition(kra, D, ctx, A, ref, args.ref_cpu_seconds)
        if not run_hutch:
            value, ms_per_step = mc.pop("evals_per_s"), mc.pop("ms_per_eval")
            roof = mc.pop("roofline")
            extra.update({k: mc.pop(k) for k in list(mc) if k not in ("estimator",)})
            extra["estimator"] = mc["estimator"]
            mc = None

    cpu = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0 and run_hutch:
        cpu = cpu_baseline(A, m, args.cpu_seconds, N, args.cpu_threads)

    pg_world = dist.get_world_size() if use_pg else None
    # distinct GPUs: a one-device rehearsal (every rank on GPU 0) is 1 GPU
    one_dev = os.environ.get("KT_BENCH_ONE_DEVICE") == "1"
    n_devices = 1 if one_dev else (pg_world if use_pg else world)
    if rank == 0:
        cfg = {"workload": wl, "n": n, "nnz": nnz, "lanczos_m": m, "fun": "exp"}
        if run_hutch:
            cfg.update({"estimator": "plain Hutchinson (BASELINE configs[3])", "probes_per_eval": N,
                        "probes_per_sweep": P, "sweep_lanes": args.lanes,
                        "parallelism": f"probes sharded x{world}"})
        else:
            cfg.update({"estimator": "mc_trace (trace_exp.m:5-6: tol 1e-4, maxit 1000, Lanczos-exp Afun)",
                        "parallelism": f"G-probe columns dealt over x{world}, S/Q replicated"})
        out = {
            "metric": _metric_name(n, nnz),
            "value": round(value, 4), "unit": "evals/s", "n_gpus": n_devices,
            "steps": args.steps if run_hutch else mc_steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
            "config": cfg, "roofline": roof, "cpu_baseline": cpu,
            **extra,
        }
        out["launch"] = {"process_group_world_size": pg_world, "backend": args.dist_backend if use_pg else None,
                         "launcher": ("torchrun" if "TORCHELASTIC_RUN_ID" in os.environ else "single process"),
                         "one_device_rehearsal": os.environ.get("KT_BENCH_ONE_DEVICE") == "1"}
        if mc is not None:
            out["mc_trace"] = mc
        print(json.dumps(out), flush=True)
    if use_pg:
        dist.destroy_process_group()


def _reference_composition(kra, D, ctx, A, ref, budget_s):
    """trace_exp as the reference composes it (trace_exp.m:5-6: mc_trace with
    the expmv Afun; expmv.m with select_taylor_degree.m / normAm.m) on the
    bench graph, twice:
      * on the GPU, once: kt_mc_trace with the device expmv Afun, serial
        (KT_TWIN=0, KT_MC_SPEC=0: every expmv call on this context, counted
        by kt_context_stat 3 / 4);
      * SURVEY §8d plan (i)'s CPU baseline, the same algorithm restated in C
        + OpenMP (oracle/mctrace_ref.c) on every CPU this process may use:
        one whole expmv call (round 1's S block, every stage and term) and a
        round's host work (qr, projection), extrapolated from that whole call
        to the GPU run's call / term / round counts; beside it the numpy /
        SciPy restatement (oracle/krylov_oracle.py) on one thread, a shorter
        sample (one select_taylor_degree call, the first Taylor terms)."""
    from oracle import krylov_oracle as O
    saved = {k: os.environ.get(k) for k in ("KT_TWIN", "KT_MC_SPEC")}
    os.environ["KT_TWIN"] = "0"
    os.environ["KT_MC_SPEC"] = "0"
    try:
        # one untimed call first (seed 1), as the headline's warm-up: the
        # natural-order CSR and its task lists are built on first use and
        # select_taylor_degree's result is cached per matrix version (the
        # same inputs give the same (s, m) every call), so the timed call is
        # a steady-state trace_exp on a resident A -- the drop-in's
        # situation across MATLAB calls (kt_mex.cpp keeps A on the device)
        kra.mc_trace("expmv", None, 1e-4, 1000, 1, 0, seed=1, A=D, ctx=ctx)
        c0, k0 = ctx.stat(3), ctx.stat(4)
        ctx.profile_reset()
        ctx.profile(True)  # HIP events around every Taylor-term launch (slot 4)
        t0 = time.perf_counter()
        tr, res, it = kra.mc_trace("expmv", None, 1e-4, 1000, 1, 0, seed=0, A=D, ctx=ctx)
        gpu_s = time.perf_counter() - t0
        ctx.profile(False)
        calls, terms = ctx.stat(3) - c0, ctx.stat(4) - k0
        t_launches, t_ms = ctx.profile_read(4)
        t_busy = ctx.profile_busy(4)
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    out = {"afun": "expmv (trace_exp.m:5-6 as the reference composes it), tol 1e-4, maxit 1000, seed 0",
           "gpu_ms": round(gpu_s * 1e3, 2), "gpu_evals_per_s": round(1.0 / gpu_s, 4), "rounds": it,
           "trace_estimate": tr, "expmv_calls": calls, "taylor_terms": terms,
           "gpu_mode": "serial: every expmv call on one stream (KT_TWIN=0, KT_MC_SPEC=0); after one "
                       "untimed warm-up call (seed 1: CSR build, cached Taylor-degree selection)"}
    if ref:
        out["rel_err"] = (tr - ref["value"]) / ref["value"]
    # the term kernel's roofline: one active term = expmv.m:75-78 on the
    # n x 10 block, P = 16 padded: CSR (4 nnz + 4 (n+1), unit weights) + the
    # gathered block b (8 n P, each row once) + f read and written + b_next
    # written (3 x 8 n P); "useful" prices the 10 live columns only
    n, nnz = A.shape[0], A.nnz
    unit = bool(A.nnz) and bool(np.all(A.data == 1.0))
    csr_b = (4 if unit else 12) * nnz + 4 * (n + 1)
    P, nc = 16, 10
    padded, useful = csr_b + 32 * n * P, csr_b + 32 * n * nc
    if terms and t_launches:
        us = t_busy * 1e3 / terms  # launch time (no-op launches included) per active term
        gbs = padded / (us * 1e-6) / 1e9
        traffic = _pmc_traffic("k_expmv_rows", P, "expmv_c4")
        roof = {"kernel": "k_expmv_rows<16>", "bound": "hbm", "unit": "GB/s", "peak": HBM_PEAK_GBS,
                "active_terms": terms, "launches": t_launches, "busy_ms": round(t_busy, 2),
                "us_per_active_term": round(us, 2),
                "bytes_per_term_padded": padded, "bytes_per_term_useful": useful,
                "achieved": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4),
                "useful_frac": round(useful / (us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
                "traffic": traffic, **_pmc_traffic_build("expmv_c4"),
                "measured": "HIP events around every term launch on the context's stream (one stream: "
                            "the union is the sum); us_per_active_term = busy / active terms, the "
                            "~4 us no-op launches past a stage's stop included"}
        if traffic:
            roof["traffic_GBs"] = round(traffic / (us * 1e-6) / 1e9, 1)
        out["roofline"] = roof
    Acsr = A.tocsr()
    n = Acsr.shape[0]
    # (1) the C + OpenMP restatement of the same algorithm (oracle/mctrace_ref.c)
    # on every CPU this process may use: ONE WHOLE trace_exp evaluation
    # (trace_exp.m:5-6, seed 0: every mc_trace round, qr, projection, expmv
    # call and Taylor term), timed -- a measurement, not an extrapolation
    # (about a minute on 16 cores; --ref-cpu-seconds 0 skips the CPU legs)
    from oracle import mctrace_ref as MR
    cores, detail = cpu_share()
    t0 = time.perf_counter()
    tr_c, res_c, it_c, st = MR.trace_exp(Acsr, seed=0, tol=1e-4, maxit=1000, nthreads=cores)
    cpu_s = time.perf_counter() - t0
    out["cpu_baseline"] = {
        "value": 1.0 / cpu_s, "unit": "evals/s", "cores": cores, "kind": "port",
        "algorithm": "the reference's: mc_trace + expmv + select_taylor_degree + normAm "
                     "(oracle/mctrace_ref.c, C + OpenMP over rows; equals the numpy restatement)",
        "seconds_per_eval": round(cpu_s, 2),
        "sample": f"one whole evaluation (seed 0, the GPU run's seed: {it_c} rounds, every expmv call and "
                  f"Taylor term, qr and projection) on {cores} OpenMP threads, timed",
        "trace_estimate": tr_c, "rounds": it_c,
        "rel_diff_vs_gpu": (tr_c - tr) / tr if tr else None,
        "stats": st, **detail}
    S1 = O.rademacher(n, range(10), 0)
    # (2) beside it, the numpy/SciPy restatement (oracle/krylov_oracle.py) on ONE
    # thread (SciPy's sparse @ dense is single-threaded), a shorter sample: one
    # select_taylor_degree call and the first Taylor terms of one 10-column call
    b = S1.copy()
    t0 = time.perf_counter()
    O.select_taylor_degree(Acsr, b)
    t_sel = time.perf_counter() - t0
    f = b.copy()
    k = 0
    ratio = 0.0  # the stop test's c2 / norm(f, inf), kept so the norms are used
    t0 = time.perf_counter()
    while k < 200 and (k == 0 or time.perf_counter() - t0 < budget_s):
        k += 1
        b = (1.0 / (20.0 * k)) * (Acsr @ b)  # b = (t/(s k)) A b, expmv.m:75 (mu = 0: no diagonal)
        f = f + b
        c2 = np.max(np.sum(np.abs(b), axis=1))  # the stop test's norms, expmv.m:79-80
        nf = np.max(np.sum(np.abs(f), axis=1))
        ratio = c2 / nf if nf > 0 else ratio
    t_term1 = (time.perf_counter() - t0) / k
    est1 = calls * t_sel + terms * t_term1
    out["cpu_baseline_scipy_1thread"] = {
        "value": 1.0 / est1 if est1 > 0 else None, "unit": "evals/s", "cores": 1, "kind": "port",
        "algorithm": "the reference's: mc_trace + expmv (oracle/krylov_oracle.py restatement, SciPy)",
        "seconds_per_eval": round(est1, 1), "select_taylor_degree_s": round(t_sel, 3),
        "taylor_term_s": round(t_term1, 4), "sample_last_c2_over_normf": ratio,
        "sample": f"one select_taylor_degree call ({t_sel:.1f} s) and {k} Taylor terms on a 10-column "
                  f"block ({t_term1:.3f} s each), one thread, extrapolated to the GPU run's {calls} expmv "
                  f"calls and {terms} Taylor terms (mc_trace's QR and projections left out: a lower bound)"}
    return out


def _mc_trace_leg(args, kra, kdist, D, ctx, m, steps, use_pg, barrier, coll_dev, world, ref, n, nnz, A):
    """tr = trace_exp(A) as trace_exp.m:5-6 computes it: mc_trace's block
    Hutchinson with nested deflation (mc_trace.m:42-58; K = ceil(1000/30)
    rounds at most, stop at relative change < 1e-4) with the Lanczos-exp Afun
    (m steps per column).  At N > 1 kt_mc_trace_sharded: S, Q replicated, the
    10 G columns of each round dealt over the ranks, one all-reduce per round.
    Timed like the headline (barrier + sync on both sides, max over ranks);
    the dominant kernel's duration from an isolated serial pass (KT_TWIN=0)."""
    def one(seed):
        if use_pg:
            return kdist.mc_trace_sharded("lanczos", None, 1e-4, 1000, 1, 0, seed, "exp", m, A=D, ctx=ctx,
                                          force=True)
        return kra.mc_trace("lanczos", None, 1e-4, 1000, 1, 0, seed=seed, fun="exp", m=m, A=D, ctx=ctx)

    one(1000)  # warm-up: twin matrices, workspaces
    redone0 = ctx.yform_redone()
    barrier()
    t0 = time.perf_counter()
    res = [one(s) for s in range(steps)]
    barrier()
    el = kdist.allreduce_max(time.perf_counter() - t0, device=coll_dev, force=use_pg)
    tr, r_last, it = res[-1]
    out = {"estimator": "mc_trace (trace_exp.m:5-6 via mc_trace.m:42-58, Lanczos-exp Afun, m=%d)" % m,
           "evals_per_s": round(steps / el, 4), "ms_per_eval": round(el * 1e3 / steps, 3),
           "timed_evals": steps, "trace_estimate": tr, "rounds": it, "res": r_last,
           "rounds_per_eval": [r[2] for r in res],
           "probe_columns_per_eval": 30 * it,
           "yform_redone_sweeps": ctx.yform_redone() - redone0,
           "probe_columns_basis": "per round: 10 S columns, the 10 columns of Q, 10 G columns "
                                  "(mc_trace.m:43-49), each one m-step Lanczos run"}
    if ref:
        out["reference_trace"] = ref["value"]
        out["rel_err"] = (tr - ref["value"]) / ref["value"]
        out["rel_err_max_over_evals"] = max(abs(r[0] - ref["value"]) / ref["value"] for r in res)
    out["roofline"] = None
    if not args.no_profile:
        # isolated serial pass: every Afun call on this context (no twin threads)
        prev = os.environ.get("KT_TWIN")
        os.environ["KT_TWIN"] = "0"
        ctx.profile_reset()
        ctx.profile(True)
        t1 = time.perf_counter()
        kra.mc_trace("lanczos", None, 1e-4, 1000, 1, 0, seed=777, fun="exp", m=m, A=D, ctx=ctx)
        serial_ms = (time.perf_counter() - t1) * 1e3
        ctx.profile(False)
        if prev is None:
            os.environ.pop("KT_TWIN")
        else:
            os.environ["KT_TWIN"] = prev
        unit = bool(A.nnz) and bool(np.all(A.data == 1.0))
        per_nnz = 4 if unit else 12
        # mc_trace_batched's sweep passes (kt_mctrace.cpp): round 1's S term
        # and a round with the next S term ahead run the explicit sweep (K1 =
        # k_spmm_dot, slot 0), 16 wide; a round's quadrature-only columns run
        # y-form passes of block-seeded sweeps (k_spmm_lanczos, slot 3), 16
        # wide and at the power of two of a remainder.  Each launch is charged
        # its own width's algorithmic bytes; a kernel's time is the union of
        # its launches' HIP-event intervals (overlapping lanes counted once).
        kinds = {
            "k_spmm_dot": (0, lambda P: per_nnz * nnz + 4 * (n + 1) + 16 * n * P,
                           f"{per_nnz} nnz + 4 (n+1) + 16 n P (the CSR, u_j gathered once, y = A u_j written)"),
            "k_spmm_lanczos": (3, lambda P: per_nnz * nnz + 4 * (n + 1) + 24 * n * P,
                               f"{per_nnz} nnz + 4 (n+1) + 24 n P (the CSR, y_j gathered once, y_j and "
                               "y_(j-1) own rows read, y_(j+1) written)"),
        }
        rf = {}
        for name, (slot, kb, basis) in kinds.items():
            nl, ms_sum = ctx.profile_read(slot)
            if not nl:
                continue
            busy = ctx.profile_busy(slot)
            widths = {P: ctx.profile_read_width(slot, P) for P in (1, 2, 4, 8, 16, 32)}
            widths = {P: v for P, v in widths.items() if v[0]}
            bytes_total = sum(v[0] * kb(P) for P, v in widths.items())
            gbs = bytes_total / (busy * 1e-3) / 1e9
            tr = {P: _pmc_traffic(name, P, args.config, args.weighted) for P in widths}
            traffic = (sum(widths[P][0] * tr[P] for P in widths) / nl) if all(tr.values()) else None
            e = {"bound": "hbm", "kernel": f"{name}<{'|'.join(str(P) for P in sorted(widths))}>",
                 "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                 "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": traffic,
                 "avg_launch_us": round(busy / nl * 1e3, 2), "launches": nl, "busy_ms": round(busy, 3),
                 "launches_by_width": {str(P): v[0] for P, v in widths.items()},
                 "avg_launch_us_by_width": {str(P): round(v[1] / v[0] * 1e3, 2) for P, v in widths.items()},
                 "avg_launch_us_overlapped": round(ms_sum / nl * 1e3, 2),
                 "algorithmic_bytes_per_launch": round(bytes_total / nl),
                 "algorithmic_bytes_basis": basis + " per launch, at the launch's sweep width P; mean"}
            if traffic:
                e["traffic_GBs"] = round(traffic * nl / (busy * 1e-3) / 1e9, 1)
            rf[name] = e
        if rf:
            main_k = max(rf, key=lambda k: rf[k]["busy_ms"])  # the dominant kernel: most time in flight
            out["roofline"] = dict(rf[main_k])
            out["roofline"]["other_kernels"] = {k: v for k, v in rf.items() if k != main_k}
            l2, ms2 = ctx.profile_read(1)
            out["roofline"]["k2_update_avg_us"] = round(ms2 / l2 * 1e3, 2) if l2 else None
            out["roofline"]["serial_eval_ms"] = round(serial_ms, 2)
            out["roofline"]["measured"] = (
                "HIP events around every sweep pass of one trace_exp after the timed region; avg_launch_us = "
                "union of the kernel's launch intervals (time with >= 1 launch in flight) / launches; the "
                "explicit and y-form sweeps of a round run side by side on two lanes, so each kernel's "
                "launches share the chip with the other's")
            # the whole evaluation: every sweep pass's algorithmic bytes (K1,
            # K2 with its basis stores, y-form passes) over the evaluation's
            # wall time, the two lanes' concurrency included
            k2_bytes = sum(ctx.profile_read_width(1, P)[0] * 32 * n * P for P in (1, 2, 4, 8, 16, 32))
            sweep_bytes = sum(rf[k]["algorithmic_bytes_per_launch"] * rf[k]["launches"] for k in rf) + k2_bytes
            eb = sweep_bytes / (serial_ms * 1e-3) / 1e9
            out["eval_roofline"] = {"sweep_bytes_per_eval": int(sweep_bytes), "eval_ms": round(serial_ms, 2),
                                    "achieved_GBs": round(eb, 1), "frac": round(eb / HBM_PEAK_GBS, 4),
                                    "basis": "sum over the evaluation's sweep launches of their algorithmic "
                                             "bytes (K1 and y-form passes as in roofline; K2 32 n P, its basis "
                                             "stores not counted) / the serial evaluation's wall time"}
    return out


if __name__ == "__main__":
    main()

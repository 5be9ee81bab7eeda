"""bench.py's launch contract, host side (no GPU): --gpus N > 1 without a
torchrun environment runs N ranks as a torchrun CHILD process (never an
exec); under torchrun, WORLD_SIZE must equal --gpus."""
import os
import subprocess
import sys
from types import SimpleNamespace

import pytest

from conftest import ROOT

sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_single_gpu_runs_in_process():
    assert bench.launch_guard(SimpleNamespace(gpus=1), env={}) is None


def test_gpus_n_without_torchrun_launches_n_ranks(monkeypatch):
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8", "--steps", "3"])
    cmd = bench.launch_guard(SimpleNamespace(gpus=8), env={})
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    i = cmd.index("--master-addr")
    assert cmd[i + 1] == "127.0.0.1"
    assert 0 < int(cmd[cmd.index("--master-port") + 1]) < 65536
    assert cmd[-4:] == ["--gpus", "8", "--steps", "3"]
    assert os.path.samefile(cmd[-5], os.path.join(ROOT, "bench.py"))


def test_under_torchrun_world_must_match():
    assert bench.launch_guard(SimpleNamespace(gpus=4), env={"WORLD_SIZE": "4"}) is None
    with pytest.raises(SystemExit, match="WORLD_SIZE=2"):
        bench.launch_guard(SimpleNamespace(gpus=8), env={"WORLD_SIZE": "2"})


def test_world_mismatch_exits_before_any_gpu_work():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1"], capture_output=True,
                       text=True, timeout=60, cwd=ROOT, env=env)
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]

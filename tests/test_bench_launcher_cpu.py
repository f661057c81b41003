"""bench.py's N-GPU entry: `python bench.py --gpus N` with no launcher
spawns N ranks through torch.distributed.run as a child process, making no HIP call itself
(the reference's mp.spawn world, train_denseclip.py:1649-1657); under a launcher --gpus must
equal WORLD_SIZE.  CPU only: the spawn itself is exercised with a gloo stand-in worker."""
import json
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_gpus_one_runs_in_process():
    assert bench.resolve_world(bench.parse(["--gpus", "1"]), env={}) == (1, False)
    assert bench.resolve_world(bench.parse([]), env={}) == (1, False)


def test_gpus_n_without_launcher_spawns():
    assert bench.resolve_world(bench.parse(["--gpus", "8"]), env={}) == (8, True)


def test_under_launcher_gpus_must_match_world():
    env = {"WORLD_SIZE": "4", "RANK": "1", "LOCAL_RANK": "1"}
    assert bench.resolve_world(bench.parse(["--gpus", "4"]), env=env) == (4, False)
    assert bench.resolve_world(bench.parse([]), env=env) == (4, False)
    with pytest.raises(SystemExit):
        bench.resolve_world(bench.parse(["--gpus", "2"]), env=env)
    with pytest.raises(SystemExit):
        bench.resolve_world(bench.parse(["--gpus", "0"]), env={})


def test_launch_cmd_and_env():
    argv = ["--gpus", "8", "--steps", "20", "--warmup", "5"]
    cmd = bench.launch_cmd(argv, 8, 29512)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nnodes=1" in cmd and "--nproc-per-node=8" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29512" in cmd
    i = cmd.index(os.path.join(ROOT, "bench.py"))
    assert cmd[i + 1:] == argv  # the ranks see the same arguments, --gpus 8 included
    env = bench.launch_env({"WORLD_SIZE": "3", "RANK": "0", "MASTER_PORT": "1", "PATH": "/bin"})
    assert "WORLD_SIZE" not in env and "RANK" not in env and "MASTER_PORT" not in env
    assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0" and env["PATH"] == "/bin"


def test_parent_makes_no_hip_call(monkeypatch):
    """main() with --gpus 2 and no launcher hands off before touching torch.cuda."""
    calls = []

    def forbidden(*a, **k):
        raise AssertionError("the launching parent touched the GPU")

    for name in ("is_available", "device_count", "set_device", "synchronize", "current_device", "init"):
        monkeypatch.setattr(torch.cuda, name, forbidden)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setattr(bench, "spawn_ranks", lambda argv, n, script=None: calls.append((list(argv), n)) or 7)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2", "--steps", "3"])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 7  # the child's status is ours
    assert calls == [(["--gpus", "2", "--steps", "3"], 2)]


@pytest.mark.timeout(240)
def test_spawn_ranks_runs_n_ranks(capfd):
    """The real child launch (torch.distributed.run, 2 ranks, gloo stand-in worker): rank 0's
    JSON line reaches our stdout and reports the process group's size and an all-reduce of
    ones over it."""
    stub = os.path.join(ROOT, "tests", "stubs", "rank_stub.py")
    rc = bench.spawn_ranks(["--gpus", "2", "--steps", "1"], 2, script=stub)
    out = capfd.readouterr().out
    assert rc == 0, out
    lines = [json.loads(ln) for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    assert lines[0]["n_gpus"] == 2 and lines[0]["rccl_ranks"] == 2
    assert lines[0]["argv"] == ["--gpus", "2", "--steps", "1"]

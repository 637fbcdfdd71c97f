"""bench.py --gpus N: the rank plan and the launch wiring (CPU; no rank touches the GPU under
--launch-check).  The driver's scaling run calls `python bench.py --gpus N` or launches the ranks
itself with torch.distributed.run; both must end with N ranks, and a WORLD_SIZE that disagrees with
--gpus must fail instead of reporting a rank count that did not run."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_rank_plan():
    assert bench.rank_plan(None, {}) == ("run", 1)
    assert bench.rank_plan(1, {}) == ("run", 1)
    assert bench.rank_plan(2, {}) == ("launch", 2)
    assert bench.rank_plan(8, {}) == ("launch", 8)
    assert bench.rank_plan(None, {"WORLD_SIZE": "4"}) == ("run", 4)
    assert bench.rank_plan(4, {"WORLD_SIZE": "4"}) == ("run", 4)
    with pytest.raises(SystemExit):
        bench.rank_plan(2, {"WORLD_SIZE": "4"})
    with pytest.raises(SystemExit):
        bench.rank_plan(0, {})


def test_launch_cmd_is_the_drivers_form():
    cmd = bench.launch_cmd(4, ["--gpus", "4", "--steps", "3"], 29600)
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--master-addr=127.0.0.1" in cmd and "--master-port=29600" in cmd
    assert cmd[-4:] == ["--gpus", "4", "--steps", "3"]
    assert cmd[cmd.index("--master-port=29600") + 1].endswith("bench.py")


def _run(args, extra_env=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(extra_env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT, env=env,
                          capture_output=True, text=True, timeout=180)


def test_gpus_2_launches_two_ranks():
    r = _run(["--gpus", "2", "--launch-check"])
    assert r.returncode == 0, r.stderr
    lines = [json.loads(s) for s in r.stdout.splitlines() if s.startswith("{")]
    assert sorted(d["rank"] for d in lines) == [0, 1]
    assert all(d["world"] == 2 for d in lines)
    assert sorted(d["local_rank"] for d in lines) == [0, 1]
    assert all(d["master"].startswith("127.0.0.1:") for d in lines)


def test_gpus_1_runs_in_process():
    r = _run(["--launch-check"])
    assert r.returncode == 0, r.stderr
    lines = [json.loads(s) for s in r.stdout.splitlines() if s.startswith("{")]
    assert lines == [{"rank": 0, "world": 1, "local_rank": 0, "master": "None:None"}]


def test_world_size_mismatch_fails():
    r = _run(["--gpus", "2", "--launch-check"], {"WORLD_SIZE": "3", "RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE=3" in r.stderr


def test_native_selfcheck_keeps_or_drops_the_native_exchange():
    """bench._native_selfcheck: the native communicator stays only if every rank's comparison with the
    torch.distributed exchange passed; a mismatch or an exception closes it and reports why (a
    one-rank gloo group in this process stands in for the ranks)."""
    import socket

    import torch.distributed as dist

    class Fake:
        closed = False

        def close(self):
            self.closed = True

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    own = not dist.is_initialized()
    if own:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        f = Fake()
        kept, note = bench._native_selfcheck(f, dist, "cpu", lambda: True, "payload")
        assert kept is f and not f.closed and note.startswith("native == torch.distributed")
        f = Fake()
        kept, note = bench._native_selfcheck(f, dist, "cpu", lambda: False, "payload")
        assert kept is None and f.closed and "torch.distributed exchange used" in note

        def boom():
            raise RuntimeError("collective timed out")

        f = Fake()
        kept, note = bench._native_selfcheck(f, dist, "cpu", boom, "payload")
        assert kept is None and f.closed and "collective timed out" in note
    finally:
        if own:
            dist.destroy_process_group()

"""bench.py's launch logic (CPU): --gpus N never yields a line that measured another number of GPUs.

The driver launches N > 1 through torch.distributed.run; a bare `python bench.py --gpus N` starts the N
ranks itself (one child process per GPU, nothing in the parent touches the GPU), and a node with fewer
GPUs than asked -- or a WORLD_SIZE that disagrees with --gpus -- is an error (exit 2, no JSON line)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_single_gpu_runs_in_process():
    assert bench.launch_plan(1, {}, 0) == ("run", None)
    assert bench.launch_plan(1, {"WORLD_SIZE": "1", "RANK": "0"}, 1) == ("run", None)


def test_launched_rank_runs_in_process():
    env = {"WORLD_SIZE": "8", "RANK": "3", "LOCAL_RANK": "3", "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": "29500"}
    assert bench.launch_plan(8, env, 8) == ("run", None)


def test_world_size_disagreeing_with_gpus_is_an_error():
    act, msg = bench.launch_plan(8, {"WORLD_SIZE": "1"}, 8)
    assert act == "error" and "WORLD_SIZE=1" in msg
    act, _ = bench.launch_plan(1, {"WORLD_SIZE": "2", "LOCAL_RANK": "0"}, 2)
    assert act == "error"


def test_ranks_sharing_a_gpu_are_an_error():
    act, msg = bench.launch_plan(2, {"WORLD_SIZE": "2", "RANK": "1", "LOCAL_RANK": "1"}, 1)
    assert act == "error" and "1 GPU" in msg


def test_fewer_gpus_than_asked_is_an_error():
    for n, have in ((2, 1), (8, 1), (8, 4), (2, 0)):
        act, msg = bench.launch_plan(n, {}, have)
        assert act == "error" and f"--gpus {n}" in msg


def test_no_launcher_spawns_one_rank_per_gpu():
    act, envs = bench.launch_plan(4, {"PATH": "/usr/bin"}, 8)
    assert act == "spawn" and len(envs) == 4
    ports = {e["MASTER_PORT"] for e in envs}
    assert len(ports) == 1 and int(ports.pop()) > 0
    for r, e in enumerate(envs):
        assert (e["RANK"], e["LOCAL_RANK"], e["WORLD_SIZE"]) == (str(r), str(r), "4")
        assert e["MASTER_ADDR"] == "127.0.0.1" and e["PATH"] == "/usr/bin"


def test_nonpositive_gpus_is_an_error():
    assert bench.launch_plan(0, {}, 8)[0] == "error"


def test_bare_multi_gpu_run_without_gpus_fails_fast():
    """This container has no GPU: `python bench.py --gpus 2` must exit non-zero with a message and no
    JSON line on stdout (the one-GPU box behaves the same: 1 < 2)."""
    env = {k: v for k, v in os.environ.items() if k not in bench.LAUNCH_ENV}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 2, r.stderr[-2000:]
    assert "refusing to measure fewer GPUs" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_spawn_ranks_propagates_a_failing_rank(tmp_path):
    """spawn_ranks returns the first non-zero exit status and kills ranks still running after the grace
    period by their own process group (here a stand-in script: rank 1 fails, rank 0 would hang)."""
    script = tmp_path / "rank.py"
    script.write_text("import os, sys, time\n"
                      "r = int(os.environ['RANK'])\n"
                      "if r == 1: sys.exit(5)\n"
                      "time.sleep(600)\n")
    envs = [dict(os.environ, RANK=str(r), WORLD_SIZE="2") for r in range(2)]
    orig = bench.__file__
    try:
        bench.__file__ = str(script)
        t0 = __import__("time").monotonic()
        rc = bench.spawn_ranks(envs, [], grace_s=1.0)
        assert __import__("time").monotonic() - t0 < 60
    finally:
        bench.__file__ = orig
    assert rc == 5


def test_user_program_leg_reports_the_launch_choice(tmp_path, monkeypatch):
    """bench.py's user-kernel leg (user_program_run) takes the program's median frame time and passes
    its launch choice (register target, blocks per CU, LDS stack entries) into the line; a failing or
    absent program gives an error / null, never a number."""
    tests_dir = tmp_path / "build" / "tests"
    tests_dir.mkdir(parents=True)
    prog = tests_dir / "fake_uk"
    prog.write_text("#!/bin/sh\necho '{\"mode\":\"bench\",\"frame_ms_median\":1.5,\"launches\":4,\"frames_per_launch\":32,"
                    "\"launch\":{\"waves_target\":6,\"blocks_per_cu\":24,\"stack_entries\":24,\"grid\":6144}}'\n")
    prog.chmod(0o755)
    bad = tests_dir / "bad_uk"
    bad.write_text("#!/bin/sh\nexit 3\n")
    bad.chmod(0o755)
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    leg = bench.user_program_run("fake_uk", 1920, 1080, 15_000_000)
    assert leg["mrays"] == 10000.0 and leg["frame_ms_median"] == 1.5
    assert leg["launch"] == {"waves_target": 6, "blocks_per_cu": 24, "stack_entries": 24, "grid": 6144}
    assert "error" in bench.user_program_run("bad_uk", 1920, 1080, 15_000_000)
    assert bench.user_program_run("absent_uk", 1920, 1080, 15_000_000) is None

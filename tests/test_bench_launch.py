"""bench.py's multi-rank launch path, on the CPU with gloo.

`python bench.py --gpus N` started without a torchrun environment must start N rank processes
itself (torch.distributed.run children, before any GPU call in the parent) and every rank must
refuse a world that is not --gpus. `--check-launch` stops each rank after the world / backend
checks, so the launch path runs here without a GPU (gloo is the backend off a GPU node).
"""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def _env():
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "ACKPHYS_DIST_BACKEND",
              "ACKPHYS_DEVICE_OVERRIDE"):
        env.pop(k, None)
    env["OMP_NUM_THREADS"] = "1"
    return env


def _json_lines(out: str):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


def test_launch_command_shape():
    import bench
    cmd = bench.launch_command(["--gpus", "8", "--steps", "20"], 8, 29500)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd and "--master-addr=127.0.0.1" in cmd
    assert "--master-port=29500" in cmd
    i = cmd.index(os.path.abspath(bench.__file__))
    assert cmd[i + 1:] == ["--gpus", "8", "--steps", "20"]  # the same arguments reach every rank


@pytest.mark.parametrize("gpus", [1, 2])
def test_gpus_flag_starts_that_many_ranks(gpus):
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(gpus), "--check-launch"],
                       capture_output=True, text=True, env=_env(), timeout=240, cwd=REPO)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout  # one line, from rank 0 only
    assert lines[0]["n_gpus"] == gpus and lines[0]["ranks"] == list(range(gpus))
    assert lines[0]["backend"] == ("none" if gpus == 1 else "gloo")


def test_world_mismatch_exits_nonzero():
    """torchrun with 2 ranks but --gpus 3: every rank refuses (the driver would otherwise record a
    2-GPU number under n_gpus 3, or a 1-GPU number under 8)."""
    import bench
    cmd = bench.launch_command(["--gpus", "3", "--check-launch"], 2, 29000 + os.getpid() % 2000)
    r = subprocess.run(cmd, capture_output=True, text=True, env=_env(), timeout=240, cwd=REPO)
    assert r.returncode != 0
    assert "world size 2 != --gpus 3" in (r.stderr + r.stdout)
    assert not _json_lines(r.stdout)

"""bench.py's multi-rank launch: ``--gpus N`` starts N ranks itself, every rank joins one
process group of exactly N ranks, and asking for more GPUs than are visible fails instead of running a
mislabelled single-rank job."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, **env):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env)
    return subprocess.run([sys.executable, BENCH] + args, env=e, capture_output=True, text=True, timeout=300)


@pytest.mark.parametrize("n", [2, 3])
def test_gpus_n_spawns_n_ranks(n):
    r = _run(["--gpus", str(n), "--world-check"], LRL_DIST_BACKEND="gloo")
    assert r.returncode == 0, r.stderr
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(line) == 1, r.stdout  # rank 0 alone prints
    out = json.loads(line[0])
    assert out["world_size"] == n and out["ranks"] == list(range(n)) and out["parallelism"] == f"dp{n}"


def test_more_gpus_than_visible_fails():
    import torch
    n = torch.cuda.device_count() + 1
    r = _run(["--gpus", str(n), "--world-check"], LRL_DIST_BACKEND="nccl")
    assert r.returncode != 0
    assert "GPU(s) visible" in r.stderr


def test_world_size_mismatch_fails():
    r = _run(["--gpus", "2", "--world-check"], LRL_DIST_BACKEND="gloo", WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    assert r.returncode != 0 and "WORLD_SIZE=1" in r.stderr

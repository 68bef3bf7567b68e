"""bench.py's launch contract (VERDICT r1 'next round' item 1): `--gpus N`
without a launcher starts N ranks itself, the parent never touches a GPU, a
WORLD_SIZE that disagrees with --gpus is an error, and the JSON carries the
rank count and whether the run was a rehearsal.  Exercised on CPU (gloo)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra=None, timeout=240):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT",
              "HIPDSML_BENCH_CHILD"):
        env.pop(k, None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True,
                          timeout=timeout, env=env, cwd=ROOT)


def _json(stdout):
    lines = [ln for ln in stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, stdout  # rank 0 prints exactly one line
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [2, 4])
def test_gpus_n_spawns_n_ranks(n):
    p = _run(["--gpus", str(n), "--cpu-dry-run", "--steps", "3", "--warmup", "1",
              "--samples-per-rank", "256"])
    assert p.returncode == 0, p.stderr[-2000:]
    out = _json(p.stdout)
    assert out["n_gpus"] == n and out["world_size"] == n
    assert out["config"]["parallelism"] == f"dp{n}"
    assert out["config"]["global_batch"] == 64 * n
    assert out["rehearsal"] is True and out["device"] == "cpu"
    assert out["physical_gpus"] == 0
    assert out["steps"] == 3 and out["warmup"] == 1 and out["value"] > 0
    assert out["replicas_identical"] is True


def test_diverged_replica_fails_the_run():
    """A replica whose parameters drift off (fault injection after the timed
    steps) must make the run exit non-zero with replicas_identical: false."""
    p = _run(["--gpus", "2", "--cpu-dry-run", "--steps", "2", "--warmup", "1",
              "--samples-per-rank", "256", "--inject-divergence", "1"])
    assert p.returncode != 0, p.stderr[-2000:]  # ranks exit 3; torchrun reports 1
    assert _json(p.stdout)["replicas_identical"] is False
    assert "exitcode  : 3" in p.stderr
    assert "replicas diverged" in p.stderr


def test_single_rank_runs_in_process():
    p = _run(["--gpus", "1", "--cpu-dry-run", "--steps", "2", "--warmup", "1",
              "--samples-per-rank", "128"])
    assert p.returncode == 0, p.stderr[-2000:]
    out = _json(p.stdout)
    assert out["n_gpus"] == 1 and out["config"]["parallelism"] == "dp1"


def test_world_size_mismatch_fails_loudly():
    p = _run(["--gpus", "4", "--cpu-dry-run", "--steps", "2", "--warmup", "0"],
             env_extra={"WORLD_SIZE": "2", "RANK": "0"})
    assert p.returncode != 0
    assert "WORLD_SIZE=2" in p.stderr


@pytest.mark.skipif(os.environ.get("HIP_VISIBLE_DEVICES") is not None, reason="GPUs masked")
def test_more_gpus_than_visible_fails_loudly():
    import torch

    if torch.cuda.device_count() >= 64:
        pytest.skip("host has 64+ GPUs")
    p = _run(["--gpus", "64", "--steps", "2", "--warmup", "0"])
    assert p.returncode == 2
    assert "visible GPUs" in p.stderr
    assert not p.stdout.strip().startswith("{")

"""Init phase timing and the total budget of the optional init / probe phases
(utils/initbudget.py, VERDICT r5 Next #6): phases are timed, optional phases
stop once the budget is spent and are listed as skipped, and the decision is
collective (the slowest rank's elapsed time) so every rank takes the same
branch."""
import json
import os
import subprocess
import sys

from spawn_util import spawn_group

from hipdsml.utils.initbudget import InitPhases

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class Clock:
    t = 0.0

    def __call__(self):
        return self.t


def test_phases_accumulate_and_budget_skips():
    clock = Clock()
    ph = InitPhases(budget_s=10.0, clock=clock)
    with ph.phase("a"):
        clock.t += 2.0
    with ph.phase("a"):
        clock.t += 1.0
    assert ph.allow("probe1")
    clock.t += 8.0
    assert not ph.allow("probe2")
    assert not ph.allow("probe3")
    rep = ph.report()
    assert rep["phases_s"] == {"a": 3.0}
    assert rep["skipped"] == ["probe2", "probe3"]
    assert rep["total_s"] == 11.0 and rep["budget_s"] == 10.0


def test_budget_from_env(monkeypatch):
    monkeypatch.setenv("HIPDSML_INIT_BUDGET_S", "12.5")
    assert InitPhases().budget_s == 12.5


def _worker(rank, world, port, outdir):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from hipdsml.parallel.dist import DistContext

    ctx = DistContext.from_env(device="cpu", watchdog_s=0)
    clock = Clock()
    ph = InitPhases(ctx, budget_s=5.0, clock=clock)
    # rank 1 is slow: its elapsed time decides for everyone
    clock.t = 6.0 if rank == 1 else 1.0
    res = ph.allow("x")
    with open(os.path.join(outdir, f"r{rank}.json"), "w") as f:
        json.dump({"allow": res, "skipped": ph.skipped}, f)
    ctx.destroy()


def test_allow_is_collective(tmp_path):
    spawn_group(_worker, 3, lambda port: (3, port, str(tmp_path)))
    outs = [json.loads((tmp_path / f"r{r}.json").read_text()) for r in range(3)]
    assert all(o == {"allow": False, "skipped": ["x"]} for o in outs)


def test_cpu_dry_run_reports_phases_and_budget_skips():
    """bench.py --cpu-dry-run --gpus 2 with a zero budget: the timed steps and
    the replica check still run, every optional probe is skipped and listed."""
    env = dict(os.environ, HIPDSML_INIT_BUDGET_S="0", OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--cpu-dry-run", "--gpus", "2",
                        "--steps", "3", "--warmup", "1", "--samples-per-rank", "640"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1]
    out = json.loads(line)
    rep = out["init_phases_s"]
    assert out["replicas_identical"] is True and out["n_gpus"] == 2
    assert {"dist_init", "data_gen", "trainer_build", "warmup_capture"} <= set(rep["phases_s"])
    assert rep["budget_s"] == 0.0

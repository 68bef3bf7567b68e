"""Chunk tuning of the in-house multi-ring all-reduce (parallel/ring_tune.py):
the selection logic against a fake communicator whose calls advance a fake
clock by a latency + bandwidth cost model of the ring schedule, and the
candidate pruning against the schedule's own rounds (ring_plan.h)."""
import pytest

from hipdsml.parallel import ring_tune as rt


class FakeComm:
    """ring_allreduce_ costs (2(n-1) steps) x rounds x (alpha + beta x bytes per round)."""

    def __init__(self, clock, n, rings, alpha_us, gbps):
        self.clock, self.n, self.rings = clock, n, rings
        self.alpha, self.gbps = alpha_us, gbps
        self.calls = []

    def cost_us(self, nbytes, chunk):
        r = rt.effective_rounds(nbytes, self.n, self.rings, chunk)
        per_round = min(chunk, -(-nbytes // (self.rings * self.n)))
        return 2 * (self.n - 1) * r * (self.alpha + per_round / (self.gbps * 1e3))

    def ring_allreduce_(self, nbytes, chunk):
        self.calls.append(chunk)
        self.clock.t += self.cost_us(nbytes, chunk) * 1e-6


class Clock:
    t = 0.0

    def __call__(self):
        return self.t


@pytest.mark.parametrize("nbytes,alpha,gbps", [(437_544, 8.0, 50.0), (1 << 20, 2.0, 5.0),
                                               (80 << 20, 8.0, 50.0), (80 << 20, 0.5, 400.0)])
def test_sweep_picks_the_cost_models_fastest_chunk(nbytes, alpha, gbps):
    clock = Clock()
    comm = FakeComm(clock, n=8, rings=6, alpha_us=alpha, gbps=gbps)
    cands = rt.distinct_chunks(nbytes, 8, 6)
    times = rt.sweep(lambda c: comm.ring_allreduce_(nbytes, c), lambda: None, cands, iters=5,
                     warmup=1, clock=clock)
    best = rt.pick_chunk(times)
    model = {c: comm.cost_us(nbytes, c) for c in cands}
    fastest = min(model.values())
    assert model[best] <= fastest * 1.02
    assert set(comm.calls) == set(cands)


def test_distinct_chunks_drop_chunks_past_the_segment():
    # 437,544 B over 6 rings x 8 ranks: ~9.1 KB segments -> every chunk >= that is one round
    cands = rt.distinct_chunks(437_544, 8, 6)
    assert cands == [64 << 10]
    big = rt.distinct_chunks(80 << 20, 8, 6)
    assert big == sorted(big) and len(big) == len(set(rt.effective_rounds(80 << 20, 8, 6, c)
                                                       for c in big))
    assert len(big) >= 5


def test_pick_prefers_larger_chunk_within_tolerance():
    assert rt.pick_chunk({65536: 100.0, 131072: 101.0, 262144: 150.0}) == 131072
    assert rt.pick_chunk({65536: 100.0, 131072: 110.0}) == 65536
    with pytest.raises(ValueError):
        rt.pick_chunk({})


def test_rounds_match_the_native_schedule():
    """effective_rounds mirrors ring_plan.h: the native schedule has
    2(n-1) x rounds groups (built without a GPU)."""
    C = pytest.importorskip("hipdsml.ops.native").require_native()
    for nbytes, chunk in ((437_544, 16384), (1 << 20, 4096), (80 << 20, 1 << 20)):
        count = nbytes // 4
        plan = C.ring_schedule(8, 3, count, 4, chunk // 4, 0)
        assert len(plan) == 2 * 7 * rt.effective_rounds(nbytes, 8, 6, chunk)


def test_choose_schedule_prefers_single_stream_unless_pipelined_clearly_wins():
    plain = {65536: 100.0, 131072: 101.0, 262144: 150.0}
    assert rt.choose_schedule(plain, None) == (131072, False)
    assert rt.choose_schedule(plain, {65536: 99.5}) == (131072, False)   # within tolerance
    assert rt.choose_schedule(plain, {65536: 80.0, 131072: 90.0}) == (65536, True)


def test_validate_pipelined_reports_a_hang_as_an_error_and_aborts():
    """VERDICT r4 Next #7: a pipelined candidate that never completes is
    reported (ring_pipe_error), its throwaway communicator aborted -- the
    tuner itself never hangs."""
    clock = Clock()
    aborted = []

    def sleep(dt):
        clock.t += dt

    err = rt.validate_pipelined(lambda: None, lambda: False, lambda ok: ok, lambda: aborted.append(1),
                                timeout_s=2.0, clock=clock, sleep=sleep)
    assert "did not complete" in err and aborted == [1]


def test_validate_pipelined_agrees_across_ranks():
    # this rank finished, a peer did not: the failure is agreed and reported here too
    aborted = []
    err = rt.validate_pipelined(lambda: None, lambda: True, lambda ok: False, lambda: aborted.append(1))
    assert err == "pipelined ring failed on a peer" and aborted == [1]
    assert rt.validate_pipelined(lambda: None, lambda: True, lambda ok: ok, lambda: None) == ""

    def boom():
        raise RuntimeError("ncclGroupEnd: unhandled error")

    assert "ncclGroupEnd" in rt.validate_pipelined(boom, lambda: True, lambda ok: ok, lambda: None)


def test_validate_pipelined_aborts_before_agreeing_on_a_local_timeout():
    """a rank whose probe timed out must abort it BEFORE
    the agreement -- an agreement that needed the GPU would queue behind the
    hung ring.  The order of the two calls is the contract."""
    clock = Clock()
    order = []

    def sleep(dt):
        clock.t += dt

    def agree(ok):
        order.append(("agree", ok))
        return ok

    err = rt.validate_pipelined(lambda: None, lambda: False, agree, lambda: order.append(("abort",)),
                                timeout_s=1.0, clock=clock, sleep=sleep)
    assert "did not complete" in err
    assert order == [("abort",), ("agree", False)]


def test_pipelined_schedule_is_opt_in(monkeypatch):
    monkeypatch.delenv("HIPDSML_RING_PIPELINE", raising=False)
    assert rt.pipeline_default() is False
    monkeypatch.setenv("HIPDSML_RING_PIPELINE", "1")
    assert rt.pipeline_default() is True


def test_watchdog_unwatch_comm():
    from hipdsml.parallel.watchdog import Watchdog

    class C:
        aborted = 0

        def async_error(self):
            return ""

        def abort(self):
            self.aborted += 1

    wd = Watchdog(timeout=60, interval=0.01, exit_on_stuck=False)
    a, b = C(), C()
    wd.watch_comm(a)
    wd.watch_comm(b)
    wd.unwatch_comm(b)
    wd.declare("test fault")
    wd.stop()
    assert a.aborted == 1 and b.aborted == 0


def _agree_worker(rank, world, port, votes, outdir):
    import os

    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from hipdsml.parallel.dist import DistContext

    ctx = DistContext.from_env(device="cpu", watchdog_s=0)
    res = [ctx.host_agree("t", v[rank]) for v in votes]
    with open(os.path.join(outdir, f"r{rank}.txt"), "w") as f:
        f.write(",".join("1" if r else "0" for r in res))
    ctx.destroy()


def test_host_agree_is_a_store_only_and(tmp_path):
    """The probe's agreement runs on the TCP store (no device tensor): an AND
    over ranks, repeated calls independent."""
    from spawn_util import spawn_group

    votes = [(True, True, True), (True, False, True), (False, False, False), (True, True, True)]
    spawn_group(_agree_worker, 3, lambda port: (3, port, votes, str(tmp_path)))
    got = [(tmp_path / f"r{r}.txt").read_text() for r in range(3)]
    assert got == ["1,0,0,1"] * 3

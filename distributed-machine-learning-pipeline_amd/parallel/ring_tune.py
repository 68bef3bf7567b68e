"""Chunk-size tuning of the in-house multi-ring all-reduce (csrc/runtime/ring_plan.h,
``RcclComm::ring_allreduce``) for the job's actual buffer and topology.

The reference's ring moves one segment per step with no chunking at all
(``gpu_coordinator_server.go:338-356``); its comparison test times one 1 MiB
call (``allreduce_comparison_test.go:116-129``).  Here every ring step is an
ncclGroup of send/recv pairs (one per directed ring) followed by one reduce
launch, and a segment larger than the chunk is split into several such
rounds.  Small chunks pipeline nothing (the rounds run back to back on one
stream) but bound the scratch; large chunks mean fewer groups and launches.
Which wins depends on the xGMI link latency vs. bandwidth at this message
size, so the chunk is measured at init, not guessed: every candidate is timed
on every rank (max over ranks: the slowest rank sets the pace of a
collective) and the fastest kept.
"""
from __future__ import annotations

import time
from typing import Callable, Dict, Iterable, Optional, Sequence

CHUNKS: Sequence[int] = (64 << 10, 128 << 10, 256 << 10, 512 << 10, 1 << 20, 2 << 20, 4 << 20)


def effective_rounds(nbytes: int, world: int, rings: int, chunk: int, align: int = 16) -> int:
    """Chunk rounds per ring step (ring_plan.h ring_schedule): the buffer is
    sliced over `rings` rings, each slice over `world` segments."""
    up = lambda x, m: (x + m - 1) // m * m  # noqa: E731
    sl = up(-(-nbytes // rings), align)
    seg = up(-(-sl // world), align)
    c = max(align, chunk // align * align)
    return max(1, -(-seg // c))


def distinct_chunks(nbytes: int, world: int, rings: int, chunks: Iterable[int] = CHUNKS) -> list:
    """The candidates that differ in their schedule: chunks beyond the segment
    size all give one round per step, so only the smallest of those is kept."""
    out, seen = [], set()
    for c in sorted(chunks):
        r = effective_rounds(nbytes, world, rings, c)
        if r not in seen:
            seen.add(r)
            out.append(c)
    return out


def pick_chunk(times_us: Dict[int, float], tol: float = 0.02) -> int:
    """Fastest chunk; within `tol` of the fastest, the LARGER chunk wins (fewer
    groups and launches, the same speed)."""
    if not times_us:
        raise ValueError("no chunk timings")
    best = min(times_us.values())
    return max(c for c, t in times_us.items() if t <= best * (1.0 + tol))


def sweep(run: Callable[[int], None], sync: Callable[[], None], chunks: Iterable[int],
          iters: int = 20, warmup: int = 3, reduce_max: Optional[Callable[[float], float]] = None,
          clock: Callable[[], float] = time.perf_counter,
          reserve: Optional[Callable[[int], None]] = None) -> Dict[int, float]:
    """µs per call of `run(chunk)` for every chunk (collective when
    `reduce_max` agrees the time over ranks).  `sync` waits for the device
    work of the calls."""
    out: Dict[int, float] = {}
    for c in chunks:
        if reserve is not None:
            reserve(c)  # ring scratch sized outside the timed loop
        for _ in range(warmup):
            run(c)
        sync()
        t0 = clock()
        for _ in range(iters):
            run(c)
        sync()
        dt = (clock() - t0) / iters
        if reduce_max is not None:
            dt = reduce_max(dt)
        out[int(c)] = round(1e6 * dt, 2)
    return out


def choose_schedule(plain_us: Dict[int, float], pipe_us: Optional[Dict[int, float]],
                    tol: float = 0.02) -> tuple:
    """(chunk, pipelined) of the fastest candidate over both schedules.  The
    pipelined schedule must beat the best single-stream time by more than
    `tol` to be chosen (it costs events and a second stream); within the
    single-stream sweep pick_chunk's larger-chunk rule applies."""
    best = pick_chunk(plain_us)
    if pipe_us:
        pc = min(pipe_us, key=pipe_us.get)
        if pipe_us[pc] < plain_us[best] * (1.0 - tol):
            return pc, True
    return best, False


def validate_pipelined(run: Callable[[], None], done: Callable[[], bool], agree: Callable[[bool], bool],
                       abort: Callable[[], None], timeout_s: float = 10.0,
                       clock: Callable[[], float] = time.monotonic,
                       sleep: Callable[[float], None] = time.sleep) -> str:
    """Run the pipelined ring ONCE with a bounded wait (collective): `run`
    enqueues it, `done` polls its completion, `agree` ANDs a flag over the
    ranks, `abort` kills the communicator it ran on (a throwaway one: a hang
    never reaches the job's communicator).  Returns '' or the error, agreed
    on every rank -- a timeout or an exception is reported, never a hang.

    A rank that timed out aborts its probe BEFORE it takes part in the
    agreement, and `agree` must be host-only (parallel/dist.py host_agree):
    an agreement that needed this rank's GPU would queue behind the hung
    ring and never return."""
    err = ""
    try:
        run()
        t_end = clock() + timeout_s
        while not done():
            if clock() > t_end:
                err = f"pipelined ring did not complete within {timeout_s:g} s"
                break
            sleep(0.001)
    except Exception as e:  # noqa: BLE001
        err = f"{type(e).__name__}: {e}"[:200]
    aborted = False
    if err:
        aborted = True
        _quiet(abort)
    ok = agree(not err)
    if not ok:
        if not aborted:
            _quiet(abort)  # a peer failed: its half of the ring never completes
        return err or "pipelined ring failed on a peer"
    return ""


def _quiet(fn: Callable[[], None]) -> None:
    try:
        fn()
    except Exception:  # noqa: BLE001 pragma: no cover
        pass


def pipeline_default() -> bool:
    """Whether the tuner times the pipelined ring schedule at all: off unless
    HIPDSML_RING_PIPELINE=1, until a multi-GPU run has recorded a pipelined
    sweep (``sweep_pipelined_us``) -- one-GPU boxes cannot run RCCL at
    nranks > 1, so the schedule is validated only by the FIFO simulation in
    tests/test_ring_plan.py so far."""
    import os

    return os.environ.get("HIPDSML_RING_PIPELINE", "0") == "1"


def tune_ring_chunk(ctx, comm, t, chunks: Iterable[int] = CHUNKS, iters: int = 20,
                    max_rings: int = 0, pipeline: Optional[bool] = None,
                    probe_timeout_s: float = 10.0) -> Dict[str, object]:
    """Collective: sweep the chunk of ``comm.ring_allreduce_`` on tensor `t`
    (restored afterwards) over the distinct candidates, for the single-stream
    schedule and -- when some candidate has several chunk rounds per step --
    the pipelined one (chunk c's reduce overlapping chunk c+1's transfer,
    ring_plan.h ring_pipeline).  The pipelined schedule first runs once on a
    throwaway communicator under a bounded wait, and must reproduce the
    single-stream result bit for bit (the same additions in the same order);
    a failure there is reported as ``ring_pipe_error``, never as a hang.  The
    faster schedule becomes the communicator's default.  Returns
    ``{"best": bytes, "pipelined": bool, "sweep_us": {bytes: us},
    "sweep_pipelined_us": {bytes: us} | None[, "ring_pipe_error": str]}``."""
    import torch

    if pipeline is None:
        pipeline = pipeline_default()
    nbytes = t.numel() * t.element_size()
    rings = len(_directed_rings(ctx.world_size, max_rings))
    cands = distinct_chunks(nbytes, ctx.world_size, rings, chunks)
    saved = t.clone()

    def sync():
        torch.cuda.synchronize(t.device)

    reduce_max = lambda v: ctx.all_reduce_scalars(v, op="max")[0]  # noqa: E731
    reserve = lambda c: comm.reserve_ring(t.numel(), c, max_rings)  # noqa: E731
    with ctx.guard("ring chunk sweep"):
        times = sweep(lambda c: comm.ring_allreduce_(t, 0, c, max_rings, 0), sync, cands, iters=iters,
                      reduce_max=reduce_max, reserve=reserve)
    out: Dict[str, object] = {"sweep_us": {str(k): v for k, v in times.items()}, "sweep_pipelined_us": None}
    multi = [c for c in cands if effective_rounds(nbytes, ctx.world_size, rings, c) > 1]
    pipe_times = None
    if pipeline and multi:
        err = _probe_pipelined(ctx, t, saved, multi[0], max_rings, probe_timeout_s)
        if err:
            out["ring_pipe_error"] = err
        else:
            with ctx.guard("pipelined ring chunk sweep"):
                pipe_times = sweep(lambda c: comm.ring_allreduce_(t, 0, c, max_rings, 1), sync, multi,
                                   iters=iters, reduce_max=reduce_max, reserve=reserve)
            out["sweep_pipelined_us"] = {str(k): v for k, v in pipe_times.items()}
    t.copy_(saved)
    best, piped = choose_schedule(times, pipe_times)
    comm.set_ring_pipeline(1 if piped else 0)
    comm.reserve_ring(t.numel(), best, max_rings)
    out["best"] = best
    out["pipelined"] = piped
    return out


def _probe_pipelined(ctx, t, src, chunk: int, max_rings: int, timeout_s: float) -> str:
    """The pipelined ring once, on a throwaway RCCL communicator and its own
    stream, bounded, and checked bit-exact against the single-stream ring on
    the same input.  The probe is never registered with the watchdog and is
    destroyed on every path (it used to stay alive, polled, next to
    the job's communicator); every agreement goes through the TCP store, so a
    hung probe cannot block it."""
    import torch

    from .dist import make_native_comm

    try:
        probe = make_native_comm(ctx, watch=False)
    except Exception as e:  # noqa: BLE001 -- collective init failed: no pipelined candidate
        return f"probe communicator: {type(e).__name__}: {e}"[:200]
    side = torch.cuda.Stream(device=t.device)
    side.wait_stream(torch.cuda.current_stream(t.device))
    want = src.clone()
    got = src.clone()
    ev = torch.cuda.Event()
    agree = lambda ok: ctx.host_agree("ring_pipe_probe", ok)  # noqa: E731
    try:
        with torch.cuda.stream(side):
            probe.reserve_ring(t.numel(), chunk, max_rings)
            probe.ring_allreduce_(want, 0, chunk, max_rings, 0)
            ev.record()
        poll = ev.query
        # the single-stream reference ring, bounded the same way
        err = validate_pipelined(lambda: None, poll, agree, probe.abort, timeout_s)
        if err:
            return "single-stream probe: " + err

        def run():
            with torch.cuda.stream(side):
                probe.ring_allreduce_(got, 0, chunk, max_rings, 1)
                ev.record()

        err = validate_pipelined(run, poll, agree, probe.abort, timeout_s)
        if err:
            return err
        side.synchronize()  # both rings completed on every rank
        if not agree(bool(torch.equal(want, got))):
            return "pipelined ring result differs from the single-stream ring"
        return ""
    finally:
        _quiet(probe.destroy)
        del probe


def _directed_rings(n: int, max_rings: int):
    from ..ops.native import require_native

    return require_native().directed_rings(n, max_rings)

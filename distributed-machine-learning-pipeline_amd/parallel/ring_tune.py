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


def tune_ring_chunk(ctx, comm, t, chunks: Iterable[int] = CHUNKS, iters: int = 20,
                    max_rings: int = 0) -> Dict[str, object]:
    """Collective: sweep the chunk of ``comm.ring_allreduce_`` on tensor `t`
    (restored afterwards) over the distinct candidates; returns
    ``{"best": bytes, "sweep_us": {bytes: us}}``."""
    import torch

    nbytes = t.numel() * t.element_size()
    rings = len(_directed_rings(ctx.world_size, max_rings))
    cands = distinct_chunks(nbytes, ctx.world_size, rings, chunks)
    saved = t.clone()

    def run(c):
        comm.ring_allreduce_(t, 0, c, max_rings)

    def sync():
        torch.cuda.synchronize(t.device)

    times = sweep(run, sync, cands, iters=iters,
                  reduce_max=lambda v: ctx.all_reduce_scalars(v, op="max")[0],
                  reserve=lambda c: comm.reserve_ring(t.numel(), c, max_rings))
    t.copy_(saved)
    best = pick_chunk(times)
    comm.reserve_ring(t.numel(), best, max_rings)
    return {"best": best, "sweep_us": {str(k): v for k, v in times.items()}}


def _directed_rings(n: int, max_rings: int):
    from ..ops.native import require_native

    return require_native().directed_rings(n, max_rings)

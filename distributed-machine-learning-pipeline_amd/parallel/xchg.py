"""xGMI peer exchange: the gradient all-reduce fused into the weight-gradient
kernel (``csrc/kernels/mlp_f32.hip`` XCHG path, ``csrc/runtime/peer_exchange.cpp``).

Why: the flagship gradient is 437 KB.  At that size an all-reduce is pure
latency — a ring (the reference's algorithm, ``gpu_coordinator_server.go:338-356``,
or RCCL's) pays 2(N-1) hops, plus a kernel boundary before and after.  On an
MI355X node every GPU has a direct xGMI link to every other, so each replica
can instead read all peers' gradient tiles directly (one-shot) inside the
kernel that produced its own, sum them in rank order and apply SGD — no
collective launch, no extra kernel, and the step stays hipGraph-capturable.

Bootstrap (collective over the process group): every rank allocates an
uncached exchange buffer, publishes its IPC handle through the TCP store,
opens the peers' handles, zeroes its flags, then all ranks barrier.
"""
from __future__ import annotations

import logging
from typing import List, Optional

import torch

from ..models.mlp import MlpLayout
from .dist import DistContext

log = logging.getLogger("hipdsml.xchg")

_key = 0


def wgrad_tiles(layout: MlpLayout) -> int:
    d = layout.spec.dims
    return sum(((d[l + 1] + 15) // 16) * ((d[l] + 31) // 32) for l in range(len(d) - 1))


class ExchangeUnavailable(RuntimeError):
    pass


def make_peer_exchange(ctx: DistContext, layout: MlpLayout, timeout_ms: float = 10000.0):
    """Exchange sized for the fused MLP step (one flag per weight-gradient tile)."""
    return make_exchange(ctx, layout.nparams, wgrad_tiles(layout), timeout_ms)


def act_payload(layout: MlpLayout) -> int:
    """Floats of one replica's pushed image (H_l, dZ_l in MFMA fragment order)."""
    from ..ops.native import require_native

    return require_native().mlp_xact_payload(layout.desc_list())


def act_supported(layout: MlpLayout) -> bool:
    d = layout.spec.dims
    return layout.batch <= 64 and all(x % 16 == 0 for x in d[:-1])


def swizzle_inputs(X: torch.Tensor, batch: int) -> torch.Tensor:
    """Input shards [N, rows, >= K] -> MFMA fragment order for the activation
    exchange (kernels/mlp_f32_xact.hip): per batch b and 16-column strip t,
    ``[w][lane = 16q + i][j] = X[b*batch + 4w + 16j + q][16t + i]`` with rows
    past the batch zero-padded to 64.  Returns [N, nbatches, K/16, 4, 64, 4]."""
    N, rows, _ = X.shape
    nb = rows // batch
    K = X.shape[2]
    if K % 16 or batch > 64:
        raise ValueError("fragment order needs K % 16 == 0 and batch <= 64")
    x = X[:, : nb * batch].reshape(N, nb, batch, K)
    if batch < 64:
        x = torch.nn.functional.pad(x, (0, 0, 0, 64 - batch))
    x = x.reshape(N, nb, 4, 4, 4, K // 16, 16)        # [N, nb, j, w, q, t, i]
    x = x.permute(0, 1, 5, 3, 4, 6, 2).contiguous()   # [N, nb, t, w, q, i, j]
    return x.reshape(N, nb, K // 16, 4, 64, 4)


def make_act_exchange(ctx: DistContext, layout: MlpLayout, timeout_ms: float = 10000.0):
    """Receive buffers for the activation exchange (kernels/mlp_f32_xact.hip):
    per parity one slot of ``act_payload`` floats per source rank, and one
    flag per (source rank, 16-column strip)."""
    n = ctx.world_size
    p = act_payload(layout)
    return make_exchange(ctx, n * p, n * (p // 1024), timeout_ms)


def make_local_act_group(layout: MlpLayout, devices: List[int], timeout_ms: float = 10000.0):
    """Activation-exchange buffers for N replicas living in one process."""
    n = len(devices)
    p = act_payload(layout)
    return make_local_group(None, devices, timeout_ms, half_floats=n * p, ntiles=n * (p // 1024))


def make_exchange(ctx: DistContext, half_floats: int, ntiles: int, timeout_ms: float = 10000.0):
    """Collective: returns a connected ``_C.PeerExchange`` for this rank, or
    raises :class:`ExchangeUnavailable` on EVERY rank if any rank failed (the
    outcome is agreed before anyone leaves, so no rank is left in a collective)."""
    from ..ops.native import require_native

    global _key
    C = require_native()
    x, err, h = None, "", b""
    if ctx.world_size > 8:
        err = "the xGMI exchange spans one node (<= 8 GPUs)"
    else:
        try:
            x = C.PeerExchange(ctx.device.index, half_floats, ntiles)
            if x.memory_kind != "uncached":
                # the fence-free release/acquire of every exchange protocol
                # relies on uncached (MTYPE UC) memory (kernels/common.h)
                raise RuntimeError(f"exchange memory is {x.memory_kind}, not uncached")
            x.set_timeout_ms(timeout_ms)
            h = x.ipc_handle()
        except Exception as e:  # noqa: BLE001
            err = f"allocation/export: {e}"
    _key += 1
    handles = ctx.all_gather_bytes(f"hipdsml/xchg/{_key}", h)  # every rank publishes
    if not err and any(len(hh) == 0 for hh in handles):
        err = "a peer could not allocate its exchange buffer"
    if not err:
        try:
            x.connect_ipc(ctx.rank, handles)
            x.reset()
            torch.cuda.synchronize(ctx.device)
        except Exception as e:  # noqa: BLE001
            err = f"connect: {e}"
    ok = ctx.all_reduce_scalars(0.0 if err else 1.0, op="min")[0]
    if not ok:
        raise ExchangeUnavailable(err or "failed on a peer")
    log.info("peer exchange: rank %d/%d, %s memory, %d tiles", ctx.rank, ctx.world_size,
             x.memory_kind, x.ntiles)
    return x


_REPLICA_STREAMS: dict = {}


def replica_streams(device: torch.device, n: int) -> List[torch.cuda.ExternalStream]:
    """`n` streams for in-process replicas that spin on each other, each on a
    hardware queue of its own (``_C.dedicated_stream``: a full CU mask makes
    HIP create a fresh queue instead of handing out the least-used of its
    GPU_MAX_HW_QUEUES).  Two replicas on one queue would serialise — a kernel
    queued behind a peer that spins for it never starts.  Created once per
    process and reused (at most 8).

    These are BLOCKING streams (the CU-mask constructor takes no flags): drive
    the replicas while torch's current stream is a non-null stream, since the
    runners join torch's current stream and an event recorded on the legacy
    null stream waits for every blocking stream — including a spinning peer."""
    from ..ops.native import require_native

    if n > 8:
        raise ValueError("at most 8 in-process replicas")
    C = require_native()
    key = (device.type, device.index)
    pool = _REPLICA_STREAMS.setdefault(key, [])
    while len(pool) < n:
        pool.append(torch.cuda.ExternalStream(C.dedicated_stream(device.index), device=device))
    return pool[:n]


def make_local_group(layout: Optional[MlpLayout], devices: List[int], timeout_ms: float = 10000.0,
                     half_floats: int = 0, ntiles: int = 0):
    """Exchanges for N replicas living in ONE process (tests / single-process
    multi-GPU): peers are referenced directly instead of through IPC."""
    from ..ops.native import require_native

    C = require_native()
    if layout is not None:
        half_floats, ntiles = layout.nparams, wgrad_tiles(layout)
    xs = [C.PeerExchange(dev, half_floats, ntiles) for dev in devices]
    for r, x in enumerate(xs):
        x.set_timeout_ms(timeout_ms)
        x.connect_local(r, xs)
    return xs


class XgmiAllReduce:
    """fp32 sum all-reduce over xGMI peer memory for buffers of up to
    `max_floats` (kernels/xchg.hip): ``algo="oneshot"`` (every rank reads every
    peer's whole buffer: one synchronisation, n bytes per link) or
    ``"twoshot"`` (reduce-scatter + all-gather: two synchronisations, 2n/N
    bytes per link).  Collective construction; calls must be issued by every
    rank in the same order (like any collective)."""

    ALGOS = {"oneshot": 0, "twoshot": 1}

    def __init__(self, ctx: DistContext, max_floats: int, max_blocks: int = 512,
                 timeout_ms: float = 10000.0, algo: str = "oneshot"):
        if algo not in self.ALGOS:
            raise ValueError(f"algo must be one of {sorted(self.ALGOS)}")
        self.ctx = ctx
        self.algo = algo
        self.max_floats = (max_floats + 3) // 4 * 4
        # the two-shot form also holds the reduced chunk: n + ceil(n / N) per parity half
        self.x = make_exchange(ctx, 2 * self.max_floats, max_blocks, timeout_ms)

    def __call__(self, t: torch.Tensor) -> torch.Tensor:
        n = t.numel()
        if n % 4 == 0 and n <= self.max_floats and t.is_contiguous():
            return self.x.allreduce_(t, self.ALGOS[self.algo])
        raise ValueError(f"xGMI all-reduce takes contiguous fp32 of <= {self.max_floats} "
                         "elements, a multiple of 4")

    def check(self) -> None:
        check(self.x)


def reset_group(ctx: DistContext, x) -> None:
    """Collective flag reset (after a resume or a self-test rewound the step
    counter): nobody may still be reading when the flags go back to zero."""
    torch.cuda.synchronize(ctx.device)
    ctx.barrier()
    x.reset()
    torch.cuda.synchronize(ctx.device)
    ctx.barrier()


def check(x, where: str = "") -> None:
    if x is not None and x.error():
        raise RuntimeError(f"xGMI peer exchange timed out waiting for a peer{where}: "
                           "a replica stopped or fell behind")


def verify_against_allreduce(trainer, steps: int = 3) -> float:
    """`steps` optimizer steps through the active exchange vs. the same steps
    with fp32 torch gradients summed by a torch.distributed all-reduce; the
    trainer state is restored afterwards.  Returns the max abs parameter
    difference over all ranks (inf if replicas disagree bit-wise, a peer timed
    out or a persistent hand-off gave up).  Every rank runs the same
    collectives whatever happens locally.

    The exchange runs the steps as TWO launches (1, then steps - 1): for the
    persistent step (sync='pk') that covers a launch split (the step counter
    and hand-off tags carried over between launches), and with >= 3 steps the
    parity halves of every receive buffer are reused (step s and s + 2 share
    one), so a stale slot or flag from two steps back would show up here."""
    import torch.distributed as dist

    from ..models.mlp import grads_ref

    ctx = trainer.ctx
    r = trainer.runner
    lay = trainer.layout
    steps = max(2, int(steps))
    P0, ctr0, st0 = trainer.P.clone(), trainer.ctr.clone(), trainer.stats.clone()
    s0 = int(ctr0[1].item())
    want = P0.clone()
    d0 = lay.spec.dims[0]
    for k in range(steps):
        b = (s0 + k) % trainer.nbatches
        Xb = trainer.X[b * trainer.batch:(b + 1) * trainer.batch, :d0]
        yb = trainer.y[b * trainer.batch:(b + 1) * trainer.batch].long()
        g = grads_ref(lay, want, Xb, yb)[0].contiguous()
        dist.all_reduce(g)
        want = want - (trainer.lr / ctx.world_size) * g
    torch.cuda.synchronize(ctx.device)
    r.step(1)
    r.step(steps - 1)
    r.synchronize()
    timed_out = float(trainer.xchg.error() != 0)
    if trainer.pk_buf is not None and r.persist_active() and r.persist_failed():
        timed_out = 1.0  # a hand-off of the persistent step itself gave up
    diff = (trainer.P - want).abs().max().reshape(1)
    ref = trainer.P.clone()
    dist.broadcast(ref, 0)
    mismatch = (trainer.P != ref).any().float().reshape(1)
    stats = torch.cat([diff, mismatch, torch.tensor([timed_out], device=diff.device)])
    dist.all_reduce(stats, op=dist.ReduceOp.MAX)
    trainer.P.copy_(P0)
    trainer.ctr.copy_(ctr0)
    trainer.stats.copy_(st0)
    reset_group(ctx, trainer.xchg)
    d, mm, to = stats.tolist()
    return float("inf") if (mm or to or d != d) else d

"""Process-group context: one process per GPU, ``torch.distributed`` over RCCL
(backend ``"nccl"`` is RCCL on ROCm) or gloo on CPU.

The reference has no process group at all: its "ranks" are positions in the
CommInit address list (``gpu_coordinator_server.go:159``).  Here ranks come from
the torchrun environment (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*), and the
native RCCL communicator (``hipdsml._C.RcclComm``) is bootstrapped by sharing an
``ncclUniqueId`` through the process group's TCP store.
"""
from __future__ import annotations

import contextlib
import datetime
import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist

from .watchdog import Watchdog, timeout_from_env


@dataclass
class DistContext:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    backend: str = "none"
    device: torch.device = torch.device("cpu")
    initialized_here: bool = False
    watchdog: Optional[Watchdog] = None

    @property
    def is_distributed(self) -> bool:
        return self.world_size > 1

    @classmethod
    def from_env(cls, device: str = "auto", backend: Optional[str] = None,
                 timeout_s: Optional[float] = None, device_index: Optional[int] = None,
                 watchdog_s: Optional[float] = None) -> "DistContext":
        """Process group from the torchrun environment.  N > 1 also starts the
        data-plane watchdog (parallel/watchdog.py; HIPDSML_WATCHDOG_S, default
        300 s, 0 disables); HIPDSML_PG_TIMEOUT_S sets the process-group timeout."""
        if timeout_s is None:
            timeout_s = float(os.environ.get("HIPDSML_PG_TIMEOUT_S", "600"))
        world = int(os.environ.get("WORLD_SIZE", "1"))
        rank = int(os.environ.get("RANK", "0"))
        local = int(os.environ.get("LOCAL_RANK", str(rank)))
        if device == "auto":
            use_gpu = torch.cuda.is_available()
        else:
            use_gpu = device.startswith("cuda")
        if use_gpu:
            idx = local if device_index is None else device_index
            torch.cuda.set_device(idx)
            dev = torch.device("cuda", idx)
        else:
            dev = torch.device("cpu")
        ctx = cls(rank=rank, world_size=world, local_rank=local, device=dev)
        if world > 1:
            be = backend or ("nccl" if use_gpu else "gloo")
            if not dist.is_initialized():
                os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
                kw = dict(backend=be, rank=rank, world_size=world,
                          timeout=datetime.timedelta(seconds=timeout_s))
                if use_gpu and be == "nccl":
                    kw["device_id"] = dev
                dist.init_process_group(**kw)
                ctx.initialized_here = True
            ctx.backend = dist.get_backend()
            wd = timeout_from_env() if watchdog_s is None else watchdog_s
            if wd > 0:
                grace = float(os.environ.get("HIPDSML_WATCHDOG_GRACE_S", "10"))
                ctx.watchdog = Watchdog(wd, grace=grace, name=f"[rank {rank}]")
        return ctx

    def guard(self, what: str):
        """Blocking section under the watchdog (no-op without one)."""
        if self.watchdog is None:
            return contextlib.nullcontext()
        return self.watchdog.guard(what)

    # -- collectives on small host/device tensors (outside timed regions) ----
    def all_reduce_(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        if not self.is_distributed:
            return t
        rop = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX,
               "min": dist.ReduceOp.MIN, "prod": dist.ReduceOp.PRODUCT}[op]
        with self.guard("all_reduce"):
            dist.all_reduce(t, op=rop)
            if t.is_cuda:
                torch.cuda.synchronize(t.device)
        return t

    def all_reduce_scalars(self, *vals: float, op: str = "sum") -> list:
        t = torch.tensor(vals, dtype=torch.float64 if self.device.type == "cpu" else torch.float32,
                         device=self.device)
        self.all_reduce_(t, op)
        return [float(v) for v in t.tolist()]

    def host_agree(self, key: str, ok: bool) -> bool:
        """Collective AND of `ok` over the ranks through the TCP store only: no
        device tensor, no stream, no synchronize -- so it cannot queue behind
        a hung kernel on this rank's GPU (the agreement after a bounded wait
        must not block on the very work it bounded)."""
        if not self.is_distributed:
            return bool(ok)
        self._agree_calls = getattr(self, "_agree_calls", 0) + 1
        vals = self.all_gather_bytes(f"hipdsml/agree/{key}/{self._agree_calls}", b"1" if ok else b"0")
        return all(v == b"1" for v in vals)

    def barrier(self) -> None:
        if self.is_distributed:
            with self.guard("barrier"):
                if self.device.type == "cuda" and self.backend == "nccl":
                    dist.barrier(device_ids=[self.device.index])
                    torch.cuda.synchronize(self.device)
                else:
                    dist.barrier()

    def share_bytes(self, key: str, value: Optional[bytes]) -> bytes:
        """Rank 0 publishes `value` under `key` in the TCP store; every rank reads it."""
        if not self.is_distributed:
            assert value is not None
            return value
        store = dist.distributed_c10d._get_default_store()
        if self.rank == 0:
            assert value is not None
            store.set(key, value)
        with self.guard(f"store.get {key}"):
            return bytes(store.get(key))

    def all_gather_bytes(self, key: str, value: bytes) -> list:
        """Every rank publishes `value`; returns all ranks' values in rank order."""
        if not self.is_distributed:
            return [value]
        store = dist.distributed_c10d._get_default_store()
        store.set(f"{key}/{self.rank}", value)
        with self.guard(f"store.get {key}"):
            return [bytes(store.get(f"{key}/{r}")) for r in range(self.world_size)]

    def replicas_identical(self, t: torch.Tensor, key: str = "replicas") -> bool:
        """Collective: whether `t` holds the same bytes on every rank (a
        SHA-256 of each rank's copy, exchanged through the TCP store).  Data
        parallelism here never broadcasts weights -- every replica applies the
        same summed gradient -- so this is the end-of-run proof that they did
        (the reference re-sent the weights to every device each step instead,
        client.go:642-644)."""
        import hashlib

        if not self.is_distributed:
            return True
        self._hash_calls = getattr(self, "_hash_calls", 0) + 1
        raw = t.detach().contiguous().reshape(-1).view(torch.uint8).cpu().numpy()
        h = hashlib.sha256(raw.tobytes()).digest()
        hs = self.all_gather_bytes(f"hipdsml/{key}/{self._hash_calls}", h)
        return all(x == hs[0] for x in hs)

    def destroy(self) -> None:
        if self.watchdog is not None:
            self.watchdog.stop()
        if self.initialized_here and dist.is_initialized():
            if self.watchdog is None or self.watchdog.fault is None:
                dist.destroy_process_group()  # a faulted group may not shut down cleanly
            self.initialized_here = False


_uid_counter = 0


def rccl_blocking_default() -> bool:
    """Blocking RCCL communicators unless HIPDSML_RCCL_NONBLOCKING=1: the
    non-blocking config has only run with single-rank communicators so far
    (ADVICE r2), so multi-GPU jobs keep RCCL's default mode until validated."""
    return os.environ.get("HIPDSML_RCCL_NONBLOCKING", "0") != "1"


def make_native_comm(ctx: DistContext, blocking: Optional[bool] = None, watch: bool = True):
    """Bootstrap a native RCCL communicator over the process group's store.

    Blocking by default (:func:`rccl_blocking_default`).  Either way the
    context's watchdog polls the communicator's async error and, on a fault or a
    stalled guarded section, aborts it from its own thread (``ncclCommAbort`` is
    legal on a blocking communicator while another thread waits in RCCL), so a
    dead peer ends the job instead of hanging it (parallel/watchdog.py).
    ``watch=False`` leaves it unregistered (a throwaway probe communicator the
    caller aborts and destroys itself)."""
    if blocking is None:
        blocking = rccl_blocking_default()
    from ..ops.native import require_native

    global _uid_counter
    C = require_native()
    _uid_counter += 1
    key = f"hipdsml/rccl_uid/{_uid_counter}"
    uid = C.rccl_unique_id() if ctx.rank == 0 else None
    uid = ctx.share_bytes(key, uid)
    with ctx.guard("ncclCommInitRank"):
        comm = C.RcclComm(uid, ctx.rank, ctx.world_size, ctx.device.index, blocking)
    if watch and ctx.watchdog is not None:
        ctx.watchdog.watch_comm(comm)
    return comm

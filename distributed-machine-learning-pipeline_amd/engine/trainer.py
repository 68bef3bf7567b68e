"""Data-parallel MLP training engine.

One replica per process / GPU.  On a GPU the whole step runs in the native
runner (three fused HIP kernels + gradient all-reduce + SGD, optionally
captured into one hipGraph); on a CPU-only host the fp32 torch reference math
runs instead (used by the CPU test-suite and gloo multi-process tests).

Reference training loop being replaced: ``DSML/client/client.go:579-653``
(10 epochs x 937 batches, forward/backward on the client CPU, gradient pushed
to every device, "AllReduceRing", gradient pulled back, SGD on the client,
weights pushed to every device).  Here weights, data and gradients never leave
HBM; each replica trains on its own shard and gradients are averaged.
"""
from __future__ import annotations

import logging
import time
from dataclasses import dataclass
from typing import Dict, Optional

import torch

from ..data.mnist import Dataset
from ..models.mlp import MlpLayout, MlpSpec, forward_ref, grads_ref, init_params
from ..parallel.dist import DistContext, make_native_comm
from ..utils.initbudget import InitPhases

log = logging.getLogger("hipdsml.trainer")

SYNC_MODES = ("auto", "pkx", "pk", "pk2", "pkg", "pkg2", "xact", "xgmi", "rccl", "ring", "torch")
# fused over xGMI peer memory: into K_C (xact, xgmi) or into the persistent step
# (pk: one-shot sum of every wave's gradient slot, pk2: two-shot, i.e.
# reduce-scatter + all-gather per slot: 2(N-1)/N slots per link instead of N-1)
EXCHANGE_MODES = ("pkx", "pk", "pk2", "pkg", "pkg2", "xact", "xgmi")
# persistent-step replica exchanges -> kernel algo (kernels/mlp_persist.hip):
# pk / pk2 the direct form with one- / two-shot gradient-slot sums; pkg / pkg2
# the Gram form (every peer's dZ1 pushed for the layer-1 correction, the
# gradient-slot sums off the critical path); pkx the Gram form with an
# exchange-free layer 1 (every replica forms the global-batch dW1 from the
# peers' dZ1 rows it already receives and the all-gathered input shards: no
# layer-1 gradient crosses xGMI, only the upper layers' 16 tile slots)
PERSIST_MODES = {"pk": 0, "pk2": 1, "pkg": 2, "pkg2": 3, "pkx": 4}
# the modes that read the all-gathered, swizzled input shards (self.Xall)
XALL_MODES = ("xact", "pkx")


@dataclass
class StepStats:
    loss_sum: float = 0.0
    correct: float = 0.0
    count: float = 0.0

    @property
    def avg_loss(self) -> float:
        return self.loss_sum / max(self.count, 1.0)

    @property
    def accuracy(self) -> float:
        return 100.0 * self.correct / max(self.count, 1.0)


def _xgmi_eligible(ctx: DistContext, node_local: Optional[bool] = None) -> bool:
    """Whether the fused xGMI exchanges apply: GPU replicas, a process group,
    2..8 ranks, all on this node (IPC peer memory).  The group's backend does
    not matter -- it carries only the control plane (IPC handles, the
    self-test all-reduce, agreement on the mode); the data moves over xGMI --
    so a gloo group with an external RCCL comm (the gpu_sim device servers,
    rpc/device_server.py ConfigureModel) qualifies like a torchrun RCCL job.
    `node_local` None: from torchrun's LOCAL_WORLD_SIZE."""
    import os

    if node_local is None:
        node_local = int(os.environ.get("LOCAL_WORLD_SIZE", ctx.world_size)) == ctx.world_size
    return (ctx.device.type == "cuda" and ctx.backend != "none" and 1 < ctx.world_size <= 8
            and bool(node_local))


def _pad_cols(X: torch.Tensor, mult: int = 4) -> torch.Tensor:
    d = X.shape[1]
    if d % mult == 0:
        return X.contiguous()
    out = torch.zeros(X.shape[0], d + (mult - d % mult), dtype=X.dtype, device=X.device)
    out[:, :d] = X
    return out


class MlpTrainer:
    def __init__(self, spec: MlpSpec, data: Dataset, batch: int = 64, lr: float = 0.01, *,
                 ctx: Optional[DistContext] = None, seed: int = 0, init: str = "reference",
                 momentum: float = 0.0, weight_decay: float = 0.0, sync: str = "rccl",
                 ring_chunk_bytes: int = 0, graph_steps: int = 0,
                 params: Optional[torch.Tensor] = None, external_comm=None,
                 capture_collectives: Optional[bool] = None, xchg_timeout_ms: float = 10000.0,
                 xact_waves: int = 0, auto_fallback: str = "rccl",
                 stream: Optional["torch.cuda.Stream"] = None, persist: Optional[bool] = None,
                 grad_allreduce=None, node_local: Optional[bool] = None,
                 persist_place_trials: Optional[int] = None,
                 init_phases: Optional[InitPhases] = None):
        if sync not in SYNC_MODES:
            raise ValueError(f"sync must be one of {SYNC_MODES}")
        self.ctx = ctx or DistContext()
        # init wall-clock phases + the total budget of the optional ones
        # (utils/initbudget.py); bench.py passes its own to cover the whole job
        self.init_phases = init_phases if init_phases is not None else InitPhases(self.ctx)
        self.spec = spec
        self.device = self.ctx.device
        self.batch = int(batch)
        self.lr = float(lr)
        self.momentum = float(momentum)
        self.weight_decay = float(weight_decay)
        self.sync = sync
        self.graph_steps = int(graph_steps)
        if len(data) < self.batch:
            raise ValueError(f"dataset has {len(data)} rows < batch {self.batch}")
        if data.X.shape[1] != spec.dims[0]:
            raise ValueError(f"data dim {data.X.shape[1]} != model input {spec.dims[0]}")
        ph = self.init_phases
        with ph.phase("upload"):
            self.X = _pad_cols(data.X.to(self.device, torch.float32))
            self.y = data.y.to(self.device, torch.int32).contiguous()
            if self.device.type == "cuda":
                torch.cuda.synchronize(self.device)
        self.nbatches = len(data) // self.batch
        self.layout = MlpLayout(spec, self.batch, self.nbatches)
        with ph.phase("param_init"):
            P = params if params is not None else init_params(self.layout, seed, init)
        if P.numel() != self.layout.nparams:
            raise ValueError("params do not match the layout")
        self.P = P.to(self.device, torch.float32).contiguous().clone()
        self.G = torch.zeros_like(self.P)
        self.V = torch.zeros_like(self.P) if (momentum or weight_decay) else torch.empty(0, device=self.device)
        self.steps_done = 0
        self._stats_cpu = StepStats()
        self.comm = external_comm
        # host replicas without a process group (device servers on CPU): a
        # callable that sums the flat fp32 gradient over the replicas in place
        # (the device-driven gRPC ring, rpc/device_server.py _rpc_ring)
        self.grad_allreduce = grad_allreduce
        self.xchg = None
        if capture_collectives is None:  # RCCL collectives recorded into the step graphs
            import os

            # off by default until a multi-GPU run has validated captured RCCL
            # collectives: eager ncclAllReduce / send-recv per step
            capture_collectives = os.environ.get("HIPDSML_CAPTURE_COLLECTIVES", "0") == "1"
        self.capture_collectives = bool(capture_collectives)
        self.xchg_timeout_ms = xchg_timeout_ms
        self.xact_waves = int(xact_waves)  # 0: 8-wave tile blocks from 4 ranks on, else 4
        # sync='auto' without RCCL (one-GPU rehearsals, where RCCL refuses two
        # ranks on a device): the non-exchange candidate is a torch.distributed
        # all-reduce between fwd/bwd and the update
        if auto_fallback not in ("rccl", "torch"):
            raise ValueError("auto_fallback must be 'rccl' or 'torch'")
        self.auto_fallback = auto_fallback
        # every rank on this node (None: torchrun's LOCAL_WORLD_SIZE says);
        # the gpu_sim device servers pass what their process group found
        self._node_local = node_local
        self.sync_active = "none"
        self.sync_times: Dict[str, float] = {}
        # data-only tables built at init, outside any timed region: name -> ms
        self.precompute_ms: Dict[str, float] = {}
        self.Xall: Optional[torch.Tensor] = None
        self._exchanges: Dict[str, object] = {}
        self.runner = None
        # caller-owned stream for the native runner; None: the runner follows
        # torch's current stream at every call (no cross-stream edges per step)
        self._stream = stream
        # persistent fused step (kernels/mlp_persist.hip): None = when supported
        # (plain SGD, 784-128-64-10 or 784-128-10 at batch <= 64); HIPDSML_PERSIST=0 disables
        if persist is None:
            import os

            persist = os.environ.get("HIPDSML_PERSIST", "1") != "0"
        self._want_persist = bool(persist)
        # hand-off buffers tried for the single-replica persistent step (the
        # fastest kept, see _place_persist_buffer); HIPDSML_PK_PLACE overrides
        import os

        if persist_place_trials is None:
            persist_place_trials = int(os.environ.get("HIPDSML_PK_PLACE", "12"))
        self._place_trials = int(persist_place_trials)
        # data parallel: candidates per rank in the collective search
        self._place_trials_dp = int(os.environ.get("HIPDSML_PK_PLACE_DP", "4"))
        self.persist_place_us: Optional[list] = None
        self.pk_buf: Optional[torch.Tensor] = None
        self.pk_err: Optional[torch.Tensor] = None
        if self.device.type == "cuda":
            self.backend = "hip"
            with ph.phase("native_init"):
                self._init_hip(ring_chunk_bytes)
        else:
            self.backend = "torch"

    # ------------------------------------------------------------------ hip --
    def _init_hip(self, ring_chunk_bytes: int) -> None:
        from ..ops.native import require_native

        C = require_native()
        if not self.layout.fused_ok:
            raise ValueError(f"model {self.spec} does not fit the fused fp32 step "
                             f"(LDS {self.layout.lds_floats * 4} B); use the wide bf16 engine")
        d = self.device
        self.ws = torch.zeros(self.layout.ws_floats, dtype=torch.float32, device=d)
        self.slab = torch.zeros(self.layout.slab_floats(), dtype=torch.float32, device=d)
        self.ctr = torch.zeros(2, dtype=torch.int64, device=d)
        self.stats = torch.zeros(4, dtype=torch.float32, device=d)
        self.runner = C.MlpRunner(self.layout.desc_list(), self.X, self.y, self.P, self.G, self.V,
                                  self.ws, self.slab, self.ctr, self.stats, self.lr, self.momentum,
                                  self.weight_decay,
                                  stream=self._stream.cuda_stream if self._stream is not None else 0,
                                  follow_torch=self._stream is None)
        self.runner.set_world_size(self.ctx.world_size)
        # chunk of the in-house ring all-reduce; <= 0: tuned at init (N > 1)
        self._ring_chunk = int(ring_chunk_bytes)
        self.ring_chunk_sweep_us: Optional[Dict[str, float]] = None
        # sync modes whose collectives have run one eager step (RCCL connects a
        # peer pair on its first send/recv, which must never happen inside a
        # graph capture): 'rccl' warms ncclAllReduce's connections, 'ring' the
        # send/recv pairs of the in-house ring -- tracked per mode
        self._warm_modes: set = set()
        if not self.ctx.is_distributed:
            plain = not (self.momentum or self.weight_decay)
            if self._want_persist and plain and C.mlp_persist_supported(self.layout.desc_list()):
                self.pk_buf = torch.zeros(C.mlp_persist_xbuf_granules(), dtype=torch.int64, device=d)
                self.pk_err = torch.zeros(1, dtype=torch.int32, device=d)
                t0 = time.perf_counter()
                with self.init_phases.phase("gram_table"):
                    self.pk_gram = self._gram_table()
                    torch.cuda.synchronize(d)
                self.precompute_ms["gram_table"] = round(1e3 * (time.perf_counter() - t0), 2)
                self.runner.set_persist_gram(self.pk_gram)
                self.runner.set_persist(self.pk_buf, self.pk_err, 2000.0)
                self.sync_active = "none"
                if self.device.type == "cuda" and self._place_trials > 1:
                    t0 = time.perf_counter()
                    with self.init_phases.phase("persist_place"):
                        self._place_persist_buffer(self._place_trials)
                    self.precompute_ms["persist_place"] = round(1e3 * (time.perf_counter() - t0), 2)
            return
        if self.sync == "torch":
            self.sync_active = "torch"
            return
        plain = not (self.momentum or self.weight_decay)
        if self.sync in EXCHANGE_MODES and not plain:
            raise ValueError(f"sync='{self.sync}' implements plain SGD; use rccl for momentum/"
                             "weight decay")
        torch_fallback = self.sync == "auto" and self.auto_fallback == "torch"
        if torch_fallback:
            self.sync_active = "torch"
        elif self.sync not in EXCHANGE_MODES:  # strict exchange modes: no RCCL fallback
            ph = self.init_phases
            if self.comm is None:
                with ph.phase("rccl_comm_init"):
                    self.comm = make_native_comm(self.ctx)
            if self._ring_chunk <= 0:
                if (self.sync in ("auto", "ring") and self.ctx.backend != "none"
                        and ph.allow("ring_tune")):
                    # measured, not guessed: every distinct chunk timed on the
                    # gradient itself, max over ranks (parallel/ring_tune.py)
                    from ..parallel.ring_tune import tune_ring_chunk

                    with ph.phase("ring_tune"):
                        res = tune_ring_chunk(self.ctx, self.comm, self.G)
                    self._ring_chunk = int(res["best"])
                    # both schedules' sweeps, the choice, and any pipelined-probe error
                    self.ring_chunk_sweep_us = {k: v for k, v in res.items() if k != "best"}
                else:
                    self._ring_chunk = 1 << 20
            # the in-house ring's scratch, sized once (never inside a graph capture)
            self.comm.reserve_ring(self.layout.nparams, self._ring_chunk)
            self.runner.set_comm(self.comm, 1 if self.sync == "ring" else 0, self._ring_chunk)
            self.sync_active = "ring" if self.sync == "ring" else "rccl"
        if self.exchange_candidates():
            with self.init_phases.phase("exchanges"):
                self._init_exchanges()

    def exchange_candidates(self) -> list:
        """The fused xGMI exchange forms _init_exchanges self-tests, in
        preference order ([] when none applies: sync='auto' needs plain SGD and
        an eligible group, see _xgmi_eligible)."""
        if self.sync in EXCHANGE_MODES:
            return [self.sync]
        plain = not (self.momentum or self.weight_decay)
        if not (self.sync == "auto" and plain and _xgmi_eligible(self.ctx, self._node_local)):
            return []
        # pk2 pays one more flag round trip per slot for fewer bytes: a
        # candidate from 3 replicas on (at 2 it moves the same bytes as pk)
        two = self.ctx.world_size >= 3
        return (["pkx", "pkg"] + (["pkg2"] if two else []) + ["pk"] + (["pk2"] if two else [])
                + ["xact", "xgmi"])

    # ------------------------------------------------------ xGMI exchanges --
    def _gather_inputs(self) -> torch.Tensor:
        """Every rank's input shard, replicated on this GPU in MFMA fragment
        order (parallel/xchg.py swizzle_inputs) — the activation exchange reads
        every rank's batch rows locally.  Collective."""
        from ..parallel.xchg import swizzle_inputs

        t0 = time.perf_counter()
        out = swizzle_inputs(self._gather_plain(), self.batch)
        torch.cuda.synchronize(self.device)
        self.precompute_ms["xall_swizzled"] = round(1e3 * (time.perf_counter() - t0), 2)
        return out

    def _activate(self, mode: Optional[str]) -> None:
        """Point the native runner at one gradient-sync mode.  None keeps the
        RCCL communicator as configured; 'rccl' / 'ring' select ncclAllReduce
        or the in-house multi-ring send/recv all-reduce on it."""
        if mode in PERSIST_MODES:
            self.xchg = self._exchanges[mode]
            # waits on peers are bounded like the other exchanges' (ranks can enter
            # a launch seconds apart, e.g. around a checkpoint)
            self.runner.set_persist(self.pk_buf, self.pk_err, max(2000.0, self.xchg_timeout_ms),
                                    self.xchg, PERSIST_MODES[mode])
            return
        if self.pk_buf is not None:
            self.runner.set_persist(None)  # leave the persistent step
        if mode in (None, "rccl", "ring", "torch"):
            self.runner.set_exchange(None)
            self.xchg = None
            if mode in ("rccl", "ring") and self.comm is not None:
                self.runner.set_comm(self.comm, 1 if mode == "ring" else 0, self._ring_chunk)
        elif mode == "xgmi":
            self.xchg = self._exchanges["xgmi"]
            self.runner.set_exchange(self.xchg)
        else:
            self.xchg = self._exchanges["xact"]
            self.runner.set_act_exchange(self.xchg, self.Xall, self.Xall[0].numel(),
                                         self.xact_waves)

    def _setup_exchange(self, mode: str) -> str:
        """Collective: build `mode`'s buffers, check three steps (in two
        launches: a launch split and a parity wrap) against fp32 torch
        gradients summed by a torch.distributed all-reduce
        (parallel/xchg.py verify_against_allreduce).  Returns '' or the
        (agreed) error."""
        from ..parallel import xchg as X

        try:
            if mode in PERSIST_MODES:
                C = self.runner_module()
                if not (self._want_persist and C.mlp_persist_supported(self.layout.desc_list())):
                    raise X.ExchangeUnavailable("the persistent step covers 784-128-64-10 and "
                                                "784-128-10 at batch <= 64")
                if PERSIST_MODES[mode] >= 2:
                    if self._replicas_per_gpu() > 2:
                        # the Gram grid places every replica's 4 chain + 16 tile
                        # blocks on XCD 0 (32 CUs, one block each): three
                        # replicas sharing a GPU cannot all be resident
                        raise X.ExchangeUnavailable("the Gram form runs at most 2 replicas per GPU")
                    if self.pk_gram_dp is None:
                        self.pk_gram_dp = self._gram_table_dp()  # collective
                    self.runner.set_persist_gram(self.pk_gram_dp)
                if mode == "pkx":
                    if self.Xall is None:
                        self.Xall = self._gather_inputs()  # collective
                    self.runner.set_persist_xall(self.Xall, self.Xall[0].numel())
                half, ntiles = C.MlpRunner.persist_xchg_size(self.ctx.world_size,
                                                             PERSIST_MODES[mode])
                x = X.make_exchange(self.ctx, half, ntiles, self.xchg_timeout_ms)
                if self.pk_buf is None:
                    self.pk_buf = torch.zeros(C.mlp_persist_xbuf_granules(), dtype=torch.int64,
                                              device=self.device)
                    self.pk_err = torch.zeros(1, dtype=torch.int32, device=self.device)
            elif mode == "xact":
                if not X.act_supported(self.layout):
                    raise X.ExchangeUnavailable("activation exchange needs batch <= 64 and "
                                                "layer input dims that are multiples of 16")
                if self.Xall is None:
                    self.Xall = self._gather_inputs()
                x = X.make_act_exchange(self.ctx, self.layout, self.xchg_timeout_ms)
            else:
                x = X.make_peer_exchange(self.ctx, self.layout, self.xchg_timeout_ms)
        except X.ExchangeUnavailable as e:  # agreed on every rank
            return str(e)
        self._exchanges[mode] = x
        self._activate(mode)
        diff = X.verify_against_allreduce(self)  # collective, same result on all ranks
        self._activate(None)
        self._rewound()  # the step counter went back: stale persistent hand-off tags
        # fp32 against fp32 torch, different summation orders (the Gram forms add
        # the correction to a separately rounded partial): the unit tests' bound
        return "" if diff <= 2e-5 else f"self-test mismatch {diff}"

    def _init_exchanges(self) -> None:
        """Set up the fused xGMI exchanges, self-test each against a
        torch.distributed all-reduce and keep (sync='auto') the fastest of
        {xact, xgmi, rccl} measured on this node.  Every decision is collective.

        * xact — activation exchange: each GPU pushes its 100 KB of activations
          and activation gradients to every peer and computes the global-batch
          weight gradients itself (kernels/mlp_f32_xact.hip);
        * xgmi — one-shot gradient exchange: each GPU reads every peer's 437 KB
          of weight-gradient tiles (kernels/mlp_f32.hip XCHG path);
        * rccl — ncclAllReduce of the gradient between fwd/bwd and the update."""
        self._exchanges: Dict[str, object] = {}
        self.Xall = None
        self.pk_gram_dp = None
        strict = self.sync in EXCHANGE_MODES
        modes = self.exchange_candidates()
        ph = self.init_phases
        ok = []
        try:
            self._init_exchange_modes(modes, strict, ok, ph)
        finally:
            # the all-gathered fp32 shards: only the tables' builds read them
            # (released on the failure path too)
            self._plain = None
        if self.sync_active not in XALL_MODES and self.Xall is not None:
            # the replicated inputs (N x the shard) are only read by xact / pkx:
            # free them, the runner's references included
            self.Xall = None
            self.runner.release_xall()

    def _init_exchange_modes(self, modes, strict: bool, ok: list, ph: InitPhases) -> None:
        for m in modes:
            if ok and not strict and not ph.allow(f"selftest_{m}"):
                continue  # init budget spent: the candidates that passed are enough
            with ph.phase(f"selftest_{m}"):
                err = self._setup_exchange(m)
            if err:
                if strict:
                    raise RuntimeError(f"{m} exchange unavailable: {err}")
                log.warning("%s exchange disabled (%s)", m, err)
            else:
                ok.append(m)
        choice = ok[0] if ok else None
        if self.sync == "auto" and ok and ph.allow("sync_timing"):
            # every candidate timed the way train_steps runs it (graph replay,
            # RCCL collectives captured too); ties go to the earlier candidate
            # (over budget: the first candidate that passed, in preference order)
            fallback = ["rccl", "ring"] if self.comm is not None else [self.sync_active]
            with ph.phase("sync_timing"):
                times = self.time_sync_modes(ok + fallback)
            choice = min(times, key=times.get)
            log.info("sync auto: %s", ", ".join(f"{k} {v:.1f} us/step" for k, v in times.items()))
            self.sync_times = times
        self._set_mode(choice or self.sync_active)
        if (self.sync_active in PERSIST_MODES and self._place_trials_dp > 1
                and ph.allow("persist_place_dp")):
            t0 = time.perf_counter()
            with ph.phase("persist_place_dp"):
                self._place_persist_buffer_dp(self._place_trials_dp)  # collective
            self.precompute_ms["persist_place_dp"] = round(1e3 * (time.perf_counter() - t0), 2)

    @staticmethod
    def runner_module():
        from ..ops.native import require_native

        return require_native()

    def _set_mode(self, mode: str) -> None:
        self._activate(mode)
        self.sync_active = mode

    def time_sync_modes(self, modes, steps: int = 0) -> Dict[str, float]:
        """Collective: µs/step (max over ranks) of each gradient-sync mode in
        `modes` (xact / xgmi / rccl / ring / torch), measured as train_steps
        runs it; the training state and the active mode are restored."""
        cur = self.sync_active
        steps = steps or max(100, 2 * self.graph_steps)
        out: Dict[str, float] = {}
        for m in modes:
            if m in EXCHANGE_MODES and m not in self._exchanges:
                continue
            if m in XALL_MODES and self.Xall is None:
                continue  # its replicated inputs were released when another mode won
            if m in ("rccl", "ring") and self.comm is None:
                continue
            self._set_mode(m)
            out[m] = round(1e6 * self._time_steps(steps), 2)
        self._set_mode(cur)
        return out

    def _time_steps(self, n: int) -> float:
        """Max-over-ranks wall time per step of the active mode, run exactly as
        train_steps runs it (graphs prepared and warmed first); state restored."""
        from ..parallel import xchg as X

        P0, ctr0, st0 = self.P.clone(), self.ctr.clone(), self.stats.clone()
        sd0 = self.steps_done
        self.train_steps(n)  # warm-up: RCCL connections, graph capture and upload
        self.runner.synchronize()
        self.ctx.barrier()
        t0 = time.perf_counter()
        self.train_steps(n)
        self.runner.synchronize()
        dt = (time.perf_counter() - t0) / n
        self.steps_done = sd0
        dt = self.ctx.all_reduce_scalars(dt, op="max")[0]
        self.P.copy_(P0)
        self.ctr.copy_(ctr0)
        self.stats.copy_(st0)
        self._rewound()
        # the counters went back: rewind every exchange's flags (collective)
        for x in getattr(self, "_exchanges", {}).values():
            X.reset_group(self.ctx, x)
        torch.cuda.synchronize(self.device)
        self.ctx.barrier()
        return dt

    def _place_persist_buffer(self, trials: int, steps: int = 300) -> None:
        """Where the single-replica persistent step's hand-off buffer lands in
        HBM sets its speed: the same kernel, re-timed on the same buffer within
        0.1 %, runs 7.0-7.95 us/step depending on which of 8 fresh allocations
        carries its flags and granules (tools/pk_placement.py,
        profiles/r5_pk_placement.json) -- the hand-offs' round trips depend on
        the physical pages' memory channels; about 1 allocation in 4-8 is fast.  So `trials` buffers are allocated
        (every earlier one kept alive: each lands on new pages), each timed
        over `steps` steps with the model state restored (_time_steps), and
        the fastest is kept.  Data-only work at init, before any timed step."""
        cands = [self.pk_buf]
        times = [self._time_steps(steps)]
        for _ in range(trials - 1):
            b = torch.zeros_like(self.pk_buf)
            cands.append(b)
            self.pk_buf = b
            self.runner.set_persist(b, self.pk_err, 2000.0)
            times.append(self._time_steps(steps))
        best = min(range(len(times)), key=times.__getitem__)
        self.pk_buf = cands[best]
        self.runner.set_persist(self.pk_buf, self.pk_err, 2000.0)
        self._rewound()
        torch.cuda.synchronize(self.device)
        self.persist_place_us = [round(1e6 * t, 3) for t in times]
        del cands  # the other candidates go back to the allocator

    def _place_persist_buffer_dp(self, trials: int, steps: int = 300) -> None:
        """Collective: the data-parallel persistent step's hand-off buffer
        placement (see _place_persist_buffer: the lone-replica pkx step at
        N = 4 runs 9.5-10.7 us/step over 8 allocations of that buffer,
        profiles/r5_pk_placement.json).  The step is as slow as its slowest
        replica, so the search is coordinate descent over the ranks: in rank
        r's turn, r alone tries `trials` - 1 fresh buffers (the others keep
        theirs) and keeps one only if the max-over-ranks step time improves.
        Every rank sees the same timings (_time_steps reduces them), so every
        decision agrees."""
        algo = PERSIST_MODES[self.sync_active]
        timeout = max(2000.0, self.xchg_timeout_ms)
        best = self._time_steps(steps)
        times = [best]
        cands = [self.pk_buf]
        for r in range(self.ctx.world_size):
            for _ in range(trials - 1):
                prev = self.pk_buf
                if self.ctx.rank == r:
                    cands.append(torch.zeros_like(prev))
                    self.pk_buf = cands[-1]
                    self.runner.set_persist(self.pk_buf, self.pk_err, timeout, self.xchg, algo)
                t = self._time_steps(steps)
                times.append(t)
                if t < best:
                    best = t
                elif self.ctx.rank == r:
                    self.pk_buf = prev
                    self.runner.set_persist(prev, self.pk_err, timeout, self.xchg, algo)
        self._rewound()
        torch.cuda.synchronize(self.device)
        self.ctx.barrier()
        self.persist_place_us = [round(1e6 * t, 3) for t in times]
        del cands

    def _hip_step_torch_sync(self, n: int) -> None:
        import torch.distributed as dist

        if self.runner.follows_torch:
            stream = torch.cuda.current_stream(self.device)
        else:
            stream = torch.cuda.ExternalStream(self.runner.stream_handle(), device=self.device)
        for _ in range(n):
            self.runner.fwd_bwd()
            with torch.cuda.stream(stream):
                dist.all_reduce(self.G)
            self.runner.update()

    # -------------------------------------------------------------- public --
    @property
    def persistent(self) -> bool:
        """Steps run as one persistent launch per train_steps call."""
        return self.runner is not None and self.pk_buf is not None and self.runner.persist_active()

    def _rewound(self) -> None:
        """The step counter went back: stale hand-off tags could match again
        (and the pipeline state a launch carries over to the next is gone)."""
        if self.pk_buf is not None:
            self.pk_buf.zero_()
            self.pk_err.zero_()
            self.runner.clear_persist_error()

    def _gram_table(self) -> torch.Tensor:
        """Per-batch Gram blocks of the single-replica persistent step
        (engine/gram.py gram_table: float[nbatches][64][64], 16 KB a batch)."""
        nb, B, d0 = self.nbatches, self.batch, self.spec.dims[0]
        # one launch of kernels/gram.hip (fp64 MFMA); engine/gram.py is its oracle
        return self.runner_module().gram_table(self.X, self.X, nb, B, d0)

    def _gather_plain(self) -> torch.Tensor:
        """Every rank's input rows (fp32 [world][rows][d0], rank order) on this
        GPU.  Collective."""
        import torch.distributed as dist

        from ..parallel.xchg import ExchangeUnavailable

        if getattr(self, "_plain", None) is not None:  # gathered once per _init_exchanges
            return self._plain
        ctx = self.ctx
        rows = self.nbatches * self.batch
        lo = ctx.all_reduce_scalars(float(rows), op="min")[0]
        hi = ctx.all_reduce_scalars(float(rows), op="max")[0]
        if lo != hi:
            raise ExchangeUnavailable("ranks hold different numbers of batches")
        own = self.X[:rows, : self.spec.dims[0]].contiguous()
        if ctx.backend == "nccl":
            out = torch.empty((ctx.world_size,) + tuple(own.shape), dtype=own.dtype, device=self.device)
            dist.all_gather_into_tensor(out, own)
        else:
            parts = [torch.empty(own.shape, dtype=own.dtype) for _ in range(ctx.world_size)]
            dist.all_gather(parts, own.cpu())
            out = torch.stack(parts).to(self.device)
        self._plain = out
        return out

    def _replicas_per_gpu(self) -> int:
        """How many ranks share this rank's GPU (1 on a node, one process per
        GPU; more in a one-GPU rehearsal).  Collective; the max over ranks."""
        if getattr(self, "_rpg", None) is None:
            import torch.distributed as dist

            ids = [None] * self.ctx.world_size
            dist.all_gather_object(ids, str(torch.cuda.get_device_properties(self.device).uuid))
            self._rpg = max(ids.count(u) for u in ids)
        return self._rpg

    def _gram_table_dp(self) -> torch.Tensor:
        """Cross-replica Gram blocks of the data-parallel persistent step in Gram
        form (sync pkg / pkg2; engine/gram.py gram_table_dp:
        float[nbatches][world][64][64]).  Collective (all-gathers the shards)."""
        nb, B, d0 = self.nbatches, self.batch, self.spec.dims[0]
        t0 = time.perf_counter()
        # every source's batches against this rank's, one launch (kernels/gram.hip)
        T = self.runner_module().gram_table(self._gather_plain(), self.X, nb, B, d0)
        torch.cuda.synchronize(self.device)
        self.precompute_ms["gram_table_dp"] = round(1e3 * (time.perf_counter() - t0), 2)
        return T

    def _params_rewritten(self) -> None:
        """P changed outside the persistent launches: the partials the last
        launch computed from the old weights must not be carried over."""
        if self.pk_buf is not None and self.runner is not None:
            self.runner.set_persist_carry(False)

    def _graphs_on(self) -> bool:
        """Whether train_steps replays hipGraphs for the active sync mode."""
        if self.graph_steps <= 0 or self.runner is None or self.persistent:
            return False
        if not self.ctx.is_distributed:
            return True
        if self.sync_active == "torch":
            return False  # torch.distributed all-reduce between native launches
        if self.sync_active in ("rccl", "ring"):
            return self.capture_collectives
        return True  # fused xGMI exchanges

    def _graph_sizes(self, n: int):
        reps, rem = divmod(n, self.graph_steps)
        return ([self.graph_steps] if reps else []) + ([rem] if rem else [])

    def prepare(self, n: int) -> None:
        """Capture (outside any timed region) the graphs train_steps(n) will
        replay: a run of n = q*G + r steps replays a G-step and an r-step graph."""
        if self.backend != "hip" or not self._graphs_on():
            return
        if self.sync_active in ("rccl", "ring") and self.sync_active not in self._warm_modes:
            return  # captured on first use, after an eager step (train_steps)
        for k in self._graph_sizes(n):
            if not self.runner.captured(k):
                self.runner.capture(k, True)

    def train_steps(self, n: int) -> None:
        """Enqueue `n` optimizer steps (asynchronous on GPU)."""
        if n <= 0:
            return
        if self.pk_buf is not None and self.runner.persist_active():
            # single replica, persistent step: ONE launch for the n steps
            self.runner.step(n)
            self.steps_done += n
            return
        if self.backend == "torch":
            for _ in range(n):
                self._torch_step()
                self.steps_done += 1
            return
        if self.ctx.is_distributed and self.sync_active == "torch":
            self._hip_step_torch_sync(n)
        elif self._graphs_on():
            self.steps_done += n
            if self.sync_active in ("rccl", "ring") and self.sync_active not in self._warm_modes:
                # RCCL connects its peers on the first collective it enqueues:
                # run that step eagerly on every rank before anything is captured
                self.runner.step(1)
                self._warm_modes.add(self.sync_active)
                n -= 1
                if n == 0:
                    return
            self.prepare(n)
            reps, rem = divmod(n, self.graph_steps)
            if reps:
                self.runner.replay(reps, self.graph_steps)
            if rem:
                self.runner.replay(1, rem)
            return
        else:
            self.runner.step(n)
        self.steps_done += n

    def synchronize(self) -> None:
        """Wait for every enqueued step; raises if a peer timed out / faulted
        (the wait runs under the job's watchdog, parallel/watchdog.py)."""
        with self.ctx.guard("synchronize"):
            if self.runner is not None:
                self.runner.join_into_torch()  # torch reads P / stats after the runner (event edge)
                self.runner.synchronize()
                if self.xchg is not None:
                    from ..parallel.xchg import check

                    check(self.xchg)
                if self.pk_buf is not None and self.runner.persist_failed():
                    self.runner.set_persist_carry(False)  # the launch left a half-written pipeline
                    raise RuntimeError("persistent step: an on-chip hand-off timed out "
                                       "(launch ended early; parameters are not valid)")
            elif self.device.type == "cuda":
                torch.cuda.synchronize(self.device)

    def read_stats(self, reset: bool = True, global_: bool = False) -> StepStats:
        if self.backend == "torch":
            s = StepStats(self._stats_cpu.loss_sum, self._stats_cpu.correct, self._stats_cpu.count)
            if reset:
                self._stats_cpu = StepStats()
        else:
            self.synchronize()
            v = self.stats.detach().cpu().tolist()
            s = StepStats(v[0], v[1], v[2])
            if reset:
                self.stats.zero_()
                torch.cuda.synchronize(self.device)
        if global_ and self.ctx.is_distributed:
            s = StepStats(*self.ctx.all_reduce_scalars(s.loss_sum, s.correct, s.count))
        return s

    @torch.no_grad()
    def evaluate(self, ds: Dataset) -> Dict[str, float]:
        X = _pad_cols(ds.X.to(self.device, torch.float32))
        y = ds.y.to(self.device, torch.int32).contiguous()
        if self.backend == "torch":
            logits, _ = forward_ref(self.layout, self.P, X[:, : self.spec.dims[0]])
            p = torch.softmax(logits, 1)
            loss = (-torch.log(p.gather(1, y.long().view(-1, 1)).squeeze(1) + 1e-10)).sum().item()
            correct = (logits.argmax(1) == y.long()).sum().item()
            n = X.shape[0]
        else:
            from ..ops.native import require_native

            C = require_native()
            n = X.shape[0]
            ev = MlpLayout(self.spec, n, 1)
            slab = torch.empty(ev.slab_floats(), dtype=torch.float32, device=self.device)
            ws = torch.empty(16, dtype=torch.float32, device=self.device)
            stats = torch.zeros(4, dtype=torch.float32, device=self.device)
            self.synchronize()
            C.mlp_eval(ev.desc_list(), X, y, 0, self.P, ws, slab, stats)
            torch.cuda.synchronize(self.device)
            loss, correct, _ = stats[:3].tolist()
        return {"loss": loss / max(n, 1), "accuracy": 100.0 * correct / max(n, 1), "n": n}

    # ------------------------------------------------- per-batch RPC helpers --
    @torch.no_grad()
    def forward_logits(self, X: torch.Tensor, y: Optional[torch.Tensor] = None):
        """Logits of rows X at the current params, plus (loss_sum, correct)
        when labels are given — the RunForward RPC.  GPU: the fused HIP
        forward kernels (K_A + the row chain in logits mode); CPU: torch."""
        rows = X.shape[0]
        if self.backend == "torch":
            logits, _ = forward_ref(self.layout, self.P, X.to(self.P.device, torch.float32))
            if y is None:
                return logits, 0.0, 0
            p = torch.softmax(logits, 1)
            yl = y.to(logits.device).long()
            loss = (-torch.log(p.gather(1, yl.view(-1, 1)).squeeze(1) + 1e-10)).sum().item()
            return logits, loss, int((logits.argmax(1) == yl).sum().item())
        from ..ops.native import require_native

        C = require_native()
        lay = MlpLayout(self.spec, rows, 1)
        Xd = _pad_cols(X.to(self.device, torch.float32))
        yd = (y.to(self.device, torch.int32) if y is not None
              else torch.zeros(rows, dtype=torch.int32, device=self.device)).contiguous()
        ws = torch.zeros(lay.ws_floats, dtype=torch.float32, device=self.device)
        slab = torch.empty(lay.slab_floats(), dtype=torch.float32, device=self.device)
        stats = torch.zeros(4, dtype=torch.float32, device=self.device)
        self.synchronize()
        logits = C.mlp_forward_logits(lay.desc_list(), Xd, yd, 0, self.P, ws, slab, stats).clone()
        torch.cuda.synchronize(self.device)
        if y is None:
            return logits, 0.0, 0
        loss, correct, _ = stats[:3].tolist()
        return logits, loss, int(correct)

    def batch_gradients(self, X: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
        """Flat gradient (param layout) of one batch at the current params —
        the RunBackward RPC.  GPU: the fused HIP kernels on a one-batch plan."""
        rows = X.shape[0]
        if self.backend == "torch":
            g, _, _ = grads_ref(self.layout, self.P, X.to(self.P.device), y.to(self.P.device))
            return g
        from ..ops.native import require_native

        C = require_native()
        lay = MlpLayout(self.spec, rows, 1)
        Xd = _pad_cols(X.to(self.device, torch.float32))
        yd = y.to(self.device, torch.int32).contiguous()
        G = torch.zeros_like(self.P)
        ws = torch.zeros(lay.ws_floats, dtype=torch.float32, device=self.device)
        slab = torch.zeros(lay.slab_floats(), dtype=torch.float32, device=self.device)
        ctr = torch.zeros(2, dtype=torch.int64, device=self.device)
        stats = torch.zeros(4, dtype=torch.float32, device=self.device)
        self.synchronize()
        r = C.MlpRunner(lay.desc_list(), Xd, yd, self.P, G, torch.empty(0, device=self.device),
                        ws, slab, ctr, stats, self.lr, 0.0, 0.0)
        r.fwd_bwd()
        r.synchronize()
        return G

    def apply_gradients(self, g: torch.Tensor, scale: float = 1.0) -> None:
        """P -= lr * scale * g (the ApplyGradients RPC; HIP kernel on GPU)."""
        from ..ops.functional import sgd_update_

        self.synchronize()
        sgd_update_(self.P, g.to(self.P.device).contiguous(), self.lr * scale)
        self._params_rewritten()
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)

    # --------------------------------------------------------------- torch --
    def _torch_step(self) -> None:
        b = self.steps_done % self.nbatches
        r0 = b * self.batch
        Xb = self.X[r0:r0 + self.batch, : self.spec.dims[0]]
        yb = self.y[r0:r0 + self.batch]
        g, loss_sum, correct = grads_ref(self.layout, self.P, Xb, yb)
        self._stats_cpu.loss_sum += float(loss_sum)
        self._stats_cpu.correct += float(correct)
        self._stats_cpu.count += self.batch
        world = self.ctx.world_size
        if self.grad_allreduce is not None:
            self.grad_allreduce(g)
        elif self.ctx.is_distributed:
            import torch.distributed as dist

            with self.ctx.guard("gradient all_reduce"):
                dist.all_reduce(g)
        if self.momentum or self.weight_decay:
            gg = g / world + self.weight_decay * self.P
            self.V.mul_(self.momentum).add_(gg)
            self.P.sub_(self.V, alpha=self.lr)
        else:
            self.P.sub_(g, alpha=self.lr / world)

    # --------------------------------------------------------- state / ckpt --
    def state_dict(self) -> Dict[str, object]:
        self.synchronize()
        sd = {"spec": list(self.spec.dims), "params": self.P.detach().cpu().clone(),
              "velocity": self.V.detach().cpu().clone(), "steps_done": self.steps_done,
              "lr": self.lr, "batch": self.batch}
        if self._carries_state():
            # the single-replica persistent step's pipeline state (the next step's
            # partials and correction), so a resume is bit-identical to running on;
            # valid only for the same batching of the same data (persist_meta)
            sd["persist_carry"] = self.pk_buf.detach().cpu().clone()
            sd["persist_meta"] = self._carry_meta()
        return sd

    def _carry_meta(self) -> Dict[str, object]:
        """What the carried pipeline state was computed from: the batching and a
        fingerprint of the Gram table (first and last batch blocks)."""
        import hashlib

        h = hashlib.sha256()
        if getattr(self, "pk_gram", None) is not None:
            h.update(self.pk_gram[0].detach().cpu().numpy().tobytes())
            h.update(self.pk_gram[-1].detach().cpu().numpy().tobytes())
        return {"batch": self.batch, "nbatches": self.nbatches, "gram_sha": h.hexdigest()[:32]}

    def _carries_state(self) -> bool:
        return (self.pk_buf is not None and not self.ctx.is_distributed and self.runner is not None
                and self.runner.persist_active() and self.runner.persist_carry())

    def load_state_dict(self, sd: Dict[str, object]) -> None:
        if list(sd["spec"]) != list(self.spec.dims):
            raise ValueError("checkpoint is for a different model")
        self.synchronize()
        self.P.copy_(sd["params"].to(self.device))
        if self.V.numel() and sd["velocity"].numel():
            self.V.copy_(sd["velocity"].to(self.device))
        self.steps_done = int(sd["steps_done"])
        if self.backend == "hip":
            # A = B = s at the start of step s (dsml.h step-counter protocol)
            self.ctr.fill_(self.steps_done)
            self._rewound()
            carry = sd.get("persist_carry")
            # a carry computed for another batching or data would feed a stale Z1
            # into the first resumed step: dropped, the prologue then recomputes it
            same = sd.get("persist_meta") == (self._carry_meta() if self.pk_buf is not None else None)
            if (carry is not None and same and self.pk_buf is not None and not self.ctx.is_distributed
                    and self.runner.persist_active() and carry.numel() == self.pk_buf.numel()):
                self.pk_buf.copy_(carry.to(self.device))
                self.runner.set_persist_carry(True)
            torch.cuda.synchronize(self.device)
            if self.xchg is not None:  # flags may be ahead of the restored step
                from ..parallel.xchg import reset_group

                reset_group(self.ctx, self.xchg)

    def fit(self, epochs: int, log_fn=None, test: Optional[Dataset] = None) -> Dict[str, float]:
        """Reference-compatible epoch loop (client.go:579-653 log lines)."""
        log_fn = log_fn or (lambda s: log.info(s))
        t0 = time.perf_counter()
        for ep in range(1, epochs + 1):
            self.train_steps(self.nbatches)
            st = self.read_stats(global_=True)
            log_fn(f"Epoch {ep} complete: Avg Loss: {st.avg_loss:.4f}, Accuracy: {st.accuracy:.2f}%")
        self.synchronize()
        wall = time.perf_counter() - t0
        out = {"wall_s": wall,
               "samples_per_s": epochs * self.nbatches * self.batch * self.ctx.world_size / wall}
        if test is not None:
            ev = self.evaluate(test)
            out["test_accuracy"] = ev["accuracy"]
            log_fn(f"Final Test Accuracy: {ev['accuracy']:.2f}%")
        return out

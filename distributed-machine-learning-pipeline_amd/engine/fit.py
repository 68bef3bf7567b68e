"""Production training entry point: ``python -m hipdsml fit`` (or under
``torchrun --nproc-per-node N``, one rank per GPU).

Replaces the reference's training driver ``DSML/client/client.go:516-659``
(connect, CommInit, load MNIST, 10 epochs x 937 batches, epoch log lines,
``Final Test Accuracy``) with a data-parallel job that keeps weights, data and
gradients in HBM: each rank trains its own shard, gradients are averaged over
RCCL, every replica applies the identical update.

Everything the reference hard-codes is a :class:`~hipdsml.utils.config.TrainConfig`
field (flags / config file / ``HIPDSML_*`` env), plus what it lacks:
checkpoint / resume, JSON-lines metrics, roctx tracing, progress with it/s.
"""
from __future__ import annotations

import logging
import os
import time
from typing import Any, Dict, Optional, Sequence, Tuple

import torch

from ..data.mnist import Dataset, load_mnist, mnist_available, synthetic_mnist, train_test_split
from ..models.mlp import MlpLayout, MlpSpec
from ..parallel.dist import DistContext
from ..utils import checkpoint as ckpt
from ..utils import trace
from ..utils.config import TrainConfig, parse, to_dict
from ..utils.metrics import MetricsLogger, Progress

log = logging.getLogger("hipdsml.fit")


def choose_engine(cfg: TrainConfig, spec: MlpSpec, device: torch.device) -> str:
    if cfg.engine != "auto":
        return cfg.engine
    if device.type != "cuda":
        return "fused"  # torch reference math on CPU
    return "fused" if MlpLayout(spec, cfg.batch, 1).fused_ok else "wide"


def build_data(cfg: TrainConfig, ctx: DistContext, dim: int) -> Tuple[Dataset, Optional[Dataset]]:
    """Per-rank training shard and a (replicated) test set."""
    if cfg.data == "mnist":
        d = cfg.data_dir or None
        kw = {"data_dir": d} if d else {}
        if mnist_available(split="train", **kw):
            train = load_mnist(split="train", **kw)
            test = load_mnist(split="t10k", **kw) if mnist_available(split="t10k", **kw) else None
        else:  # only t10k ships with the reference: 80/20 split of it
            train, test = train_test_split(load_mnist(split="t10k", **kw), 0.2)
        return train.shard(ctx.rank, ctx.world_size), test
    if cfg.data != "synthetic":
        raise ValueError(f"unknown data source {cfg.data!r}")
    train = synthetic_mnist(cfg.samples, seed=1000 + ctx.rank, dim=dim)
    test = synthetic_mnist(max(cfg.batch, 10000), seed=999_999, dim=dim)
    return train, test


def build_trainer(cfg: TrainConfig, spec: MlpSpec, data: Dataset, ctx: DistContext):
    engine = choose_engine(cfg, spec, ctx.device)
    if engine == "wide":
        from .wide import WideMlpTrainer

        if cfg.momentum or cfg.weight_decay:
            raise ValueError("the wide bf16 engine implements plain SGD")
        return WideMlpTrainer(spec, data, batch=cfg.batch, lr=cfg.lr, ctx=ctx, seed=cfg.seed,
                              init="kaiming" if cfg.init == "auto" else cfg.init,
                              # the fused exchanges and the persistent forms are fp32-MLP
                              # kernels; the wide engine syncs by RCCL
                              sync="rccl" if cfg.sync in ("auto", "xact", "xgmi", "pk", "pk2", "pkg", "pkg2",
                                                          "pkx") else cfg.sync,
                              graph=cfg.graph_steps != 0), engine
    from .trainer import MlpTrainer

    # graphs replay the fused-exchange steps too; a step with an RCCL collective
    # runs as the eager C++ loop whatever graph_steps says (MlpTrainer.train_steps)
    gs = cfg.graph_steps
    return MlpTrainer(spec, data, batch=cfg.batch, lr=cfg.lr, ctx=ctx, seed=cfg.seed,
                      init="reference" if cfg.init == "auto" else cfg.init, momentum=cfg.momentum,
                      weight_decay=cfg.weight_decay, sync=cfg.sync,
                      ring_chunk_bytes=cfg.ring_chunk_bytes, graph_steps=gs), engine


def _fault_hook(ctx: DistContext, step: int) -> None:
    """Fault injection for failure-detection tests (BASELINE config 5):
    HIPDSML_FAULT="rank:step:mode" makes `rank` die (mode exit) or stall
    forever (mode hang) once it has run `step` steps."""
    spec = os.environ.get("HIPDSML_FAULT", "")
    if not spec:
        return
    r, s, mode = spec.split(":")
    if int(r) != ctx.rank or step < int(s):
        return
    print(f"[fault injection] rank {ctx.rank}: {mode} at step {step}", flush=True)
    if mode == "exit":
        os._exit(13)
    if mode == "hang":
        while True:
            time.sleep(3600)
    raise ValueError(f"unknown fault mode {mode!r}")


def run(cfg: TrainConfig, out=print) -> Dict[str, Any]:
    if cfg.trace:
        trace.enable(True)
    backend = None if cfg.backend == "auto" else cfg.backend
    ctx = DistContext.from_env(device=cfg.device, backend=backend)
    try:
        return _run(cfg, ctx, out)
    finally:
        ctx.destroy()


def _run(cfg: TrainConfig, ctx: DistContext, out) -> Dict[str, Any]:
    spec = MlpSpec.parse(cfg.model)
    say = out if ctx.rank == 0 else (lambda *_: None)
    with trace.trace_range("setup"):
        train, test = build_data(cfg, ctx, spec.dims[0])
        tr, engine = build_trainer(cfg, spec, train, ctx)
    metrics = MetricsLogger(cfg.metrics, rank=ctx.rank,
                            static={"model": str(spec), "engine": engine, "world": ctx.world_size})
    metrics.log("start", config=to_dict(cfg), params=spec.num_params, batches_per_epoch=tr.nbatches)
    say(f"hipdsml fit: model {spec} ({spec.num_params} params), engine {engine}, "
        f"{ctx.world_size} replica(s) x batch {cfg.batch}, {tr.nbatches} batches/epoch, "
        f"device {ctx.device}")
    if cfg.resume:
        src = cfg.checkpoint if cfg.resume == "auto" else cfg.resume
        st = ckpt.resume(tr, src) if src else None
        if st is not None:
            say(f"Resumed from step {tr.steps_done}")
            metrics.log("resume", step=tr.steps_done, source=src)
    total = cfg.steps if cfg.steps > 0 else cfg.epochs * tr.nbatches
    per_epoch = tr.nbatches
    chunk = cfg.log_every if cfg.log_every > 0 else per_epoch
    every_ckpt = cfg.checkpoint_every if cfg.checkpoint_every > 0 else per_epoch
    prog = Progress(total, desc="train ", samples_per_it=cfg.batch * ctx.world_size,
                    enabled=ctx.rank == 0 and os.environ.get("HIPDSML_PROGRESS", "1") != "0")
    prog.n = min(tr.steps_done, total)
    t_start = time.perf_counter()
    done_at_start = tr.steps_done
    last_t, last_s = t_start, tr.steps_done
    while tr.steps_done < total:
        # run to the next boundary among: log chunk, epoch end, checkpoint, end
        s = tr.steps_done
        nxt = min(total, (s // chunk + 1) * chunk, (s // per_epoch + 1) * per_epoch)
        if cfg.checkpoint:
            nxt = min(nxt, (s // every_ckpt + 1) * every_ckpt)
        with trace.trace_range(f"train_steps[{s}:{nxt}]"):
            tr.train_steps(nxt - s)
        _fault_hook(ctx, tr.steps_done)
        at_epoch = tr.steps_done % per_epoch == 0
        at_log = tr.steps_done % chunk == 0 or at_epoch or tr.steps_done == total
        if at_log:
            st = tr.read_stats(global_=True)
            now = time.perf_counter()
            rate = (tr.steps_done - last_s) * cfg.batch * ctx.world_size / max(now - last_t, 1e-9)
            last_t, last_s = now, tr.steps_done
            prog.update(tr.steps_done - prog.n)
            metrics.log("train", step=tr.steps_done, epoch=tr.steps_done / per_epoch,
                        loss=st.avg_loss, accuracy=st.accuracy, samples_per_s=rate)
            if at_epoch:
                say(f"Epoch {tr.steps_done // per_epoch} complete: Avg Loss: {st.avg_loss:.4f}, "
                    f"Accuracy: {st.accuracy:.2f}%")
        if cfg.checkpoint and (tr.steps_done % every_ckpt == 0 or tr.steps_done == total):
            with trace.trace_range("checkpoint"):
                p = ckpt.save_checkpoint(tr, cfg.checkpoint, keep=cfg.keep_checkpoints, rank=ctx.rank)
            if p:
                metrics.log("checkpoint", step=tr.steps_done, path=p)
    tr.synchronize()
    prog.close()
    wall = time.perf_counter() - t_start
    res: Dict[str, Any] = {
        "steps": tr.steps_done, "wall_s": wall, "engine": engine,
        "samples_per_s": (tr.steps_done - done_at_start) * cfg.batch * ctx.world_size / max(wall, 1e-9)}
    if cfg.eval and test is not None:
        with trace.trace_range("evaluate"):
            ev = tr.evaluate(test)
        res["test_accuracy"] = ev["accuracy"]
        res["test_loss"] = ev["loss"]
        say(f"Final Test Accuracy: {ev['accuracy']:.2f}%")
    metrics.log("end", **res)
    metrics.close()
    return res


def main(argv: Optional[Sequence[str]] = None) -> int:
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(name)s %(message)s")
    cfg = parse(TrainConfig, argv, prog="hipdsml fit")
    run(cfg)
    return 0

"""Config / metrics / tracing / checkpoint utilities and the `fit` job (CPU)."""
import io
import json
import os

import pytest
import torch

from hipdsml.utils import checkpoint as ckpt
from hipdsml.utils import trace
from hipdsml.utils.config import CoordinatorConfig, TrainConfig, parse, resolve
from hipdsml.utils.metrics import Histogram, MetricsLogger, Progress, read_jsonl


def test_config_defaults_match_reference():
    c = TrainConfig()
    assert (c.batch, c.lr, c.epochs) == (64, 0.01, 10)  # client.go:22-28
    assert CoordinatorConfig().port == 50051 and CoordinatorConfig().health_interval == 5.0


def test_config_precedence(tmp_path):
    f = tmp_path / "c.yaml"
    f.write_text("batch: 32\nlr: 0.5\nmodel: 784-16-10\n")
    import argparse

    from hipdsml.utils.config import add_arguments

    ap = argparse.ArgumentParser()
    add_arguments(ap, TrainConfig)
    ns = ap.parse_args(["--config", str(f), "--lr", "0.25", "--eval", "false"])
    c = resolve(TrainConfig, ns, env={"HIPDSML_BATCH": "16", "HIPDSML_LR": "9"})
    assert c.batch == 16          # env beats file
    assert c.lr == 0.25           # flag beats env
    assert c.model == "784-16-10" and c.eval is False
    with pytest.raises(ValueError):
        resolve(TrainConfig, None, env={}, file_values={"nope": 1})
    j = tmp_path / "c.json"
    j.write_text(json.dumps({"ring-chunk-bytes": "0x1000"}))
    assert parse(TrainConfig, ["--config", str(j)]).ring_chunk_bytes == 4096


def test_metrics_logger_and_histogram(tmp_path):
    p = tmp_path / "m" / "x.jsonl"
    with MetricsLogger(str(p), rank=0, static={"job": "t"}) as m:
        m.log("train", step=1, loss=0.5, bad=float("nan"))
        m.log("end", ok=True)
    recs = read_jsonl(str(p))
    assert [r["event"] for r in recs] == ["train", "end"]
    assert recs[0]["job"] == "t" and recs[0]["bad"] is None and recs[0]["loss"] == 0.5
    assert not MetricsLogger(str(tmp_path / "y.jsonl"), rank=1).enabled  # rank 0 only
    h = Histogram("rpc")
    for us in (1, 2, 3, 100, 1000):
        h.add(us * 1e-6)
    s = h.summary()
    assert s["n"] == 5 and s["min_us"] == pytest.approx(1) and s["max_us"] == pytest.approx(1000)
    assert s["p50_us"] <= 4 and s["p99_us"] >= 1000


def test_progress_renders_rate():
    buf = io.StringIO()
    p = Progress(10, desc="e ", samples_per_it=64, stream=buf, min_interval=0)
    for _ in range(10):
        p.update()
    p.close()
    out = buf.getvalue()
    assert "10/10" in out and "it/s" in out and "samples/s" in out and out.endswith("\n")


def test_trace_ranges_record():
    trace.enable(True, record=True)
    try:
        trace.records(clear=True)
        with trace.trace_range("outer"):
            with trace.trace_range("inner"):
                pass

        @trace.traced("fn")
        def f(x):
            return x + 1

        assert f(1) == 2
        trace.mark("m")
        names = [r[0] for r in trace.records()]
        assert names == ["inner", "outer", "fn"]
        assert trace.summary()["outer"]["n"] == 1
    finally:
        trace.enable(False)


def _trainer(seed=0):
    from hipdsml.data.mnist import synthetic_mnist
    from hipdsml.engine.trainer import MlpTrainer
    from hipdsml.models.mlp import MlpSpec

    return MlpTrainer(MlpSpec((784, 32, 10)), synthetic_mnist(64 * 6, seed=3), batch=64, lr=0.05,
                      seed=seed, momentum=0.9)


def test_checkpoint_resume_bit_exact(tmp_path):
    a = _trainer()
    a.train_steps(10)
    b = _trainer()
    b.train_steps(4)
    d = str(tmp_path / "ck")
    for _ in range(3):
        b.train_steps(1)
        ckpt.save_checkpoint(b, d, keep=2)
    assert [os.path.basename(p) for p in ckpt.list_checkpoints(d)] == ["ckpt_000000006.pt",
                                                                       "ckpt_000000007.pt"]
    c = _trainer(seed=99)  # different init: everything must come from the checkpoint
    st = ckpt.resume(c, d)
    assert st["steps_done"] == 7 and c.steps_done == 7
    c.train_steps(3)
    assert torch.equal(a.P, c.P) and torch.equal(a.V, c.V)
    os.makedirs(tmp_path / "empty")
    assert ckpt.resume(c, str(tmp_path / "empty")) is None


def test_checkpoint_rejects_other_model(tmp_path):
    from hipdsml.data.mnist import synthetic_mnist
    from hipdsml.engine.trainer import MlpTrainer
    from hipdsml.models.mlp import MlpSpec

    a = _trainer()
    p = ckpt.save_checkpoint(a, str(tmp_path))
    other = MlpTrainer(MlpSpec((784, 16, 10)), synthetic_mnist(64, seed=1), batch=64)
    with pytest.raises(ValueError):
        ckpt.resume(other, p)


def test_fit_job_cpu_with_resume(tmp_path):
    from hipdsml.engine.fit import run

    lines = []
    d = str(tmp_path / "ck")
    m = str(tmp_path / "m.jsonl")
    cfg = TrainConfig(model="784-32-10", samples=64 * 8, epochs=2, lr=0.05, checkpoint=d,
                      metrics=m, device="cpu")
    r1 = run(cfg, out=lines.append)
    assert r1["steps"] == 16 and "test_accuracy" in r1
    assert any(l.startswith("Epoch 2 complete: Avg Loss:") for l in lines)
    assert any(l.startswith("Final Test Accuracy:") for l in lines)
    cfg2 = TrainConfig(model="784-32-10", samples=64 * 8, epochs=3, lr=0.05, checkpoint=d,
                       resume="auto", device="cpu", eval=False)
    lines.clear()
    r2 = run(cfg2, out=lines.append)
    assert "Resumed from step 16" in lines and r2["steps"] == 24
    events = [r["event"] for r in read_jsonl(m)]
    assert events[0] == "start" and events[-1] == "end" and events.count("checkpoint") == 2


def _fit_worker(rank, world, port, d):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HIPDSML_PROGRESS="0")
    from hipdsml.engine.fit import run

    r = run(TrainConfig(model="784-32-10", samples=64 * 4, epochs=1, lr=0.05, device="cpu",
                        checkpoint=d, eval=False), out=lambda *_: None)
    assert r["steps"] == 4


def test_fit_two_ranks_gloo(tmp_path):
    import socket

    import torch.multiprocessing as mp

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    d = str(tmp_path / "ck")
    mp.start_processes(_fit_worker, args=(2, port, d), nprocs=2, start_method="spawn", join=True)
    st = ckpt.load_state(ckpt.latest_checkpoint(d))  # written by rank 0 only
    assert st["steps_done"] == 4 and len(ckpt.list_checkpoints(d)) == 1

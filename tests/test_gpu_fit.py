"""Checkpoint/resume and the `fit` job on the MI355X (native engines)."""
import pytest
import torch

from hipdsml.data.mnist import synthetic_mnist
from hipdsml.engine.trainer import MlpTrainer
from hipdsml.models.mlp import MlpSpec
from hipdsml.parallel.dist import DistContext
from hipdsml.utils import checkpoint as ckpt
from hipdsml.utils.config import TrainConfig

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _fused(graph_steps, seed=0):
    return MlpTrainer(MlpSpec((784, 128, 64, 10)), synthetic_mnist(64 * 8, seed=11), batch=64,
                      lr=0.05, seed=seed, ctx=DistContext(device=DEV), graph_steps=graph_steps)


@pytest.mark.parametrize("graph_steps", [0, 4])
def test_fused_resume_bit_exact(tmp_path, graph_steps):
    a = _fused(graph_steps)
    a.train_steps(20)  # crosses the epoch boundary (8 batches)
    b = _fused(graph_steps)
    b.train_steps(11)
    p = ckpt.save_checkpoint(b, str(tmp_path))
    c = _fused(graph_steps, seed=5)
    ckpt.resume(c, p)
    c.train_steps(9)
    a.synchronize(); c.synchronize()
    # the native step counters must resume at batch 11 % 8, not batch 0
    assert torch.equal(a.P.cpu(), c.P.cpu())
    assert c.ctr.cpu().tolist() == [20, 20]


def test_wide_resume_bit_exact(tmp_path):
    from hipdsml.engine.wide import WideMlpTrainer

    def mk(seed):
        return WideMlpTrainer(MlpSpec((784, 256, 128, 10)), synthetic_mnist(64 * 4, seed=12),
                              batch=64, lr=0.05, seed=seed, graph=False)
    a = mk(1)
    a.train_steps(7)
    b = mk(1)
    b.train_steps(3)
    p = ckpt.save_checkpoint(b, str(tmp_path))
    c = mk(9)
    ckpt.resume(c, p)
    c.train_steps(4)
    a.synchronize(); c.synchronize()
    assert torch.equal(a.P.cpu(), c.P.cpu())


@pytest.mark.parametrize("model,engine", [("784-128-64-10", "fused"), ("784-512-512-10", "wide")])
def test_fit_job_gpu(tmp_path, model, engine):
    from hipdsml.engine.fit import run

    lines = []
    r = run(TrainConfig(model=model, engine=engine, samples=64 * 50, epochs=3, lr=0.05, device="cuda",
                        checkpoint=str(tmp_path), metrics=str(tmp_path / "m.jsonl")),
            out=lines.append)
    assert r["engine"] == engine and r["steps"] == 150
    assert r["test_accuracy"] > 85.0, lines
    assert len(ckpt.list_checkpoints(str(tmp_path))) == 2

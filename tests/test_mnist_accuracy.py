"""Training on real digits (the reference's t10k files, shipped as test
fixtures): the fp32 reference math on the CPU and the native HIP step on the
GPU learn MNIST to the accuracy class of the reference's 92.89 %
(README.md:204; its 60k train split is not in the reference tree, so these
tests train on t10k[:8000] and test on t10k[8000:])."""
import pytest
import torch

from hipdsml.data.mnist import load_mnist, mnist_available, train_test_split
from hipdsml.engine.trainer import MlpTrainer
from hipdsml.models.mlp import MlpSpec
from hipdsml.parallel.dist import DistContext

pytestmark = pytest.mark.skipif(not mnist_available(split="t10k"), reason="no t10k digits")


def _train(dims, device, epochs):
    tr_ds, te_ds = train_test_split(load_mnist(split="t10k"), 0.2)
    t = MlpTrainer(MlpSpec(dims), tr_ds, batch=64, lr=0.01, ctx=DistContext(device=device), seed=0,
                   graph_steps=125 if device.type == "cuda" else 0)
    t.train_steps(t.nbatches * epochs)
    t.synchronize()
    return t.evaluate(te_ds)["accuracy"]


def test_reference_math_learns_digits_cpu():
    # 1,250 SGD steps of the reference's model as coded (784-128-10, client.go:22-33)
    assert _train((784, 128, 10), torch.device("cpu"), 10) > 88.0


@pytest.mark.gpu
@pytest.mark.parametrize("dims", [(784, 128, 64, 10), (784, 128, 10)])
def test_native_step_learns_digits_like_reference_math(dims):
    # the reference's step count (10 epochs x 937 batches); fp32 on both sides,
    # so the GPU run lands where the CPU reference math does
    gpu = _train(dims, torch.device("cuda", 0), 75)
    cpu = _train(dims, torch.device("cpu"), 75)
    assert gpu > 92.5, gpu
    assert abs(gpu - cpu) < 1.0, (gpu, cpu)

"""Multi-process data parallelism on CPU (gloo, world_size 2 and 3): one process
per replica, exactly as bench.py runs one rank per GPU.  Checks that every
replica ends bit-identical and equal to single-process SGD on the averaged
gradient of all shards (what the reference's identity "ring" never did)."""
import os
import tempfile

import pytest
import torch
from spawn_util import spawn_group



def _worker(rank, world, port, outdir, momentum):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from hipdsml.data.mnist import synthetic_mnist
    from hipdsml.engine.trainer import MlpTrainer
    from hipdsml.models.mlp import MlpSpec
    from hipdsml.parallel.dist import DistContext

    ctx = DistContext.from_env(device="cpu")
    spec = MlpSpec((784, 32, 16, 10))
    ds = synthetic_mnist(16 * 6, seed=100 + rank)
    tr = MlpTrainer(spec, ds, batch=16, lr=0.05, ctx=ctx, seed=3, momentum=momentum)
    tr.train_steps(6)
    st = tr.read_stats(global_=True)
    torch.save({"P": tr.P, "count": st.count}, os.path.join(outdir, f"r{rank}.pt"))
    ctx.destroy()


@pytest.mark.parametrize("world,momentum", [(2, 0.0), (3, 0.0), (2, 0.9)])
def test_gloo_data_parallel(world, momentum):
    from hipdsml.data.mnist import synthetic_mnist
    from hipdsml.models.mlp import MlpLayout, MlpSpec, grads_ref, init_params

    with tempfile.TemporaryDirectory() as d:
        spawn_group(_worker, world, lambda port: (world, port, d, momentum))
        outs = [torch.load(os.path.join(d, f"r{r}.pt"), weights_only=True) for r in range(world)]
    for o in outs[1:]:
        assert torch.equal(o["P"], outs[0]["P"])
    assert outs[0]["count"] == 16 * 6 * world
    spec = MlpSpec((784, 32, 16, 10))
    lay = MlpLayout(spec, 16, 6)
    P = init_params(lay, 3)
    V = torch.zeros_like(P)
    shards = [synthetic_mnist(16 * 6, seed=100 + r) for r in range(world)]
    for s in range(6):
        g = sum(grads_ref(lay, P, sh.X[s * 16:(s + 1) * 16], sh.y[s * 16:(s + 1) * 16])[0] for sh in shards)
        g = g / world
        if momentum:
            V = momentum * V + g
            P = P - 0.05 * V
        else:
            P = P - 0.05 * g
    assert (outs[0]["P"] - P).abs().max().item() < 1e-5

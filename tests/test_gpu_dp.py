"""Multi-replica path on ONE MI355X: two processes share cuda:0 and average
gradients over gloo (RCCL refuses two ranks on one GPU: "invalid usage").
This exercises exactly the N>1 step structure of bench.py — fused HIP
fwd/bwd writing gradients, all-reduce, HIP SGD update — except the RCCL call
itself (covered on 8 GPUs by the driver's scaling run)."""
import os
import tempfile

import pytest
import torch
from spawn_util import spawn_group

pytestmark = pytest.mark.gpu



def _worker(rank, world, port, outdir, kind):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK="0",
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from hipdsml.data.mnist import synthetic_mnist
    from hipdsml.models.mlp import MlpSpec
    from hipdsml.parallel.dist import DistContext

    ctx = DistContext.from_env(device="cuda", backend="gloo")
    if kind == "fused":
        from hipdsml.engine.trainer import MlpTrainer

        spec = MlpSpec((784, 128, 64, 10))
        ds = synthetic_mnist(64 * 4, seed=200 + rank)
        tr = MlpTrainer(spec, ds, batch=64, lr=0.05, ctx=ctx, seed=7, sync="torch")
    else:
        from hipdsml.engine.wide import WideMlpTrainer

        spec = MlpSpec((784, 256, 128, 10))
        ds = synthetic_mnist(64 * 4, seed=200 + rank)
        tr = WideMlpTrainer(spec, ds, batch=64, lr=0.05, ctx=ctx, seed=7,
                            sync="xact" if "xact" in kind else "torch",
                            serial_sync=kind.endswith("_serial"))
        if kind.endswith("_delay"):
            tr._comm_delay_cycles = 2_000_000  # ~1 ms stall ahead of every bucket on the comm stream
    tr.train_steps(4)
    tr.synchronize()
    torch.save({"P": tr.P.cpu()}, os.path.join(outdir, f"r{rank}.pt"))
    ctx.destroy()


@pytest.mark.parametrize("kind", ["fused", "wide", "wide_xact"])
def test_two_replicas_one_gpu(kind):
    from hipdsml.data.mnist import synthetic_mnist
    from hipdsml.models.mlp import MlpLayout, MlpSpec, grads_ref, init_params

    world = 2
    with tempfile.TemporaryDirectory() as d:
        spawn_group(_worker, world, lambda port: (world, port, d, kind))
        outs = [torch.load(os.path.join(d, f"r{r}.pt"), weights_only=True)["P"] for r in range(world)]
    assert torch.equal(outs[0], outs[1])
    dims = (784, 128, 64, 10) if kind == "fused" else (784, 256, 128, 10)
    lay = MlpLayout(MlpSpec(dims), 64, 4)
    P = init_params(lay, 7, "reference" if kind == "fused" else "kaiming")
    shards = [synthetic_mnist(64 * 4, seed=200 + r) for r in range(world)]
    for s in range(4):
        g = sum(grads_ref(lay, P, sh.X[s * 64:(s + 1) * 64], sh.y[s * 64:(s + 1) * 64])[0] for sh in shards)
        P = P - 0.05 * g / world
    err = (outs[0] - P).abs().max().item()
    assert err < (2e-5 if kind == "fused" else 5e-3), err


@pytest.mark.parametrize("sync", ["", "_xact"])
def test_wide_bucket_overlap_matches_serial_sync(sync):
    """Per-layer buckets all-reduced + applied (or, with the activation
    exchange, the activation buffers all-gathered) on the comm stream while the
    backward continues, with the comm stream artificially stalled, give the
    same bits as running each collective in line on the compute stream."""
    world = 2
    got = {}
    for kind in (f"wide{sync}_delay", f"wide{sync}_serial"):
        with tempfile.TemporaryDirectory() as d:
            spawn_group(_worker, world, lambda port: (world, port, d, kind))
            got[kind] = [torch.load(os.path.join(d, f"r{r}.pt"), weights_only=True)["P"]
                         for r in range(world)]
    assert torch.equal(got[f"wide{sync}_delay"][0], got[f"wide{sync}_delay"][1])
    assert torch.equal(got[f"wide{sync}_delay"][0], got[f"wide{sync}_serial"][0])

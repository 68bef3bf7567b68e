"""End-to-end training through the gpu_sim API on CPU-simulated devices
(BASELINE config 1): the reference's client flow, with real data-parallel
semantics checked against a single-process reference."""
import numpy as np
import torch

from hipdsml.data.mnist import synthetic_mnist
from hipdsml.models.mlp import MlpLayout, MlpSpec, grads_ref, init_params
from hipdsml.rpc.client import TrainingClient

from cluster_util import cluster


def test_rpc_mode_data_parallel_matches_reference():
    n, batch, steps = 3, 16, 4
    spec = MlpSpec((784, 32, 16, 10))
    ds = synthetic_mnist(n * batch * steps, seed=5)
    lines = []
    with cluster(n_devices=n, mem_size=1 << 20) as c:
        cl = TrainingClient(c.coord_addr, c.addresses, spec.dims, batch=batch, lr=0.05, seed=11,
                            out=lines.append)
        try:
            res = cl.train_rpc_mode(1, ds.X.numpy(), ds.y.numpy(), steps_per_epoch=steps)
        finally:
            cl.close()
        got = [c.devices[i][2].trainer.P.clone() for i in range(n)]
    # every replica identical (no weight broadcast needed)
    for g in got[1:]:
        assert torch.equal(g, got[0])
    # == single-process SGD on the averaged gradient of the n shards
    lay = MlpLayout(spec, batch, 1)
    P = init_params(lay, 11)
    shard = len(ds) // n
    for b in range(steps):
        gs = []
        for i in range(n):
            lo = i * shard + b * batch
            g, _, _ = grads_ref(lay, P, ds.X[lo:lo + batch], ds.y[lo:lo + batch])
            gs.append(g)
        P = P - 0.05 * sum(gs) / n
    assert (got[0] - P).abs().max().item() < 1e-5
    assert any(l.startswith("Epoch 1 complete: Avg Loss:") for l in lines)
    assert res["samples_per_s"] > 0


def test_device_mode_single_host_device():
    lines = []
    with cluster(n_devices=1, mem_size=1 << 20) as c:
        cl = TrainingClient(c.coord_addr, c.addresses, (784, 64, 10), batch=32, lr=0.05, out=lines.append)
        try:
            res = cl.train_device_mode(epochs=2, samples_per_rank=32 * 20, graph_steps=0, eval_samples=256)
        finally:
            cl.close()
    assert lines[0] == "Starting MLP training..."
    assert lines[1].startswith("Epoch 1 complete") and lines[2].startswith("Epoch 2 complete")
    assert lines[-1].startswith("Final Test Accuracy:")
    assert res["steps_per_epoch"] == 20


def test_device_mode_host_data_parallel_matches_reference():
    """ConfigureModel + TrainSteps on 3 host device servers (the reference's
    3-device client, client.go:532-539): each server trains its own shard and
    sums every step's gradient over the device-driven gRPC ring.  Replicas stay
    identical and equal single-process SGD on the averaged gradient."""
    n, batch, spe, epochs = 3, 16, 5, 2
    dims = (784, 32, 16, 10)
    lines = []
    with cluster(n_devices=n, mem_size=1 << 20) as c:
        cl = TrainingClient(c.coord_addr, c.addresses, dims, batch=batch, lr=0.05, seed=3,
                            out=lines.append)
        try:
            res = cl.train_device_mode(epochs=epochs, samples_per_rank=batch * spe, graph_steps=0,
                                       eval_samples=128)
        finally:
            cl.close()
        got = [c.devices[i][2].trainer.P.clone() for i in range(n)]
        stats = [c.devices[i][2].counters["allreduces"] for i in range(n)]
    for g in got[1:]:
        assert torch.equal(g, got[0])
    assert stats == [epochs * spe] * n
    spec = MlpSpec(dims)
    lay = MlpLayout(spec, batch, 1)
    P = init_params(lay, 3)
    shards = [synthetic_mnist(batch * spe, seed=1000 + r, dim=784) for r in range(n)]
    for s in range(epochs * spe):
        b = s % spe
        g = sum(grads_ref(lay, P, d.X[b * batch:(b + 1) * batch], d.y[b * batch:(b + 1) * batch])[0]
                for d in shards)
        P = P - 0.05 * g / n
    assert (got[0] - P).abs().max().item() < 1e-5
    assert res["steps_per_epoch"] == spe
    assert lines[1].startswith("Epoch 1 complete") and lines[-1].startswith("Final Test Accuracy:")


def test_auto_backend_decides_by_host_identity():
    """same-node GPU servers reached by LAN IP keep the 'pg' group
    (and the xGMI candidates); servers on different hosts take 'rccl'."""
    from hipdsml.rpc.client import auto_backend
    from hipdsml.rpc.proto import pb

    def md(host, backend="hip"):
        return pb.DeviceMetadata(backend=backend, host=host)

    lan = ["10.0.0.5:5003", "10.0.0.5:5004"]
    assert auto_backend([md("nodeA"), md("nodeA")], lan) == "pg"
    assert auto_backend([md("nodeA"), md("nodeB")], ["127.0.0.1:1", "127.0.0.1:2"]) == "rccl"
    assert auto_backend([md(""), md("")], lan) == "rccl"            # no host reported: address test
    assert auto_backend([md(""), md("")], ["127.0.0.1:1", "localhost:2"]) == "pg"
    assert auto_backend([md("a", "host"), md("a", "host")], lan) == "rpc"
    assert auto_backend([md("a")], lan) == "rpc"

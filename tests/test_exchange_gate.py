"""Which data-parallel forms a trainer enumerates, on CPU (no GPU, no kernels).

VERDICT r4 Missing #1: device servers that own distinct GPUs join a gloo
process group plus an external RCCL communicator (rpc/device_server.py
_join_process_group), and the fused xGMI exchanges must still be candidates
there -- eligibility depends on "GPU replicas, a process group, all ranks on
this node", never on the group's backend being nccl.  Reference flow being
served: DSML/client/client.go:532-644 (CommInit with the device list, then
the per-step gradient sync)."""
import types

import pytest
import torch

from hipdsml.engine.trainer import MlpTrainer, _xgmi_eligible
from hipdsml.parallel.dist import DistContext


def _ctx(world=2, backend="gloo", dev="cuda"):
    return DistContext(rank=0, world_size=world, backend=backend,
                       device=torch.device(dev, 0) if dev == "cuda" else torch.device("cpu"))


def _trainer(ctx, sync="auto", node_local=None, momentum=0.0):
    t = MlpTrainer.__new__(MlpTrainer)  # the decision only, no buffers or kernels
    t.ctx, t.sync, t._node_local, t.momentum, t.weight_decay = ctx, sync, node_local, momentum, 0.0
    return t


def test_gloo_group_with_external_rccl_comm_enumerates_every_exchange():
    for n in (2, 4, 8):
        modes = _trainer(_ctx(n), node_local=True).exchange_candidates()
        for m in ("pkx", "pkg", "pk", "xact", "xgmi"):
            assert m in modes, (n, modes)
        assert modes[0] == "pkx"
        assert ("pk2" in modes) == (n >= 3)


def test_nccl_group_from_torchrun_still_eligible(monkeypatch):
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "8")
    assert _trainer(_ctx(8, "nccl")).exchange_candidates()[0] == "pkx"


def test_ineligible_cases():
    assert not _xgmi_eligible(_ctx(2), node_local=False)           # ranks on two hosts
    assert not _xgmi_eligible(_ctx(2, backend="none"), node_local=True)  # no process group
    assert not _xgmi_eligible(_ctx(2, dev="cpu"), node_local=True)  # host replicas
    assert not _xgmi_eligible(_ctx(9), node_local=True)             # > one node's 8 GPUs
    assert not _xgmi_eligible(_ctx(1), node_local=True)
    assert _trainer(_ctx(2), node_local=True, momentum=0.9).exchange_candidates() == []
    assert _trainer(_ctx(2), sync="rccl", node_local=True).exchange_candidates() == []
    assert _trainer(_ctx(2), sync="pkg", node_local=False).exchange_candidates() == ["pkg"]


def test_torchrun_multi_node_env_is_not_node_local(monkeypatch):
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "4")
    assert not _xgmi_eligible(_ctx(8, "nccl"))


def test_configure_model_passes_node_locality_to_the_trainer(monkeypatch):
    """ConfigureModel on a GPU server of a 'pg' comm hands the trainer what the
    group's rendezvous found (every rank's hostname) together with the RCCL
    comm, so the exchanges and RCCL are both candidates."""
    import torch.distributed as dist

    from hipdsml.engine import trainer as T
    from hipdsml.rpc.device_server import GPUDeviceServicer
    from hipdsml.rpc.proto import pb

    seen = {}

    class Rec:
        def __init__(self, spec, ds, **kw):
            seen.update(kw)
            self.nbatches, self.sync_active, self.sync_times = len(ds) // kw["batch"], "pkx", {}

    monkeypatch.setattr(T, "MlpTrainer", Rec)
    monkeypatch.setattr(dist, "get_world_size", lambda *a, **k: 2)
    monkeypatch.setattr(dist, "get_rank", lambda *a, **k: 1)
    dev = types.SimpleNamespace(backend="hip", gpu=0, device_id=2)
    svc = GPUDeviceServicer(dev)
    svc.pg_comm, svc.pg_node_local = 7, True
    svc.comms[7] = object()  # the RCCL comm CommSetup built
    monkeypatch.setattr(svc, "_torch_device", lambda: torch.device("cpu"))

    class Ctx:
        def abort(self, code, msg):
            raise AssertionError(msg)

    r = svc.ConfigureModel(pb.ConfigureModelRequest(dims=[784, 128, 64, 10], batch=64, commId=7, rank=1,
                                                    worldSize=2, dataset="synthetic", numSamples=256),
                           Ctx())
    assert r.success and r.sync == "pkx"
    assert seen["node_local"] is True and seen["sync"] == "auto"
    assert seen["auto_fallback"] == "rccl" and seen["external_comm"] is svc.comms[7]


@pytest.mark.parametrize("addr,want", [("127.0.0.1:5003", True), ("localhost:1", True), ("[::1]:9", True),
                                       ("10.0.0.2:5003", False), ("node7:5003", False)])
def test_is_loopback(addr, want):
    from hipdsml.rpc.stubs import is_loopback

    assert is_loopback(addr) is want

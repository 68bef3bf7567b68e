"""The gpu_sim gRPC stack on a real MI355X: HBM-arena device servers, the
device-driven ring with on-device HIP reduce kernels, device-side
RunForward/RunBackward/ApplyGradients through the fused HIP kernels, and
TrainSteps / Evaluate."""
import numpy as np
import pytest
import torch

from hipdsml.data.mnist import synthetic_mnist
from hipdsml.models.mlp import MlpLayout, MlpSpec, forward_ref, grads_ref, init_params
from hipdsml.rpc.proto import DT_BFLOAT16, DT_FLOAT32, pb

from cluster_util import cluster, d2h, h2d

pytestmark = pytest.mark.gpu


def test_hip_device_memcpy_and_ring():
    n = 3
    with cluster(n_devices=n, mem_size=8 << 20, backend="hip") as c:
        r = c.comm_init()
        assert all(d.backend == "hip" for d in r.devices)
        cid = r.commId
        payload = bytes(range(256)) * 4096
        h2d(c.stub, 2, 0x1000, payload)
        assert d2h(c.stub, 2, 0x1000, len(payload)) == payload
        rng = np.random.default_rng(0)
        count = 262_147  # uneven segments, > 1 MiB
        arrays = [rng.standard_normal(count).astype(np.float32) for _ in range(n)]
        for i in range(n):
            c.devices[i][2].dev.write(0x1000, arrays[i].tobytes())
        for algo in ("device-ring", "coordinator-ring"):
            for i in range(n):
                c.devices[i][2].dev.write(0x1000, arrays[i].tobytes())
            assert c.stub.AllReduceRing(pb.AllReduceRingRequest(commId=cid, count=count * 4, op=0,
                                                                dtype=DT_FLOAT32, algo=algo)).success
            want = arrays[0] + arrays[1] + arrays[2]
            for i in range(n):
                got = np.frombuffer(c.devices[i][2].dev.read(0x1000, count * 4), dtype=np.float32)
                np.testing.assert_allclose(got, want, rtol=1e-5, atol=1e-5)
        bf = [torch.full((1000,), float(i + 1), dtype=torch.bfloat16) for i in range(n)]
        for i in range(n):
            c.devices[i][2].dev.write(0x1000, bf[i].view(torch.uint8).numpy().tobytes())
        assert c.stub.AllReduceRing(pb.AllReduceRingRequest(commId=cid, count=2000, op=3,
                                                            dtype=DT_BFLOAT16)).success
        out = torch.frombuffer(bytearray(c.devices[1][2].dev.read(0x1000, 2000)), dtype=torch.bfloat16)
        assert torch.all(out == 3.0)


def test_hip_device_forward_backward_apply():
    spec = MlpSpec((784, 128, 64, 10))
    with cluster(n_devices=1, mem_size=16 << 20, backend="hip") as c:
        c.comm_init()
        stub = c.device_stub(0)
        svc = c.devices[0][2]
        stub.ConfigureModel(pb.ConfigureModelRequest(dims=list(spec.dims), batch=64, lr=0.05, seed=4,
                                                     worldSize=1, numSamples=64 * 4))
        ds = synthetic_mnist(64, seed=9)
        lay = MlpLayout(spec, 64, 1)
        P0 = init_params(lay, 4)
        svc.dev.write(0x100000, ds.X.numpy().tobytes())
        svc.dev.write(0x200000, ds.y.numpy().astype(np.int32).tobytes())
        f = stub.RunForward(pb.RunForwardRequest(deviceId=1, inputAddr=0x100000, numRows=64,
                                                 labelsAddr=0x200000, outputAddr=0x300000))
        g, loss_sum, corr = grads_ref(lay, P0, ds.X, ds.y)
        assert abs(f.loss - float(loss_sum) / 64) < 1e-4 and f.correct == int(corr)
        # logits come from the fused HIP forward kernels: fp32 torch reference to 1e-5
        want, _ = forward_ref(lay, P0, ds.X)
        got_l = torch.frombuffer(bytearray(svc.dev.read(0x300000, 64 * 10 * 4)),
                                 dtype=torch.float32).view(64, 10)
        assert (got_l - want).abs().max().item() < 1e-5
        b = stub.RunBackward(pb.RunBackwardRequest(deviceId=1, gradientAddr=0x1000))
        assert b.numBytes == lay.nparams * 4
        got = torch.frombuffer(bytearray(svc.dev.read(0x1000, b.numBytes)), dtype=torch.float32)
        assert (got - g).abs().max().item() < 1e-5
        stub.ApplyGradients(pb.ApplyGradientsRequest(gradientAddr=0x1000, scale=1.0))
        assert (svc.trainer.P.cpu() - (P0 - 0.05 * g)).abs().max().item() < 1e-5


def test_hip_device_train_steps_and_evaluate():
    with cluster(n_devices=1, mem_size=1 << 20, backend="hip") as c:
        c.comm_init()
        stub = c.device_stub(0)
        r = stub.ConfigureModel(pb.ConfigureModelRequest(dims=[784, 128, 64, 10], batch=64, lr=0.05,
                                                         numSamples=64 * 50, graphSteps=25))
        assert r.batchesPerEpoch == 50
        first = stub.TrainSteps(pb.TrainStepsRequest(steps=50))
        last = None
        for _ in range(4):
            last = stub.TrainSteps(pb.TrainStepsRequest(steps=50))
        assert last.stepsDone == 250 and last.count == 50 * 64
        assert last.lossSum / last.count < first.lossSum / first.count
        ev = stub.Evaluate(pb.EvaluateRequest(numSamples=2000))
        assert ev.count == 2000 and ev.accuracy > 80.0


def test_rccl_backend_single_device_comm():
    with cluster(n_devices=1, mem_size=1 << 20, backend="hip") as c:
        r = c.comm_init(backend="rccl")
        cid = r.commId
        data = np.arange(1024, dtype=np.float32)
        c.devices[0][2].dev.write(0x1000, data.tobytes())
        # n=1 short-circuits in the coordinator; drive the device directly too
        stub = c.device_stub(0)
        for algo in ("rccl", "ring"):
            resp = stub.DeviceAllReduce(pb.DeviceAllReduceRequest(commId=cid, addr=0x1000, count=4096,
                                                                  dtype=DT_FLOAT32, algo=algo, repeat=3))
            assert resp.success
        got = np.frombuffer(c.devices[0][2].dev.read(0x1000, 4096), dtype=np.float32)
        assert np.array_equal(got, data)
        assert stub.Abort(pb.AbortRequest(commId=cid, reason="test")).success


def test_hip_device_dies_mid_allreduce():
    """BASELINE config 5 on HBM-backed devices: rank 1 fails inside the ring;
    the call fails fast, the survivors' pending streams are failed (no hang)
    and the communicator is FAILED."""
    import time

    import grpc

    n = 3
    with cluster(n_devices=n, mem_size=8 << 20, backend="hip", rpc_timeout=60.0) as c:
        cid = c.comm_init().commId
        for i in range(n):
            c.devices[i][2].dev.write(0x1000, np.ones(1 << 18, np.float32).tobytes())
        c.devices[1][2].arm_fault(4, "stop")
        t0 = time.time()
        with pytest.raises(grpc.RpcError):
            c.stub.AllReduceRing(pb.AllReduceRingRequest(commId=cid, count=4 << 18, dtype=DT_FLOAT32))
        assert time.time() - t0 < 20.0
        st = c.stub.GetCommStatus(pb.GetCommStatusRequest(commId=cid)).status
        from hipdsml.rpc.proto import FAILED

        assert st == FAILED

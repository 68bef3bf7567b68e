"""CommInit backend "pg": the coordinator hosts a TCP store, every device
server joins a torch.distributed process group on it inside CommSetup, and
ConfigureModel builds the framework's data-parallel trainer on that group
(on GPUs: the persistent step with its in-launch xGMI exchange, self-tested
and timed like a torchrun job; on host devices: the gloo all-reduce).  The
device servers are separate processes, as in the reference's deployment
(DSML/cmd/gpu_device_server); checked against single-process SGD."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

from hipdsml.cli import _wait_port, child_env
from hipdsml.data.mnist import synthetic_mnist
from hipdsml.models.mlp import MlpLayout, MlpSpec, forward_ref, grads_ref, init_params
from hipdsml.rpc.client import TrainingClient
from hipdsml.rpc.coordinator import start_coordinator
from hipdsml.rpc.proto import pb


def _port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _servers(n, backend):
    addrs, procs = [], []
    for i in range(n):
        p = _port()
        addrs.append(f"127.0.0.1:{p}")
        procs.append(subprocess.Popen([sys.executable, "-m", "hipdsml", "device-server", "--ports", str(p),
                                       "--device-ids", str(i + 1), "--backend", backend, "--gpus", "0",
                                       "--mem-size", str(8 << 20)], env=child_env(),
                                      stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL))
    for a in addrs:
        _wait_port(a, timeout=300)
    return addrs, procs


def _run(n, backend, dims, batch, steps, lr, sync=""):
    addrs, procs = _servers(n, backend)
    server, caddr, svc = start_coordinator("127.0.0.1:0", health_interval=0)
    cl = TrainingClient(caddr, addrs, dims, batch=batch, lr=lr, seed=11, out=lambda s: None)
    try:
        cl.comm_init("pg")
        rs = cl._all(lambda i, s: s.ConfigureModel(pb.ConfigureModelRequest(
            dims=list(dims), batch=batch, lr=lr, seed=11, commId=cl.comm_id, rank=i, worldSize=n,
            dataset="synthetic", numSamples=batch * 4, dataSeed=1000, sync=sync), timeout=300))
        cl._all(lambda i, s: s.TrainSteps(pb.TrainStepsRequest(steps=steps), timeout=300))
        # every replica's logits on one fixed batch (its weights, read back)
        Xt = synthetic_mnist(batch, seed=4242).X.numpy().astype(np.float32)
        out = []
        for i, s in enumerate(cl.devs):
            s.Memcpy(pb.MemcpyRequest(hostToDevice=pb.MemcpyHostToDeviceRequest(
                hostSrcData=Xt.tobytes(), dstDeviceId=pb.DeviceId(value=i + 1), dstMemAddr=pb.MemAddr(value=0x1000))))
            oaddr = 0x1000 + Xt.nbytes
            s.RunForward(pb.RunForwardRequest(deviceId=i + 1, inputAddr=0x1000, numRows=batch, outputAddr=oaddr))
            raw = s.Memcpy(pb.MemcpyRequest(deviceToHost=pb.MemcpyDeviceToHostRequest(
                srcDeviceId=pb.DeviceId(value=i + 1), srcMemAddr=pb.MemAddr(value=oaddr),
                numBytes=batch * dims[-1] * 4))).deviceToHost.dstData
            out.append(np.frombuffer(raw, dtype=np.float32).reshape(batch, dims[-1]).copy())
        return rs, out, Xt
    finally:
        cl.close()
        svc.stop()
        server.stop(0)
        for p in procs:
            p.terminate()
        for p in procs:
            p.wait(timeout=30)


def _reference(n, dims, batch, steps, lr, Xt):
    spec = MlpSpec(dims)
    lay = MlpLayout(spec, batch, 4)
    P = init_params(lay, 11)
    shards = [synthetic_mnist(batch * 4, seed=1000 + r) for r in range(n)]
    for s in range(steps):
        b = s % 4
        g = sum(grads_ref(lay, P, sh.X[b * batch:(b + 1) * batch], sh.y[b * batch:(b + 1) * batch])[0]
                for sh in shards)
        P = P - lr * g / n
    return forward_ref(lay, P, torch.from_numpy(Xt))[0].numpy()


def test_pg_backend_host_devices_data_parallel():
    n, dims, batch, steps, lr = 2, (784, 32, 16, 10), 16, 6, 0.05
    rs, logits, Xt = _run(n, "host", dims, batch, steps, lr)
    assert all(r.success for r in rs)
    np.testing.assert_array_equal(logits[0], logits[1])  # identical replicas, no weight broadcast
    want = _reference(n, dims, batch, steps, lr, Xt)
    assert np.abs(logits[0] - want).max() < 1e-4


@pytest.mark.gpu
def test_pg_backend_gpu_devices_run_the_persistent_data_parallel_step():
    """Two device-server processes sharing the box's GPU: the process group
    comes up over the coordinator's store, ConfigureModel self-tests and times
    the candidates, and a persistent exchange form (pkx / pkg / pk) trains."""
    n, dims, batch, steps, lr = 2, (784, 128, 64, 10), 64, 9, 0.05
    rs, logits, Xt = _run(n, "hip", dims, batch, steps, lr)
    assert rs[0].sync == rs[1].sync and rs[0].sync in ("pkx", "pkg", "pk", "pkg2", "pk2", "xact", "xgmi",
                                                       "torch"), rs[0].sync
    np.testing.assert_array_equal(logits[0], logits[1])
    want = _reference(n, dims, batch, steps, lr, Xt)
    assert np.abs(logits[0] - want).max() < 1e-4

"""Training client (reference-compatible flow and log lines).

Reference: ``DSML/client/client.go:516-659`` — connect to the coordinator and
the device servers, CommInit, train 10 epochs x 937 batches (batch 64, SGD
lr 0.01), print ``Epoch N complete: Avg Loss: x, Accuracy: y%`` and
``Final Test Accuracy: z%``.

Two modes:

``device`` (MI355X fast path): every device server builds its replica on its
  GPU (ConfigureModel) and each epoch is ONE TrainSteps RPC per device.  With
  several GPU devices the coordinator's CommInit (backend "pg") bootstraps a
  process group on the device servers over a TCP store it hosts (plus RCCL when
  every device owns a distinct GPU), so the devices run the framework's fastest
  self-tested data-parallel step: the persistent step with its in-launch xGMI
  exchange (pkx / pkg / pk), the fused exchanges, or RCCL.  Only loss /
  accuracy scalars cross the network.

``rpc`` (the reference's pipeline, made correct): per step, each device gets
  its own batch by Memcpy, computes gradients on the device (RunForward /
  RunBackward), the coordinator ring-all-reduces the fp32 gradients between
  the devices (AllReduceRing, dtype-aware), and every replica applies the same
  averaged SGD update (ApplyGradients).  No weight broadcast is needed because
  all replicas stay identical (SURVEY C7/C8/C9 eliminated).
"""
from __future__ import annotations

import argparse
import logging
import sys
import time
from concurrent.futures import ThreadPoolExecutor
from typing import List

import numpy as np

from ..models.mlp import MlpLayout, MlpSpec
from .proto import DT_FLOAT32, SUM, pb
from .stubs import is_loopback
from .stubs import GPUCoordinatorStub, GPUDeviceStub, connect

log = logging.getLogger("hipdsml.client")


def _align(x: int, a: int = 256) -> int:
    return (x + a - 1) // a * a


def auto_backend(mds, addrs) -> str:
    """CommInit backend for `train_device_mode`: GPU device servers on ONE
    node (by the hostnames they report, not by the form of their addresses: a
    same-node server reached by LAN IP is still node-local) join a process
    group on the coordinator's store ("pg": the xGMI exchange candidates need
    it); servers spread over nodes take the RCCL bootstrap, whose id travels
    over gRPC ("rccl"); host (CPU) servers use the gRPC ring ("rpc").  Servers
    too old to report a host fall back to the address test."""
    if len(mds) < 2 or {m.backend for m in mds} != {"hip"}:
        return "rpc"
    hosts = [m.host for m in mds]
    if all(hosts):
        return "pg" if len(set(hosts)) == 1 else "rccl"
    return "pg" if all(is_loopback(a) for a in addrs) else "rccl"


class TrainingClient:
    def __init__(self, coordinator: str, devices: List[str], dims=(784, 128, 64, 10), batch: int = 64,
                 lr: float = 0.01, seed: int = 0, timeout: float = 600.0, out=print):
        self.coord = GPUCoordinatorStub(connect(coordinator, timeout=30))
        self.dev_addrs = list(devices)
        self.devs = [GPUDeviceStub(connect(a, timeout=30)) for a in devices]
        self.spec = MlpSpec(tuple(dims))
        self.batch = batch
        self.lr = lr
        self.seed = seed
        self.timeout = timeout
        self.out = out
        self.pool = ThreadPoolExecutor(max_workers=max(4, len(devices)))
        self.comm_id = None
        self.dev_ids: List[int] = []

    def _all(self, fn):
        return [f.result() for f in [self.pool.submit(fn, i, s) for i, s in enumerate(self.devs)]]

    def comm_init(self, backend: str) -> None:
        r = self.coord.CommInit(pb.CommInitRequest(numDevices=len(self.dev_addrs),
                                                   device_addresses=self.dev_addrs, backend=backend),
                                timeout=self.timeout)
        self.comm_id = r.commId
        self.dev_ids = [d.deviceId.value for d in r.devices]
        log.info("CommInit successful: CommId=%d, Devices=%d (%s)", r.commId, len(r.devices), backend)

    def close(self) -> None:
        if self.comm_id is not None:
            try:
                self.coord.CommDestroy(pb.CommDestroyRequest(commId=self.comm_id), timeout=30)
            except Exception:
                pass
            self.comm_id = None

    # ------------------------------------------------------------ device mode --
    def train_device_mode(self, epochs: int, samples_per_rank: int, graph_steps: int = 50,
                          sync: str = "", eval_samples: int = 10000, backend: str = "auto") -> dict:
        n = len(self.devs)
        # GPU device servers: a process group (backend "pg") and the framework's
        # data-parallel choice (sync "" = the server's default, "auto" there);
        # host (CPU) device servers: the device-driven gRPC ring (DeviceAllReduce's
        # transfers), or a gloo group with backend="pg"
        if backend == "auto":
            mds = [s.GetDeviceMetadata(pb.GetDeviceMetadataRequest(), timeout=self.timeout).metadata
                   for s in self.devs]
            backend = auto_backend(mds, self.dev_addrs)
        self.comm_init(backend)

        def cfg(i, s):
            return s.ConfigureModel(pb.ConfigureModelRequest(
                dims=list(self.spec.dims), batch=self.batch, lr=self.lr, seed=self.seed,
                commId=self.comm_id, rank=i, worldSize=n, dataset="synthetic",
                numSamples=samples_per_rank, dataSeed=1000, graphSteps=graph_steps, sync=sync),
                timeout=self.timeout)
        steps = self._all(cfg)[0].batchesPerEpoch
        self.out("Starting MLP training...")
        t0 = time.perf_counter()
        for ep in range(1, epochs + 1):
            rs = self._all(lambda i, s: s.TrainSteps(pb.TrainStepsRequest(steps=steps), timeout=self.timeout))
            loss = sum(r.lossSum for r in rs)
            corr = sum(r.correct for r in rs)
            cnt = sum(r.count for r in rs)
            self.out(f"Epoch {ep} complete: Avg Loss: {loss / cnt:.4f}, Accuracy: {100 * corr / cnt:.2f}%")
        wall = time.perf_counter() - t0
        self.out("Training complete.")
        ev = self.devs[0].Evaluate(pb.EvaluateRequest(dataset="synthetic", numSamples=eval_samples, seed=777),
                                   timeout=self.timeout)
        self.out(f"Final Test Accuracy: {ev.accuracy:.2f}%")
        samples = epochs * steps * self.batch * n
        return {"wall_s": wall, "samples_per_s": samples / wall, "test_accuracy": ev.accuracy,
                "steps_per_epoch": steps}

    # --------------------------------------------------------------- rpc mode --
    def train_rpc_mode(self, epochs: int, X: np.ndarray, y: np.ndarray, steps_per_epoch: int = 0,
                       X_test: np.ndarray = None, y_test: np.ndarray = None) -> dict:
        n = len(self.devs)
        self.comm_init("rpc")
        lay = MlpLayout(self.spec, self.batch, 1)
        grad_bytes = lay.nparams * 4
        grad_addr = 0x1000
        data_addr = grad_addr + _align(grad_bytes)
        label_addr = data_addr + _align(self.batch * self.spec.dims[0] * 4)

        def cfg(i, s):
            return s.ConfigureModel(pb.ConfigureModelRequest(
                dims=list(self.spec.dims), batch=self.batch, lr=self.lr, seed=self.seed, rank=i,
                worldSize=1, dataset="synthetic", numSamples=self.batch), timeout=self.timeout)
        self._all(cfg)
        shard = len(X) // n
        nb = steps_per_epoch or shard // self.batch
        self.out("Starting MLP training...")
        t0 = time.perf_counter()
        for ep in range(1, epochs + 1):
            loss_sum = corr_sum = 0.0
            for b in range(nb):
                def fwd_bwd(i, s):
                    lo = i * shard + b * self.batch
                    xb = np.ascontiguousarray(X[lo:lo + self.batch], dtype=np.float32)
                    yb = np.ascontiguousarray(y[lo:lo + self.batch], dtype=np.int32)
                    for addr, data in ((data_addr, xb.tobytes()), (label_addr, yb.tobytes())):
                        s.Memcpy(pb.MemcpyRequest(hostToDevice=pb.MemcpyHostToDeviceRequest(
                            hostSrcData=data, dstDeviceId=pb.DeviceId(value=self.dev_ids[i]),
                            dstMemAddr=pb.MemAddr(value=addr))), timeout=self.timeout)
                    f = s.RunForward(pb.RunForwardRequest(deviceId=self.dev_ids[i], inputAddr=data_addr,
                                                          numRows=self.batch, labelsAddr=label_addr),
                                     timeout=self.timeout)
                    s.RunBackward(pb.RunBackwardRequest(deviceId=self.dev_ids[i], gradientAddr=grad_addr),
                                  timeout=self.timeout)
                    return f
                fs = self._all(fwd_bwd)
                loss_sum += sum(f.loss for f in fs) / n
                corr_sum += sum(f.correct for f in fs)
                self.coord.AllReduceRing(pb.AllReduceRingRequest(
                    commId=self.comm_id, count=grad_bytes, op=SUM, dtype=DT_FLOAT32), timeout=self.timeout)
                self._all(lambda i, s: s.ApplyGradients(pb.ApplyGradientsRequest(
                    gradientAddr=grad_addr, scale=1.0 / n), timeout=self.timeout))
            self.out(f"Epoch {ep} complete: Avg Loss: {loss_sum / nb:.4f}, "
                     f"Accuracy: {100.0 * corr_sum / (nb * self.batch * n):.2f}%")
        wall = time.perf_counter() - t0
        self.out("Training complete.")
        out = {"wall_s": wall, "samples_per_s": epochs * nb * self.batch * n / wall}
        if X_test is not None:
            acc = self.test_rpc(X_test, y_test, data_addr, label_addr)
            self.out(f"Final Test Accuracy: {acc:.2f}%")
            out["test_accuracy"] = acc
        return out

    def test_rpc(self, X, y, data_addr, label_addr) -> float:
        s, dev = self.devs[0], self.dev_ids[0]
        correct = total = 0
        for lo in range(0, len(X) - self.batch + 1, self.batch):  # full batches, like client.go:478
            xb = np.ascontiguousarray(X[lo:lo + self.batch], dtype=np.float32)
            yb = np.ascontiguousarray(y[lo:lo + self.batch], dtype=np.int32)
            for addr, data in ((data_addr, xb.tobytes()), (label_addr, yb.tobytes())):
                s.Memcpy(pb.MemcpyRequest(hostToDevice=pb.MemcpyHostToDeviceRequest(
                    hostSrcData=data, dstDeviceId=pb.DeviceId(value=dev), dstMemAddr=pb.MemAddr(value=addr))))
            f = s.RunForward(pb.RunForwardRequest(deviceId=dev, inputAddr=data_addr, numRows=self.batch,
                                                  labelsAddr=label_addr))
            correct += f.correct
            total += self.batch
        return 100.0 * correct / max(total, 1)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="hipdsml train", description=__doc__.splitlines()[0])
    ap.add_argument("--coordinator", default="127.0.0.1:50051")
    ap.add_argument("--devices", default="127.0.0.1:5003,127.0.0.1:5004,127.0.0.1:5005")
    ap.add_argument("--mode", choices=["device", "rpc"], default="device")
    ap.add_argument("--model", default="784-128-64-10")
    ap.add_argument("--epochs", type=int, default=10)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--lr", type=float, default=0.01)
    ap.add_argument("--samples", type=int, default=60032, help="training samples per device")
    ap.add_argument("--steps-per-epoch", type=int, default=0)
    ap.add_argument("--graph-steps", type=int, default=50)
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(message)s")
    cl = TrainingClient(a.coordinator, a.devices.split(","), MlpSpec.parse(a.model).dims, a.batch, a.lr)
    try:
        if a.mode == "device":
            res = cl.train_device_mode(a.epochs, a.samples, a.graph_steps)
        else:
            from ..data.mnist import synthetic_mnist

            n = len(cl.devs)
            ds = synthetic_mnist(a.samples * n, seed=1000)
            te = synthetic_mnist(2048, seed=777)
            res = cl.train_rpc_mode(a.epochs, ds.X.numpy(), ds.y.numpy(), a.steps_per_epoch,
                                    te.X.numpy(), te.y.numpy())
        print(res)
    finally:
        cl.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())

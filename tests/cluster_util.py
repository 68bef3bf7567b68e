"""In-process test cluster: N device servers + a coordinator on ephemeral
localhost ports (the reference's fixtures start real gRPC servers on
``localhost:0`` the same way: gpu_coordinator_server_test.go:20-64)."""
from __future__ import annotations

import contextlib

from hipdsml.rpc.coordinator import start_coordinator
from hipdsml.rpc.device_server import start_device_server
from hipdsml.rpc.proto import pb
from hipdsml.rpc.stubs import GPUCoordinatorStub, GPUDeviceStub, connect


class Cluster:
    def __init__(self, n_devices=3, mem_size=1 << 20, backend="host", health_interval=0.0,
                 first_device_id=1, **coord_kw):
        self.devices = []
        for i in range(n_devices):
            server, addr, svc = start_device_server(first_device_id + i, mem_size, backend=backend)
            self.devices.append((server, addr, svc))
        self.coord_server, self.coord_addr, self.coord = start_coordinator(
            health_interval=health_interval, **coord_kw)
        self.channel = connect(self.coord_addr, timeout=5)
        self.stub = GPUCoordinatorStub(self.channel)
        self._dev_channels = []

    @property
    def addresses(self):
        return [a for (_, a, _) in self.devices]

    def device_stub(self, i) -> GPUDeviceStub:
        ch = connect(self.devices[i][1], timeout=5)
        self._dev_channels.append(ch)
        return GPUDeviceStub(ch)

    def comm_init(self, addresses=None, backend=""):
        addresses = self.addresses if addresses is None else addresses
        return self.stub.CommInit(pb.CommInitRequest(numDevices=len(addresses),
                                                     device_addresses=addresses, backend=backend))

    def close(self):
        for ch in self._dev_channels:
            ch.close()
        self.channel.close()
        self.coord.stop()
        self.coord_server.stop(0)
        for s, _, _ in self.devices:
            s.stop(0)


@contextlib.contextmanager
def cluster(**kw):
    c = Cluster(**kw)
    try:
        yield c
    finally:
        c.close()


def h2d(stub, device_id, addr, data):
    return stub.Memcpy(pb.MemcpyRequest(hostToDevice=pb.MemcpyHostToDeviceRequest(
        hostSrcData=data, dstDeviceId=pb.DeviceId(value=device_id), dstMemAddr=pb.MemAddr(value=addr))))


def d2h(stub, device_id, addr, n=0):
    return stub.Memcpy(pb.MemcpyRequest(deviceToHost=pb.MemcpyDeviceToHostRequest(
        srcDeviceId=pb.DeviceId(value=device_id), srcMemAddr=pb.MemAddr(value=addr),
        numBytes=n))).deviceToHost.dstData

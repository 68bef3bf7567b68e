"""gRPC client stubs and server registration for the ``gpu_sim`` services,
generated at import time from ``rpc/proto.py`` (no codegen step)."""
from __future__ import annotations

import time
from concurrent import futures
from typing import Optional, Tuple

import grpc

from ..utils.metrics import Histogram
from .proto import method_path, service_methods

# gRPC's default 4 MiB message cap would cap a Memcpy at ~4 MiB;
# raise it so a whole 28x28 dataset shard or an 80 MB wide-MLP gradient fits.
MAX_MSG = 1 << 30
CHANNEL_OPTIONS = [("grpc.max_send_message_length", MAX_MSG),
                   ("grpc.max_receive_message_length", MAX_MSG)]


class _Stub:
    _service = ""

    def __init__(self, channel: grpc.Channel):
        self.channel = channel
        for meth, req, resp, cstream in service_methods(self._service):
            path = method_path(self._service, meth)
            if cstream:
                fn = channel.stream_unary(path, request_serializer=req.SerializeToString,
                                          response_deserializer=resp.FromString)
            else:
                fn = channel.unary_unary(path, request_serializer=req.SerializeToString,
                                         response_deserializer=resp.FromString)
            setattr(self, meth, fn)


class GPUDeviceStub(_Stub):
    _service = "GPUDevice"


class GPUCoordinatorStub(_Stub):
    _service = "GPUCoordinator"


def _timed(fn, hist: Histogram):
    def handler(request, context):
        t0 = time.perf_counter()
        try:
            return fn(request, context)
        finally:  # aborted calls (context.abort raises) are timed too
            hist.add(time.perf_counter() - t0)
    return handler


def add_servicer(server: grpc.Server, service: str, servicer) -> None:
    """Register `servicer` (an object with one method per RPC, signature
    ``(request, context)``; client-streaming ones get the request iterator).
    Methods the servicer lacks answer UNIMPLEMENTED, like the Go
    ``Unimplemented*`` defaults (gpu_sim_grpc.pb.go:560-562).  Every
    implemented RPC is timed into ``servicer.rpc_latency[method]`` (a log2
    :class:`~hipdsml.utils.metrics.Histogram`; the reference only logs)."""
    handlers = {}
    lat = getattr(servicer, "rpc_latency", None)
    if lat is None:
        lat = {}
        servicer.rpc_latency = lat
    for meth, req, resp, cstream in service_methods(service):
        impl = getattr(servicer, meth, None)
        if impl is None:
            def impl(request, context, _m=meth):  # noqa: E306
                context.abort(grpc.StatusCode.UNIMPLEMENTED, f"method {_m} not implemented")
        else:
            impl = _timed(impl, lat.setdefault(meth, Histogram(meth)))
        if cstream:
            h = grpc.stream_unary_rpc_method_handler(impl, request_deserializer=req.FromString,
                                                     response_serializer=resp.SerializeToString)
        else:
            h = grpc.unary_unary_rpc_method_handler(impl, request_deserializer=req.FromString,
                                                    response_serializer=resp.SerializeToString)
        handlers[meth] = h
    server.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(f"gpu_sim.{service}", handlers),))


def make_server(max_workers: int = 16) -> grpc.Server:
    return grpc.server(futures.ThreadPoolExecutor(max_workers=max_workers), options=CHANNEL_OPTIONS)


def serve(service: str, servicer, address: str = "127.0.0.1:0",
          max_workers: int = 16) -> Tuple[grpc.Server, str]:
    """Start a server; returns (server, "host:port") — port 0 picks a free one."""
    server = make_server(max_workers)
    add_servicer(server, service, servicer)
    host = address.rsplit(":", 1)[0]
    port = server.add_insecure_port(address)
    if port == 0:
        raise RuntimeError(f"could not bind {address}")
    server.start()
    return server, f"{host}:{port}"


def is_loopback(address: str) -> bool:
    """Whether a host[:port] address names this machine's loopback interface."""
    host = address.rsplit(":", 1)[0] if address.count(":") == 1 or address.startswith("[") else address
    host = host.strip("[]")
    return host in ("localhost", "::1") or host.startswith("127.")


def connect(address: str, timeout: Optional[float] = None) -> grpc.Channel:
    """Insecure channel; with `timeout`, wait until it is READY (an explicit
    connect, unlike the reference's lazy grpc.Dial retry loop)."""
    ch = grpc.insecure_channel(address, options=CHANNEL_OPTIONS)
    if timeout is not None:
        grpc.channel_ready_future(ch).result(timeout=timeout)
    return ch

"""GPUDevice service — mirrors the reference's device unit tests
(DSML/gpu_device_service/gpu_device_server_test.go:46-164) over real gRPC, on the
CPU-simulated device runtime, plus memory-semantics checks the reference lacked."""
import grpc
import pytest

from hipdsml.rpc.device_server import start_device_server
from hipdsml.rpc.proto import IN_PROGRESS, SUCCESS, FAILED, pb
from hipdsml.rpc.stubs import GPUDeviceStub, connect
from hipdsml.runtime.device import HostDevice


@pytest.fixture
def dev():
    server, addr, svc = start_device_server(1001, 1 << 20, backend="host")
    ch = connect(addr, timeout=5)
    yield GPUDeviceStub(ch), svc, addr
    ch.close()
    server.stop(0)


def test_get_device_metadata(dev):  # TestGetDeviceMetadata (:46-63)
    stub, _, _ = dev
    md = stub.GetDeviceMetadata(pb.GetDeviceMetadataRequest()).metadata
    assert md.deviceId.value == 1001
    assert md.minMemAddr.value == 0x1000
    assert md.maxMemAddr.value == 0x101000
    assert md.backend == "host"


def test_rpc_latency_histograms(dev):
    """Every served RPC is timed per method (log2 histogram), reported by GetStats."""
    import json

    stub, svc, _ = dev
    for _ in range(5):
        stub.GetDeviceMetadata(pb.GetDeviceMetadataRequest())
    with pytest.raises(grpc.RpcError):  # aborted calls are timed too
        stub.GetStreamStatus(pb.GetStreamStatusRequest(streamId=pb.StreamId(value=7)))
        stub.BeginReceive(pb.BeginReceiveRequest(streamId=pb.StreamId(value=(1001 << 32) | 99),
                                                 recvBuffAddr=pb.MemAddr(value=0x1000)))
    h = svc.rpc_latency["GetDeviceMetadata"]
    assert h.n == 5 and 0 < h.min <= h.max and h.quantile(0.5) >= h.min
    st = json.loads(stub.GetStats(pb.GetStatsRequest()).json)
    assert st["rpc_latency"]["GetDeviceMetadata"]["n"] == 5
    assert st["rpc_latency"]["BeginReceive"]["n"] == 1


def test_begin_send(dev):  # TestBeginSend (:65-79)
    stub, _, _ = dev
    r = stub.BeginSend(pb.BeginSendRequest(sendBuffAddr=pb.MemAddr(value=0x1000), numBytes=1024,
                                           dstRank=pb.Rank(value=1)))
    assert r.initiated and r.streamId.value != 0


def test_begin_receive(dev):  # TestBeginReceive (:81-105)
    stub, _, _ = dev
    sid = stub.BeginSend(pb.BeginSendRequest(sendBuffAddr=pb.MemAddr(value=0x1000), numBytes=1024,
                                             dstRank=pb.Rank(value=1))).streamId.value
    r = stub.BeginReceive(pb.BeginReceiveRequest(streamId=pb.StreamId(value=sid),
                                                 recvBuffAddr=pb.MemAddr(value=0x2000), numBytes=1024,
                                                 srcRank=pb.Rank(value=0)))
    assert r.initiated


def test_begin_receive_errors(dev):
    stub, _, _ = dev
    own_unknown = (1001 << 32) | 999
    with pytest.raises(grpc.RpcError) as e:
        stub.BeginReceive(pb.BeginReceiveRequest(streamId=pb.StreamId(value=own_unknown),
                                                 recvBuffAddr=pb.MemAddr(value=0x2000), numBytes=8))
    assert e.value.code() == grpc.StatusCode.NOT_FOUND
    sid = stub.BeginSend(pb.BeginSendRequest(sendBuffAddr=pb.MemAddr(value=0x1000), numBytes=8)).streamId.value
    with pytest.raises(grpc.RpcError) as e:
        stub.BeginReceive(pb.BeginReceiveRequest(streamId=pb.StreamId(value=sid),
                                                 recvBuffAddr=pb.MemAddr(value=0x900), numBytes=8))
    assert e.value.code() == grpc.StatusCode.INVALID_ARGUMENT


def test_stream_send(dev):  # TestStreamSend (:107-144)
    stub, svc, _ = dev
    sid = stub.BeginSend(pb.BeginSendRequest(sendBuffAddr=pb.MemAddr(value=0x1000), numBytes=12,
                                             dstRank=pb.Rank(value=1))).streamId.value
    stub.BeginReceive(pb.BeginReceiveRequest(streamId=pb.StreamId(value=sid),
                                             recvBuffAddr=pb.MemAddr(value=0x2000), numBytes=12))
    chunks = [pb.DataChunk(data=b"chunk1", streamId=sid), pb.DataChunk(data=b"chunk2", streamId=sid)]
    assert stub.StreamSend(iter(chunks)).success
    assert svc.dev.read(0x2000, 12) == b"chunk1chunk2"
    assert stub.GetStreamStatus(pb.GetStreamStatusRequest(streamId=pb.StreamId(value=sid))).status == SUCCESS


def test_stream_send_length_mismatch_fails(dev):
    stub, _, _ = dev
    sid = stub.BeginSend(pb.BeginSendRequest(sendBuffAddr=pb.MemAddr(value=0x1000), numBytes=100)).streamId.value
    stub.BeginReceive(pb.BeginReceiveRequest(streamId=pb.StreamId(value=sid),
                                             recvBuffAddr=pb.MemAddr(value=0x2000), numBytes=100))
    assert not stub.StreamSend(iter([pb.DataChunk(data=b"short", streamId=sid)])).success
    assert stub.GetStreamStatus(pb.GetStreamStatusRequest(streamId=pb.StreamId(value=sid))).status == FAILED
    with pytest.raises(grpc.RpcError) as e:
        stub.StreamSend(iter([pb.DataChunk(data=b"x", streamId=0)]))
    assert e.value.code() == grpc.StatusCode.INVALID_ARGUMENT


def test_get_stream_status(dev):  # TestGetStreamStatus (:146-164)
    stub, _, _ = dev
    sid = stub.BeginSend(pb.BeginSendRequest(sendBuffAddr=pb.MemAddr(value=0x1000), numBytes=8)).streamId.value
    assert stub.GetStreamStatus(pb.GetStreamStatusRequest(streamId=pb.StreamId(value=sid))).status == IN_PROGRESS
    assert stub.GetStreamStatus(pb.GetStreamStatusRequest(streamId=pb.StreamId(value=12345))).status == FAILED


def test_memcpy_semantics(dev):
    stub, _, _ = dev
    w = lambda a, d: stub.Memcpy(pb.MemcpyRequest(hostToDevice=pb.MemcpyHostToDeviceRequest(  # noqa: E731
        hostSrcData=d, dstMemAddr=pb.MemAddr(value=a))))
    r = lambda a, n=0: stub.Memcpy(pb.MemcpyRequest(deviceToHost=pb.MemcpyDeviceToHostRequest(  # noqa: E731
        srcMemAddr=pb.MemAddr(value=a), numBytes=n))).deviceToHost.dstData
    assert w(0x1000, b"Hello GPU!").hostToDevice.success
    assert r(0x1000) == b"Hello GPU!"            # numBytes=0: whole last write (reference)
    assert r(0x1000, 5) == b"Hello"              # exact numBytes (Q12 fix)
    w(0x1006, b"MI355X")                          # linear memory: partial overwrite
    assert r(0x1000, 12) == b"Hello MI355X"
    for bad in (0x0, 0xFFF, 0x101000):
        with pytest.raises(grpc.RpcError) as e:
            w(bad, b"x")
        assert e.value.code() == grpc.StatusCode.INVALID_ARGUMENT
    with pytest.raises(grpc.RpcError) as e:
        r(0x5000)
    assert e.value.code() == grpc.StatusCode.INTERNAL  # "no data found"


def test_device_to_device_push():
    a_srv, a_addr, a = start_device_server(1, 1 << 16, backend="host")
    b_srv, b_addr, b = start_device_server(2, 1 << 16, backend="host")
    try:
        sa = GPUDeviceStub(connect(a_addr, timeout=5))
        sb = GPUDeviceStub(connect(b_addr, timeout=5))
        payload = bytes(range(256)) * 40
        a.dev.write(0x1000, payload)
        sid = sa.BeginSend(pb.BeginSendRequest(sendBuffAddr=pb.MemAddr(value=0x1000),
                                               numBytes=len(payload), dstRank=pb.Rank(value=1),
                                               dstAddress=b_addr)).streamId.value
        sb.BeginReceive(pb.BeginReceiveRequest(streamId=pb.StreamId(value=sid),
                                               recvBuffAddr=pb.MemAddr(value=0x3000),
                                               numBytes=len(payload), srcRank=pb.Rank(value=0)))
        import time
        for _ in range(500):
            st = sa.GetStreamStatus(pb.GetStreamStatusRequest(streamId=pb.StreamId(value=sid))).status
            if st != IN_PROGRESS:
                break
            time.sleep(0.01)
        assert st == SUCCESS
        assert b.dev.read(0x3000, len(payload)) == payload
    finally:
        a_srv.stop(0)
        b_srv.stop(0)


def test_host_device_reduce_dtypes():
    d = HostDevice(1, 1 << 12)
    import numpy as np
    a = np.arange(8, dtype=np.float32)
    d.write(0x1000, a.tobytes())
    d.write(0x1100, (a * 2).tobytes())
    d.reduce(0x1000, 0x1100, 32, 0, 0)
    assert np.array_equal(np.frombuffer(d.read(0x1000, 32), dtype=np.float32), a * 3)
    d.write(0x1200, bytes([200, 100]))
    d.write(0x1300, bytes([100, 100]))
    d.reduce(0x1200, 0x1300, 2, 1, 0)   # uint8 wraps like the reference byte add
    assert d.read(0x1200, 2) == bytes([44, 200])

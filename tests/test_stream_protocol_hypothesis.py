"""Property-based stress of the device servicer's stream protocol (SURVEY §5,
race detection): random interleavings of BeginSend / BeginReceive /
StreamSend / GetStreamStatus / Memcpy against one device server (host
backend, real gRPC), checked against a byte-level model of device memory and
of every stream's state; plus concurrent senders from a thread pool.

Reference protocol: gpu_device_server.go BeginSend/BeginReceive/StreamSend/
GetStreamStatus; the reference's own tests only walk one
stream through it (gpu_device_server_test.go:65-164)."""
import concurrent.futures as cf

import grpc
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st
from hypothesis.stateful import Bundle, RuleBasedStateMachine, invariant, rule

from hipdsml.rpc.device_server import start_device_server
from hipdsml.rpc.proto import FAILED, IN_PROGRESS, SUCCESS, pb
from hipdsml.rpc.stubs import GPUDeviceStub, connect

BASE, SIZE = 0x1000, 1 << 14


def _addr_len():
    return st.integers(1, 512).flatmap(
        lambda n: st.tuples(st.integers(BASE, BASE + SIZE - n), st.just(n)))


class StreamProtocol(RuleBasedStateMachine):
    def __init__(self):
        super().__init__()
        self.server, addr, self.svc = start_device_server(7, SIZE, backend="host")
        self.ch = connect(addr, timeout=5)
        self.stub = GPUDeviceStub(self.ch)
        self.mem = bytearray(SIZE)  # model: what the device memory must hold
        self.written = bytearray(SIZE)  # 1 where the model knows the byte
        self.state = {}  # stream id -> {"n", "recv", "status"}

    def teardown(self):
        self.ch.close()
        self.server.stop(0)

    streams = Bundle("streams")

    @rule(target=streams, al=_addr_len())
    def begin_send(self, al):
        a, n = al
        r = self.stub.BeginSend(pb.BeginSendRequest(sendBuffAddr=pb.MemAddr(value=a), numBytes=n,
                                                    dstRank=pb.Rank(value=1)))
        assert r.initiated and r.streamId.value not in self.state
        self.state[r.streamId.value] = {"n": n, "recv": None, "status": IN_PROGRESS}
        return r.streamId.value

    @rule(sid=streams, dst=st.integers(BASE, BASE + SIZE - 1))
    def begin_receive(self, sid, dst):
        s = self.state[sid]
        if s["recv"] is not None or s["status"] != IN_PROGRESS:
            return
        n = s["n"]
        # the coordinator's ring receives into the device's private scratch
        # window directly above max_addr, so the RPC accepts that window too
        ok_range = dst + n <= BASE + SIZE + self.svc.dev.scratch_size
        try:
            r = self.stub.BeginReceive(pb.BeginReceiveRequest(
                streamId=pb.StreamId(value=sid), recvBuffAddr=pb.MemAddr(value=dst), numBytes=n,
                srcRank=pb.Rank(value=0)))
        except grpc.RpcError as e:
            assert not ok_range and e.code() == grpc.StatusCode.INVALID_ARGUMENT
            return
        assert ok_range and r.initiated
        s["recv"] = dst

    @rule(sid=streams, data=st.data(), short=st.booleans())
    def stream_send(self, sid, data, short):
        s = self.state[sid]
        if s["recv"] is None or s["status"] != IN_PROGRESS:
            return
        n = s["n"] - (1 if short and s["n"] > 1 else 0)
        payload = data.draw(st.binary(min_size=n, max_size=n))
        cuts = sorted(data.draw(st.lists(st.integers(0, n), max_size=4)))
        pieces = [payload[a:b] for a, b in zip([0] + cuts, cuts + [n])]
        chunks = [pb.DataChunk(data=p, streamId=sid) for p in pieces if p] or \
            [pb.DataChunk(data=b"", streamId=sid)]
        r = self.stub.StreamSend(iter(chunks))
        o = s["recv"] - BASE
        m = max(0, min(n, SIZE - o))  # bytes inside the user range (the rest is scratch)
        if n == s["n"]:
            assert r.success
            s["status"] = SUCCESS
            self.mem[o:o + m] = payload[:m]
            self.written[o:o + m] = b"\x01" * m
        else:
            assert not r.success
            s["status"] = FAILED
            # chunks land as they arrive: a failed stream leaves its region undefined
            mm = max(0, min(s["n"], SIZE - o))
            self.written[o:o + mm] = b"\x00" * mm

    @rule(al=_addr_len(), data=st.data())
    def memcpy_roundtrip(self, al, data):
        a, n = al
        payload = data.draw(st.binary(min_size=n, max_size=n))
        assert self.stub.Memcpy(pb.MemcpyRequest(hostToDevice=pb.MemcpyHostToDeviceRequest(
            hostSrcData=payload, dstMemAddr=pb.MemAddr(value=a)))).hostToDevice.success
        o = a - BASE
        self.mem[o:o + n] = payload
        self.written[o:o + n] = b"\x01" * n
        got = self.stub.Memcpy(pb.MemcpyRequest(deviceToHost=pb.MemcpyDeviceToHostRequest(
            srcMemAddr=pb.MemAddr(value=a), numBytes=n))).deviceToHost.dstData
        assert got == payload

    @rule(sid=st.integers(1, 1 << 40))
    def unknown_status(self, sid):
        if sid in self.state:
            return
        assert self.stub.GetStreamStatus(pb.GetStreamStatusRequest(
            streamId=pb.StreamId(value=sid))).status == FAILED

    @invariant()
    def statuses_and_memory_agree(self):
        for sid, s in self.state.items():
            got = self.stub.GetStreamStatus(pb.GetStreamStatusRequest(streamId=pb.StreamId(value=sid))).status
            assert got == s["status"], (sid, got, s)
        known = bytes(self.written)
        dev = self.svc.dev.read(BASE, SIZE)
        for i in range(0, SIZE, 1024):
            seg = slice(i, i + 1024)
            if any(known[seg]):
                assert bytes(b for b, k in zip(dev[seg], known[seg]) if k) == \
                    bytes(b for b, k in zip(self.mem[seg], known[seg]) if k)


StreamProtocol.TestCase.settings = settings(max_examples=25, stateful_step_count=20, deadline=None,
                                            suppress_health_check=[HealthCheck.too_slow])
test_stream_protocol_state_machine = StreamProtocol.TestCase


@settings(max_examples=10, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(st.lists(st.integers(1, 4096), min_size=2, max_size=12), st.integers(1, 8))
def test_concurrent_streams_land_intact(sizes, workers):
    """Many streams pushed concurrently (thread pool) to disjoint receive
    buffers: every one completes and lands byte-exact."""
    server, addr, svc = start_device_server(9, 1 << 16, backend="host")
    ch = connect(addr, timeout=5)
    stub = GPUDeviceStub(ch)
    try:
        plans, off = [], BASE
        for i, n in enumerate(sizes):
            payload = bytes((i * 31 + j) & 0xFF for j in range(n))
            sid = stub.BeginSend(pb.BeginSendRequest(sendBuffAddr=pb.MemAddr(value=BASE), numBytes=n,
                                                     dstRank=pb.Rank(value=1))).streamId.value
            stub.BeginReceive(pb.BeginReceiveRequest(streamId=pb.StreamId(value=sid),
                                                     recvBuffAddr=pb.MemAddr(value=off), numBytes=n))
            plans.append((sid, off, payload))
            off += n

        def push(p):
            sid, _, payload = p
            step = max(1, len(payload) // 3)
            chunks = [pb.DataChunk(data=payload[i:i + step], streamId=sid)
                      for i in range(0, len(payload), step)]
            return stub.StreamSend(iter(chunks)).success

        with cf.ThreadPoolExecutor(workers) as ex:
            assert all(ex.map(push, plans))
        for sid, dst, payload in plans:
            assert stub.GetStreamStatus(pb.GetStreamStatusRequest(
                streamId=pb.StreamId(value=sid))).status == SUCCESS
            assert svc.dev.read(dst, len(payload)) == payload
    finally:
        ch.close()
        server.stop(0)


if __name__ == "__main__":
    pytest.main([__file__, "-q"])

"""GPUCoordinator — mirrors DSML/gpu_coordinator_service/gpu_coordinator_server_test.go
and allreduce_comparison_test.go (real gRPC servers on ephemeral ports), then adds
what the reference never checked: all-reduce VALUES for every op / dtype / n."""
import time

import grpc
import numpy as np
import pytest

from hipdsml.rpc.proto import DT_BFLOAT16, DT_FLOAT32, DT_INT32, DT_UINT8, FAILED, IN_PROGRESS, SUCCESS, pb

from cluster_util import Cluster, cluster, d2h, h2d


def _status(c, cid):
    return c.stub.GetCommStatus(pb.GetCommStatusRequest(commId=cid)).status


def test_comm_init_with_invalid_devices():  # TestCommInitWithInvalidDevices (:67-99)
    with cluster(n_devices=1, connect_timeout=0.5) as c:
        with pytest.raises(grpc.RpcError) as e:
            c.comm_init([c.addresses[0], "localhost:99999", "wrongformat"])
        assert e.value.code() == grpc.StatusCode.INTERNAL
        assert "device 1" in e.value.details() and "device 2" in e.value.details()


def test_comm_init_validates_num_devices():
    with cluster(n_devices=2) as c:
        with pytest.raises(grpc.RpcError) as e:
            c.stub.CommInit(pb.CommInitRequest(numDevices=3, device_addresses=c.addresses))
        assert e.value.code() == grpc.StatusCode.INVALID_ARGUMENT


def test_comm_init_returns_real_metadata_and_ids():
    with cluster(n_devices=3, mem_size=1 << 16) as c:
        r0 = c.comm_init()
        r1 = c.comm_init()
        assert r0.success and r0.commId == 0 and r1.commId == 1
        assert [d.deviceId.value for d in r0.devices] == [1, 2, 3]
        assert all(d.maxMemAddr.value == 0x1000 + (1 << 16) for d in r0.devices)  # Q8 fix


def test_memcpy_host_to_device_and_device_to_host():  # TestMemcpyHostToDeviceAndDeviceToHost (:102-173)
    with cluster(n_devices=3) as c:
        r = c.comm_init()
        dev_id = r.devices[1].deviceId.value
        assert h2d(c.stub, dev_id, 0x1000, b"Hello GPU!").hostToDevice.success
        assert d2h(c.stub, dev_id, 0x1000) == b"Hello GPU!"
        # one source of truth: the bytes are really on that device (Q3 fix)
        assert c.devices[1][2].dev.read(0x1000, 10) == b"Hello GPU!"
        assert c.stub.CommDestroy(pb.CommDestroyRequest(commId=r.commId)).success


def test_memcpy_unknown_device():
    with cluster(n_devices=1) as c:
        with pytest.raises(grpc.RpcError) as e:
            h2d(c.stub, 42, 0x1000, b"x")
        assert e.value.code() == grpc.StatusCode.NOT_FOUND


def test_group_operations_without_comm():  # TestGroupOperationsWithoutComm (:176-200)
    with cluster(n_devices=0) as c:
        for fn, req in ((c.stub.GroupStart, pb.GroupStartRequest), (c.stub.GroupEnd, pb.GroupEndRequest)):
            with pytest.raises(grpc.RpcError) as e:
                fn(req(commId=9999))
            assert e.value.code() == grpc.StatusCode.NOT_FOUND


def test_comm_destroy_invalid_id():  # TestCommDestroyInvalidId (:203-224)
    with cluster(n_devices=0) as c:
        with pytest.raises(grpc.RpcError) as e:
            c.stub.CommDestroy(pb.CommDestroyRequest(commId=9999))
        assert e.value.code() == grpc.StatusCode.NOT_FOUND


def test_coordinator_allreduce_ring_no_devices():  # TestCoordinatorAllReduceRing (:227-317)
    with cluster(n_devices=0) as c:
        cid = c.comm_init([]).commId
        assert c.stub.GroupStart(pb.GroupStartRequest(commId=cid)).success
        assert c.stub.AllReduceRing(pb.AllReduceRingRequest(commId=cid, count=16, op=0)).success
        assert _status(c, cid) == SUCCESS
        assert c.stub.GroupEnd(pb.GroupEndRequest(commId=cid)).success
        assert c.stub.CommDestroy(pb.CommDestroyRequest(commId=cid)).success


def test_allreduce_ring_single_device():  # TestAllReduceRingSingleDevice (:319-368)
    with cluster(n_devices=1) as c:
        cid = c.comm_init().commId
        assert c.stub.AllReduceRing(pb.AllReduceRingRequest(commId=cid, count=0, op=0)).success
        assert _status(c, cid) == SUCCESS


def test_coordinator_device_failure():  # TestCoordinatorDeviceFailure (:370-429), 6 s sleep -> 0.2 s interval
    with cluster(n_devices=2, health_interval=0.2, health_timeout=0.5) as c:
        cid = c.comm_init().commId
        assert _status(c, cid) == IN_PROGRESS
        c.devices[0][0].stop(0)  # kill device 0
        deadline = time.time() + 10
        while _status(c, cid) != FAILED and time.time() < deadline:
            time.sleep(0.05)
        assert _status(c, cid) == FAILED
        err = c.stub.GetCommStatus(pb.GetCommStatusRequest(commId=cid)).error
        assert "lost devices 1" in err
        with pytest.raises(grpc.RpcError) as e:
            c.stub.AllReduceRing(pb.AllReduceRingRequest(commId=cid, count=16))
        assert e.value.code() == grpc.StatusCode.FAILED_PRECONDITION


def _fill(c, n, arrays, addr=0x1000):
    for i in range(n):
        c.devices[i][2].dev.write(addr, arrays[i].tobytes())


def _read(c, i, nbytes, dtype, addr=0x1000):
    return np.frombuffer(c.devices[i][2].dev.read(addr, nbytes), dtype=dtype)


@pytest.mark.parametrize("n", [2, 3, 4, 5, 8])
@pytest.mark.parametrize("op,fn", [(0, np.sum), (1, np.prod), (2, np.min), (3, np.max)])
def test_rpc_ring_values_float32(n, op, fn):
    rng = np.random.default_rng(n * 10 + op)
    count = 1003  # not divisible by n: uneven segments
    arrays = [rng.uniform(0.5, 1.5, count).astype(np.float32) for _ in range(n)]
    with cluster(n_devices=n, mem_size=1 << 16) as c:
        cid = c.comm_init().commId
        _fill(c, n, arrays)
        r = c.stub.AllReduceRing(pb.AllReduceRingRequest(commId=cid, count=count * 4, op=op,
                                                         dtype=DT_FLOAT32))
        assert r.success
        want = fn(np.stack(arrays), axis=0)
        for i in range(n):
            np.testing.assert_allclose(_read(c, i, count * 4, np.float32), want, rtol=1e-5)
        assert _status(c, cid) == SUCCESS


def test_rpc_ring_dtypes_and_addresses():
    n = 3
    with cluster(n_devices=n, mem_size=1 << 16) as c:
        cid = c.comm_init().commId
        # per-rank buffer addresses (memAddrs honoured, Q7)
        req = pb.AllReduceRingRequest(commId=cid, count=64, op=0, dtype=DT_UINT8)
        addrs = [0x1000, 0x2000, 0x3000]
        for r, a in enumerate(addrs):
            req.memAddrs[r].value = a
            c.devices[r][2].dev.write(a, bytes([100 + r] * 64))
        assert c.stub.AllReduceRing(req).success
        for r, a in enumerate(addrs):
            assert c.devices[r][2].dev.read(a, 64) == bytes([(100 + 101 + 102) % 256] * 64)
        ints = [np.arange(50, dtype=np.int32) * (r + 1) for r in range(n)]
        _fill(c, n, ints)
        assert c.stub.AllReduceRing(pb.AllReduceRingRequest(commId=cid, count=200, op=3, dtype=DT_INT32)).success
        assert np.array_equal(_read(c, 2, 200, np.int32), np.arange(50, dtype=np.int32) * 3)
        import torch
        bf = [torch.full((40,), float(r + 1), dtype=torch.bfloat16) for r in range(n)]
        for r in range(n):
            c.devices[r][2].dev.write(0x4000, bf[r].view(torch.uint8).numpy().tobytes())
        req = pb.AllReduceRingRequest(commId=cid, count=80, op=0, dtype=DT_BFLOAT16)
        for r in range(n):
            req.memAddrs[r].value = 0x4000
        assert c.stub.AllReduceRing(req).success
        out = torch.frombuffer(bytearray(c.devices[0][2].dev.read(0x4000, 80)), dtype=torch.bfloat16)
        assert torch.all(out == 6.0)
        with pytest.raises(grpc.RpcError) as e:
            c.stub.AllReduceRing(pb.AllReduceRingRequest(commId=cid, count=6, dtype=DT_FLOAT32))
        assert e.value.code() == grpc.StatusCode.INVALID_ARGUMENT


def test_group_batches_collectives_and_finalize():
    n = 2
    with cluster(n_devices=n, mem_size=1 << 14) as c:
        cid = c.comm_init().commId
        _fill(c, n, [np.ones(16, np.float32), np.ones(16, np.float32) * 2])
        c.stub.GroupStart(pb.GroupStartRequest(commId=cid))
        assert c.stub.AllReduceRing(pb.AllReduceRingRequest(commId=cid, count=64)).success
        assert _status(c, cid) == IN_PROGRESS          # queued until GroupEnd
        assert np.all(_read(c, 0, 64, np.float32) == 1)
        assert c.stub.GroupEnd(pb.GroupEndRequest(commId=cid)).success
        assert np.all(_read(c, 0, 64, np.float32) == 3)
        assert c.stub.CommFinalize(pb.CommFinalizeRequest(commId=cid)).success
        assert _status(c, cid) == SUCCESS


def test_ring_chunked_large_buffer():
    n = 3
    count = 300_000  # 1.2 MB: several 256 KiB chunks per segment
    rng = np.random.default_rng(0)
    arrays = [rng.standard_normal(count).astype(np.float32) for _ in range(n)]
    with cluster(n_devices=n, mem_size=4 << 20) as c:
        cid = c.comm_init().commId
        _fill(c, n, arrays)
        assert c.stub.AllReduceRing(pb.AllReduceRingRequest(commId=cid, count=count * 4,
                                                            chunkBytes=256 << 10)).success
        np.testing.assert_allclose(_read(c, 1, count * 4, np.float32), sum(arrays), rtol=1e-5, atol=1e-5)


def test_allreduce_comparison():  # TestAllReduceComparison (allreduce_comparison_test.go:32-133)
    with cluster(n_devices=3, mem_size=4 << 20) as c:
        cid = c.comm_init().commId
        data = bytes([1]) * (1 << 20)
        for d in range(3):
            h2d(c.stub, d + 1, 0x1000, data)
        naive = c.stub.NaiveAllReduce(pb.NaiveAllReduceRequest(commId=cid, dataSize=1 << 20, latencyMs=10))
        assert naive.success and naive.totalDataTransferred == 6 * (1 << 20)
        assert naive.totalTimeMs >= 60  # 6 injected 10 ms sleeps inside the timed region
        assert c.devices[0][2].dev.read(0x2000, 16) == bytes([3]) * 16
        t0 = time.perf_counter()
        ring = c.stub.AllReduceRing(pb.AllReduceRingRequest(commId=cid, count=1 << 20, dtype=DT_UINT8))
        ring_ms = (time.perf_counter() - t0) * 1e3
        assert ring.success
        assert c.devices[2][2].dev.read(0x1000, 16) == bytes([3]) * 16  # values checked (the reference never did)
        print(f"naive={naive.totalTimeMs} ms ring={ring_ms:.1f} ms")


@pytest.mark.parametrize("algo", ["device-ring", "coordinator-ring"])
def test_device_failure_during_allreduce_fails_fast(algo):
    """BASELINE config 5 (fault injection), CPU plumbing: a device dies, the next
    AllReduceRing must fail promptly (peers aborted, no hang) and the
    communicator must end FAILED."""
    n = 3
    with cluster(n_devices=n, mem_size=1 << 20, rpc_timeout=60.0) as c:
        cid = c.comm_init().commId
        for i in range(n):
            c.devices[i][2].dev.write(0x1000, np.ones(4096, np.float32).tobytes())
        c.devices[2][0].stop(0)  # kill rank 2 without waiting for the health probe
        t0 = time.time()
        with pytest.raises(grpc.RpcError) as e:
            c.stub.AllReduceRing(pb.AllReduceRingRequest(commId=cid, count=4096 * 4, algo=algo))
        assert time.time() - t0 < 20.0
        assert e.value.code() == grpc.StatusCode.INTERNAL
        assert _status(c, cid) == FAILED
        with pytest.raises(grpc.RpcError) as e:
            c.stub.AllReduceRing(pb.AllReduceRingRequest(commId=cid, count=16))
        assert e.value.code() == grpc.StatusCode.FAILED_PRECONDITION


@pytest.mark.parametrize("algo", ["device-ring", "coordinator-ring"])
def test_device_dies_mid_allreduce_fails_fast(algo):
    """BASELINE config 5 proper: the fault fires INSIDE AllReduceRing (rank 2
    stops on its 3rd data-plane RPC, i.e. mid-ring), not before it."""
    n = 3
    with cluster(n_devices=n, mem_size=1 << 20, rpc_timeout=60.0) as c:
        cid = c.comm_init().commId
        for i in range(n):
            c.devices[i][2].dev.write(0x1000, np.ones(4096, np.float32).tobytes())
        c.devices[2][2].arm_fault(3, "stop")
        t0 = time.time()
        with pytest.raises(grpc.RpcError) as e:
            c.stub.AllReduceRing(pb.AllReduceRingRequest(commId=cid, count=4096 * 4, algo=algo))
        assert time.time() - t0 < 20.0
        assert e.value.code() == grpc.StatusCode.INTERNAL
        assert c.devices[2][2].failed
        assert _status(c, cid) == FAILED


def test_crashed_device_process_detected(tmp_path):
    """A device-server PROCESS configured with --fail-after crashes (os._exit)
    during the ring; the all-reduce errors out and the health monitor keeps the
    communicator FAILED."""
    import subprocess
    import sys

    from hipdsml.cli import child_env
    from hipdsml.rpc.coordinator import start_coordinator

    ports = []
    for _ in range(3):
        import socket

        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            ports.append(s.getsockname()[1])
    procs = []
    try:
        for i, p in enumerate(ports):
            extra = ["--fail-after", "4", "--fail-mode", "exit"] if i == 1 else []
            procs.append(subprocess.Popen(
                [sys.executable, "-m", "hipdsml", "device-server", "--ports", str(p),
                 "--device-ids", str(i + 1), "--backend", "host", "--mem-size", str(1 << 20)] + extra,
                env=child_env(), stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL))
        server, addr, svc = start_coordinator(health_interval=0.3, health_timeout=0.5)
        try:
            from hipdsml.rpc.stubs import GPUCoordinatorStub, connect

            stub = GPUCoordinatorStub(connect(addr, timeout=10))
            addrs = [f"127.0.0.1:{p}" for p in ports]
            deadline = time.time() + 120
            while True:
                try:
                    cid = stub.CommInit(pb.CommInitRequest(numDevices=3, device_addresses=addrs)).commId
                    break
                except grpc.RpcError:
                    if time.time() > deadline:
                        raise
                    time.sleep(0.5)
            with pytest.raises(grpc.RpcError):
                stub.AllReduceRing(pb.AllReduceRingRequest(commId=cid, count=1 << 16), timeout=60)
            assert procs[1].wait(timeout=30) == 17
            time.sleep(1.0)
            st = stub.GetCommStatus(pb.GetCommStatusRequest(commId=cid)).status
            assert st == FAILED
        finally:
            svc.stop()
            server.stop(0)
    finally:
        for p in procs:
            p.terminate()
        for p in procs:
            try:
                p.wait(timeout=10)
            except subprocess.TimeoutExpired:
                p.kill()


def test_ring_streams_close_when_idle_and_on_abort():
    """every comm's long-lived RingChannel holds one of the
    successor's gRPC workers; it must end when idle (and reopen on the next
    ring step) and when the comm is aborted, not live for a day."""
    n = 3
    with cluster(n_devices=n, mem_size=1 << 14) as c:
        for _, _, svc in c.devices:
            svc.RING_IDLE_S = 0.3
        cid = c.comm_init().commId
        arrays = [np.full(64, float(r + 1), dtype=np.float32) for r in range(n)]
        _fill(c, n, arrays)
        assert c.stub.AllReduceRing(pb.AllReduceRingRequest(commId=cid, count=256, dtype=DT_FLOAT32)).success
        assert all(cid in svc._ring_out for _, _, svc in c.devices)
        t_end = time.time() + 10
        while any(cid in svc._ring_out for _, _, svc in c.devices) and time.time() < t_end:
            time.sleep(0.05)
        assert not any(cid in svc._ring_out for _, _, svc in c.devices)  # idle: closed
        assert c.stub.AllReduceRing(pb.AllReduceRingRequest(commId=cid, count=256, dtype=DT_FLOAT32)).success
        np.testing.assert_array_equal(_read(c, 0, 256, np.float32), np.full(64, 18.0, np.float32))
        svc0 = c.devices[0][2]
        assert cid in svc0._ring_out  # reopened by the second call
        svc0.Abort(pb.AbortRequest(commId=cid, reason="test"), None)
        assert cid not in svc0._ring_out


def test_xgmi_algo_is_never_answered_by_rccl():
    """an explicit algo 'xgmi' on a comm whose data plane is RCCL
    must run (or fail as) the xGMI path, never report RCCL's time under that name."""
    with cluster(n_devices=2, mem_size=1 << 14) as c:
        cid = c.comm_init().commId
        c.coord.comms[cid].data_backend = "rccl"
        with pytest.raises(grpc.RpcError) as e:  # host devices: the xGMI path refuses
            c.stub.AllReduceRing(pb.AllReduceRingRequest(commId=cid, count=64, dtype=DT_FLOAT32, algo="xgmi"))
        assert "xgmi" in e.value.details().lower() or "xGMI" in e.value.details()


def test_pg_comm_with_loopback_store_and_remote_devices_is_refused_and_torn_down():
    """a 'pg' store bound to 127.0.0.1 is unreachable from devices
    on other hosts -- CommInit fails at once with a pointer to --store-host
    instead of every device waiting out its rendezvous timeout; the devices
    that were set up leave again (CommTeardown)."""
    from hipdsml.rpc import coordinator as C

    with cluster(n_devices=2, mem_size=1 << 14) as c:
        torn = []
        orig = c.coord._teardown_devices
        c.coord._teardown_devices = lambda comm: (torn.append(comm.id), orig(comm))
        real = C.is_loopback
        C.is_loopback = lambda a: a == "127.0.0.1" or (real(a) and a != c.addresses[1])
        try:
            with pytest.raises(grpc.RpcError) as e:
                c.comm_init(backend="pg")
        finally:
            C.is_loopback = real
        assert e.value.code() == grpc.StatusCode.INTERNAL and "--store-host" in e.value.details()
        assert torn == [0]


def test_allreduce_dispatch_picks_the_fast_path():
    """VERDICT r5 Next #4: with no algo flag, fp32 SUM on GPU devices of one
    node in a 'pg' comm runs over xGMI; RCCL comms run the tuned in-house ring;
    host devices the stream ring; an explicit algo always wins."""
    from hipdsml.rpc.coordinator import Communicator, GPUCoordinatorServicer as S

    def req(**kw):
        kw.setdefault("count", 1 << 20)
        kw.setdefault("dtype", DT_FLOAT32)
        return pb.AllReduceRingRequest(commId=0, **kw)

    xg = Communicator(0, [], backend="pg", xgmi=True)
    assert S.choose_algo(xg, req()) == "xgmi"
    assert S.choose_algo(xg, req(op=3)) == "stream-ring"             # MAX: not the xGMI sum
    assert S.choose_algo(xg, req(dtype=DT_UINT8, count=64)) == "stream-ring"
    assert S.choose_algo(xg, req(count=20)) == "stream-ring"         # not a 16-B multiple
    xg.data_backend = "rccl"
    assert S.choose_algo(xg, req()) == "xgmi"                        # same node: peer memory first
    assert S.choose_algo(xg, req(op=1)) == "ring"
    rc = Communicator(0, [], backend="rccl")
    assert S.choose_algo(rc, req()) == "ring"
    host = Communicator(0, [], backend="rpc")
    assert S.choose_algo(host, req()) == "stream-ring"
    assert S.choose_algo(host, req(algo="device-ring")) == "device-ring"


def test_allreduce_response_names_the_algorithm_that_ran():
    with cluster(n_devices=3, mem_size=1 << 14) as c:
        cid = c.comm_init().commId
        r = c.stub.AllReduceRing(pb.AllReduceRingRequest(commId=cid, count=256, dtype=DT_FLOAT32))
        assert r.success and r.algo == "stream-ring"
        r = c.stub.AllReduceRing(pb.AllReduceRingRequest(commId=cid, count=256, dtype=DT_FLOAT32,
                                                         algo="device-ring"))
        assert r.algo == "rpc-ring"
        assert not c.coord.comms[cid].xgmi                            # host devices: no peer memory

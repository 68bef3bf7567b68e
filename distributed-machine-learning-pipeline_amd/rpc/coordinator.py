"""GPUCoordinator servicer: control plane, collectives and failure detection.

Replaces ``DSML/gpu_coordinator_service/gpu_coordinator_server.go``.  Behaviour
kept: communicator ids from 0, rank = position in ``device_addresses``, the
status / error-code contract of SURVEY §2.2, NaiveAllReduce's injected-latency
benchmark, a periodic health probe that marks a communicator FAILED.

Deliberate fixes: the ring really moves data between devices
(Q1) and reduces by dtype (Q2) on the devices themselves; there is one source
of truth — device memory — and the coordinator Memcpy forwards to it (Q3); any
n works (Q4); ``op`` / ``memAddrs`` / ``numDevices`` are honoured (Q7); CommInit
returns each device's real metadata (Q8); the health probe runs outside the
lock (Q9) with an explicit connect deadline (Q10); CommDestroy closes channels
(Q11); CommFinalize is implemented; Group{Start,End} really batch collectives;
on a failure survivors are told to Abort their RCCL communicators so no rank
hangs.

Two data planes for AllReduceRing:
  backend "rpc"  : 2(n-1) ring steps; in each, every device pushes one segment
                   to its successor (BeginSend with dstAddress ->
                   StreamSend), the successor reduces it into place with a
                   device kernel (Reduce RPC).  Works for CPU-simulated devices.
  backend "rccl" : one DeviceAllReduce RPC per device; the devices run the
                   ring (ncclSend/ncclRecv, or RCCL's own all-reduce) GPU<->GPU
                   over xGMI.
"""
from __future__ import annotations

import logging
import threading
import time
from concurrent.futures import FIRST_EXCEPTION, ThreadPoolExecutor, wait
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional

import grpc
import numpy as np

from .proto import DT_FLOAT32, DT_SIZE, FAILED, IN_PROGRESS, SUCCESS, SUM, pb
from .stubs import GPUDeviceStub, connect, is_loopback

log = logging.getLogger("hipdsml.coordinator")

DEFAULT_ADDR = 0x1000  # reference gradientMemAddr / ring send buffer


@dataclass
class DeviceInfo:
    rank: int
    device_id: int
    address: str
    channel: grpc.Channel
    stub: GPUDeviceStub
    metadata: object
    last_health: float = 0.0


@dataclass
class Communicator:
    id: int
    devices: List[DeviceInfo]
    backend: str = "rpc"
    status: int = IN_PROGRESS
    error: str = ""
    group_active: bool = False
    pending: List[object] = field(default_factory=list)
    lock: threading.Lock = field(default_factory=threading.Lock)
    finalized: bool = False
    store: object = None        # backend "pg": the TCP store the devices' process group meets on
    data_backend: str = "rpc"   # what the devices' CommSetup reported ("rccl" when RCCL is up)
    xgmi: bool = False          # every device a GPU of one node in a "pg" group: xGMI peer memory


class CollectiveError(RuntimeError):
    pass


class GPUCoordinatorServicer:
    def __init__(self, health_interval: float = 5.0, health_timeout: float = 2.0,
                 connect_timeout: float = 3.0, rpc_timeout: float = 120.0,
                 sleep: Callable[[float], None] = time.sleep, max_parallel: int = 64,
                 store_host: str = "127.0.0.1"):
        # host the "pg" communicators' TCP stores bind to (the devices connect to it)
        self.store_host = store_host
        self._mu = threading.Lock()
        self._next_id = 0
        self.comms: Dict[int, Communicator] = {}
        self.health_interval = health_interval
        self.health_timeout = health_timeout
        self.connect_timeout = connect_timeout
        self.rpc_timeout = rpc_timeout
        self._sleep = sleep
        self._pool = ThreadPoolExecutor(max_workers=max_parallel)
        self._stop = threading.Event()
        self._health = threading.Thread(target=self._health_loop, daemon=True)
        if health_interval > 0:
            self._health.start()

    def stop(self) -> None:
        self._stop.set()
        self._pool.shutdown(wait=False)

    # ---------------------------------------------------------------- helpers --
    def _get(self, comm_id: int, context) -> Communicator:
        with self._mu:
            c = self.comms.get(comm_id)
        if c is None:
            context.abort(grpc.StatusCode.NOT_FOUND, f"communicator {comm_id} not found")
        return c

    def _parallel(self, fns, on_error=None):
        futs = [self._pool.submit(f) for f in fns]
        if on_error is not None:
            done, _ = wait(futs, return_when=FIRST_EXCEPTION)
            if any(f.exception() is not None for f in done):
                on_error()  # e.g. abort peers still blocked on the failed rank
        errs, out = [], []
        for f in futs:
            try:
                out.append(f.result())
            except Exception as e:  # collect every failure
                errs.append(e)
                out.append(None)
        if errs:
            raise CollectiveError("; ".join(str(e) for e in errs))
        return out

    def _device_by_id(self, device_id: int) -> Optional[DeviceInfo]:
        with self._mu:
            for c in self.comms.values():
                for d in c.devices:
                    if d.device_id == device_id:
                        return d
        return None

    def _fail(self, comm: Communicator, err: str, abort_devices: bool = True) -> None:
        with comm.lock:
            comm.status = FAILED
            comm.error = err
            devices = list(comm.devices)
        log.warning("communicator %d FAILED: %s", comm.id, err)
        if abort_devices and (comm.backend == "rccl" or comm.data_backend == "rccl"):
            for d in devices:
                self._pool.submit(self._safe_abort, d, comm.id, err)

    def _safe_abort(self, d: DeviceInfo, comm_id: int, reason: str) -> None:
        try:
            d.stub.Abort(pb.AbortRequest(commId=comm_id, reason=reason), timeout=self.health_timeout)
        except Exception:
            pass

    # --------------------------------------------------------------- CommInit --
    def CommInit(self, request, context):
        addrs = list(request.device_addresses)
        if request.numDevices and request.numDevices != len(addrs):
            context.abort(grpc.StatusCode.INVALID_ARGUMENT,
                          f"numDevices={request.numDevices} but {len(addrs)} device addresses")
        devices: List[DeviceInfo] = []
        errors: List[str] = []
        for rank, addr in enumerate(addrs):
            try:
                ch = connect(addr, timeout=self.connect_timeout)
                stub = GPUDeviceStub(ch)
                md = stub.GetDeviceMetadata(pb.GetDeviceMetadataRequest(),
                                            timeout=self.connect_timeout).metadata
                devices.append(DeviceInfo(rank, md.deviceId.value, addr, ch, stub, md, time.time()))
            except Exception as e:
                errors.append(f"device {rank} at {addr}: {type(e).__name__}: {e}")
        if errors:
            for d in devices:
                d.channel.close()
            context.abort(grpc.StatusCode.INTERNAL, "CommInit failed: " + "; ".join(errors))
        backend = request.backend or "rpc"
        if backend not in ("rpc", "rccl", "pg"):
            context.abort(grpc.StatusCode.INVALID_ARGUMENT, f"unknown backend {backend!r}")
        with self._mu:
            cid = self._next_id
            self._next_id += 1
        comm = Communicator(cid, devices, backend)
        try:
            self._setup_devices(comm)
        except Exception as e:
            # devices that did join (a process group, an RCCL comm) leave again:
            # the id was never registered, so CommDestroy could not reach them
            self._teardown_devices(comm)
            context.abort(grpc.StatusCode.INTERNAL, f"CommInit device setup failed: {e}")
        with self._mu:
            self.comms[cid] = comm
        log.info("CommInit: comm %d with %d devices (%s)", cid, len(devices), backend)
        return pb.CommInitResponse(success=True, commId=cid, devices=[d.metadata for d in devices])

    def _setup_devices(self, comm: Communicator) -> None:
        n = len(comm.devices)
        if n == 0:
            return
        peers = [d.address for d in comm.devices]
        uid = b""
        store_addr = ""
        if comm.backend == "rccl":
            uid = comm.devices[0].stub.GetCommUniqueId(
                pb.GetCommUniqueIdRequest(commId=comm.id), timeout=self.rpc_timeout).uniqueId
        elif comm.backend == "pg" and n > 1:
            # the devices' process group meets on a TCP store this coordinator
            # hosts (control plane only: IPC handles, self-test all-reduces,
            # agreement on the sync mode); the data plane is xGMI / RCCL
            import datetime

            import torch.distributed as dist

            if is_loopback(self.store_host) and not all(is_loopback(p) for p in peers):
                raise CollectiveError(
                    f"backend 'pg': the process-group store would bind to {self.store_host}, which "
                    f"devices on other hosts cannot reach (start the coordinator with --store-host, "
                    f"or use backend 'rccl')")
            comm.store = dist.TCPStore(self.store_host, 0, is_master=True, wait_for_workers=False,
                                       timeout=datetime.timedelta(seconds=self.rpc_timeout))
            store_addr = f"{self.store_host}:{comm.store.port}"
        # RCCL init / process-group rendezvous are collective: every rank must
        # enter them concurrently.
        rs = self._parallel([
            (lambda d=d: d.stub.CommSetup(pb.CommSetupRequest(
                commId=comm.id, uniqueId=uid, rank=d.rank, nranks=n, peerAddresses=peers,
                storeAddress=store_addr), timeout=self.rpc_timeout))
            for d in comm.devices])
        if all(r is not None and "rccl" in r.backend for r in rs):
            comm.data_backend = "rccl"
        comm.xgmi = n > 1 and all(r is not None and "xgmi" in r.backend for r in rs)

    # -------------------------------------------------------- status / lifecycle --
    def GetCommStatus(self, request, context):
        c = self._get(request.commId, context)
        with c.lock:
            return pb.GetCommStatusResponse(status=c.status, error=c.error)

    def CommDestroy(self, request, context):
        with self._mu:
            c = self.comms.pop(request.commId, None)
        if c is None:
            context.abort(grpc.StatusCode.NOT_FOUND, f"communicator {request.commId} not found")
        self._teardown_devices(c)
        return pb.CommDestroyResponse(success=True)

    def _teardown_devices(self, c: Communicator) -> None:
        """CommTeardown on every device (best effort), close the channels and
        drop the process group's store."""
        # a process group's teardown is collective: every device leaves together
        tmo = self.rpc_timeout if c.backend == "pg" else self.health_timeout
        futs = [self._pool.submit(d.stub.CommTeardown, pb.CommTeardownRequest(commId=c.id), timeout=tmo)
                for d in c.devices]
        for f in futs:
            try:
                f.result()
            except Exception:
                pass
        for d in c.devices:
            d.channel.close()
        c.store = None

    def CommFinalize(self, request, context):
        c = self._get(request.commId, context)
        with c.lock:
            pending = list(c.pending)
            c.pending.clear()
            c.group_active = False
        for op in pending:  # flush any unfinished group
            self._run_allreduce(c, op)
        with c.lock:
            c.finalized = True
            ok = c.status != FAILED
            if ok:
                c.status = SUCCESS
        return pb.CommFinalizeResponse(success=ok)

    def GroupStart(self, request, context):
        c = self._get(request.commId, context)
        with c.lock:
            c.group_active = True
        return pb.GroupStartResponse(success=True)

    def GroupEnd(self, request, context):
        c = self._get(request.commId, context)
        with c.lock:
            c.group_active = False
            pending = list(c.pending)
            c.pending.clear()
        ok = True
        for op in pending:
            ok = self._run_allreduce(c, op) and ok
        return pb.GroupEndResponse(success=ok)

    # -------------------------------------------------------------- AllReduce --
    def AllReduceRing(self, request, context):
        c = self._get(request.commId, context)
        with c.lock:
            status = c.status
            n = len(c.devices)
        if status == FAILED:
            context.abort(grpc.StatusCode.FAILED_PRECONDITION,
                          f"communicator {c.id} is in FAILED state: {c.error}")
        es = DT_SIZE.get(request.dtype, 0)
        if es == 0:
            context.abort(grpc.StatusCode.INVALID_ARGUMENT, f"unknown dtype {request.dtype}")
        if n < 2:
            with c.lock:
                c.status = SUCCESS
            return pb.AllReduceRingResponse(success=True)
        if request.count % es:
            context.abort(grpc.StatusCode.INVALID_ARGUMENT,
                          f"count={request.count} bytes is not a multiple of the element size {es}")
        op = pb.AllReduceRingRequest()
        op.CopyFrom(request)
        with c.lock:
            if c.group_active:
                c.pending.append(op)
                c.status = IN_PROGRESS
                return pb.AllReduceRingResponse(success=True)
        t0 = time.perf_counter()
        ran = {}
        ok = self._run_allreduce(c, op, ran)
        us = (time.perf_counter() - t0) * 1e6
        if not ok:
            context.abort(grpc.StatusCode.INTERNAL, f"AllReduceRing failed: {c.error}")
        return pb.AllReduceRingResponse(success=True, elapsedUs=us, algo=ran.get("algo", ""),
                                        chunkBytes=ran.get("chunk", 0))

    @staticmethod
    def choose_algo(c: Communicator, op) -> str:
        """The algorithm an AllReduceRing runs (the reference has one: its
        loopback ring, gpu_coordinator_server.go:338-356).  An explicit
        `algo` wins.  Otherwise the fastest path the communicator supports:

        * "xgmi" -- fp32 SUM of a 16-B multiple on GPU devices of one node in
          a "pg" group: one two-shot launch over xGMI peer memory
          (1.00 ms vs 2.45 ms for the stream ring with 3 devices on one GPU,
          profiles/r4_allreduce_rpc_hip.json);
        * "ring" -- RCCL is up (distinct GPUs): the in-house ring on
          ncclSend/ncclRecv with the chunk tuned per size class on the devices;
        * "stream-ring" -- host devices / no RCCL: the device-driven ring over
          long-lived gRPC streams."""
        if op.algo:
            return op.algo
        if c.xgmi and op.dtype == DT_FLOAT32 and op.op == SUM and op.count % 16 == 0:
            return "xgmi"
        if c.backend == "rccl" or c.data_backend == "rccl":
            return "ring"
        return "stream-ring"

    def _run_allreduce(self, c: Communicator, op, ran: Optional[dict] = None) -> bool:
        algo = self.choose_algo(c, op)
        ran = {} if ran is None else ran
        try:
            # an explicit algo "xgmi" runs over peer memory even when RCCL is up
            # ("pg" comms of GPU devices), so a benchmark asking for it never
            # gets RCCL's time under that name
            if algo == "xgmi":  # one launch over xGMI peer memory
                rs = self._parallel([
                    (lambda d=d: d.stub.DeviceAllReduce(pb.DeviceAllReduceRequest(
                        commId=c.id, addr=self._addr(op, d.rank), count=op.count, dtype=op.dtype,
                        op=op.op, algo="xgmi"), timeout=self.rpc_timeout))
                    for d in c.devices], on_error=lambda: self._abort_all(c, "peer failed during all-reduce"))
            elif c.backend == "rccl" or c.data_backend == "rccl":
                rs = self._allreduce_rccl(c, op, algo)
            elif algo == "coordinator-ring":
                self._allreduce_rpc_ring(c, op)
                rs = []
            else:  # "stream-ring" (default) / "device-ring": devices drive the ring themselves
                rs = self._allreduce_device_ring(c, op, algo)
        except Exception as e:
            self._fail(c, f"{type(e).__name__}: {e}")
            return False
        ran["algo"] = (rs[0].algo if rs and rs[0] is not None and rs[0].algo else algo)
        ran["chunk"] = rs[0].chunkBytes if rs and rs[0] is not None else 0
        with c.lock:
            if c.status != FAILED:
                c.status = SUCCESS
        return True

    def _addr(self, op, rank: int) -> int:
        return op.memAddrs[rank].value if rank in op.memAddrs else DEFAULT_ADDR

    def _allreduce_rccl(self, c: Communicator, op, algo: str = "ring"):
        algo = algo if algo in ("ring", "rccl") else "ring"
        return self._parallel([
            (lambda d=d: d.stub.DeviceAllReduce(pb.DeviceAllReduceRequest(
                commId=c.id, addr=self._addr(op, d.rank), count=op.count, dtype=op.dtype, op=op.op,
                algo=algo, chunkBytes=op.chunkBytes), timeout=self.rpc_timeout))
            for d in c.devices], on_error=lambda: self._abort_all(c, "peer failed during all-reduce"))

    def _abort_all(self, c: Communicator, reason: str) -> None:
        for d in list(c.devices):
            self._pool.submit(self._safe_abort, d, c.id, reason)

    def _allreduce_device_ring(self, c: Communicator, op, algo: str = "stream-ring"):
        return self._parallel([
            (lambda d=d: d.stub.DeviceAllReduce(pb.DeviceAllReduceRequest(
                commId=c.id, addr=self._addr(op, d.rank), count=op.count, dtype=op.dtype, op=op.op,
                algo="rpc-ring" if algo == "device-ring" else "stream-ring",
                chunkBytes=op.chunkBytes), timeout=self.rpc_timeout))
            for d in c.devices], on_error=lambda: self._abort_all(c, "peer failed during all-reduce"))

    def _wait_stream(self, d: DeviceInfo, sid: int) -> None:
        delay, t_end = 2e-4, time.time() + self.rpc_timeout
        while True:
            st = d.stub.GetStreamStatus(pb.GetStreamStatusRequest(streamId=pb.StreamId(value=sid)),
                                        timeout=self.rpc_timeout).status
            if st == SUCCESS:
                return
            if st == FAILED:
                raise CollectiveError(f"stream {sid} on device {d.device_id} failed")
            if time.time() > t_end:
                raise CollectiveError(f"stream {sid} on device {d.device_id} timed out")
            time.sleep(delay)
            delay = min(delay * 2, 0.01)

    def _begin_send(self, src: DeviceInfo, dst: DeviceInfo, src_addr: int, nbytes: int) -> int:
        return src.stub.BeginSend(pb.BeginSendRequest(
            sendBuffAddr=pb.MemAddr(value=src_addr), numBytes=nbytes, dstRank=pb.Rank(value=dst.rank),
            dstAddress=dst.address), timeout=self.rpc_timeout).streamId.value

    def _begin_receive(self, src: DeviceInfo, dst: DeviceInfo, sid: int, dst_addr: int, nbytes: int):
        dst.stub.BeginReceive(pb.BeginReceiveRequest(
            streamId=pb.StreamId(value=sid), recvBuffAddr=pb.MemAddr(value=dst_addr),
            numBytes=nbytes, srcRank=pb.Rank(value=src.rank)), timeout=self.rpc_timeout)

    def _transfer(self, src: DeviceInfo, dst: DeviceInfo, src_addr: int, dst_addr: int,
                  nbytes: int, reduce_op=None) -> None:
        """Device `src` pushes nbytes to device `dst` (device-driven stream).
        The receiver's WaitStream / Reduce(waitStreamId) block server-side on
        the stream's completion event — no status polling."""
        sid = self._begin_send(src, dst, src_addr, nbytes)
        self._begin_receive(src, dst, sid, dst_addr, nbytes)
        if reduce_op is None:
            st = dst.stub.WaitStream(pb.WaitStreamRequest(streamId=pb.StreamId(value=sid)),
                                     timeout=self.rpc_timeout).status
            if st != SUCCESS:
                raise CollectiveError(f"stream {sid} to device {dst.device_id} failed")
        else:
            red_dst, dtype, op = reduce_op
            dst.stub.Reduce(pb.ReduceRequest(dstAddr=red_dst, srcAddr=dst_addr, numBytes=nbytes,
                                             dtype=dtype, op=op, waitStreamId=sid),
                            timeout=self.rpc_timeout)

    def _allreduce_rpc_ring(self, c: Communicator, op) -> None:
        devs = c.devices
        n = len(devs)
        es = DT_SIZE[op.dtype]
        elems = op.count // es
        al = 16 // es
        seg = (-(-elems // n) + al - 1) // al * al
        off = [min(i * seg, elems) * es for i in range(n + 1)]
        scratch = min(d.metadata.maxMemAddr.value for d in devs)  # private window above max
        chunk = (op.chunkBytes or (1 << 20)) // es * es
        chunk = max(es, chunk)
        base = [self._addr(op, r) for r in range(n)]
        # Reduce-scatter: step s, rank r sends segment (r - s) to r + 1, which
        # reduces it into its own copy; rank r then owns segment (r + 1).
        for s in range(n - 1):
            for co in range(0, seg * es, chunk):
                jobs = []
                for r in range(n):
                    si = (r - s) % n
                    lo = off[si] + co
                    ln = max(0, min(chunk, off[si + 1] - lo))
                    if ln == 0:
                        continue
                    src, dst = devs[r], devs[(r + 1) % n]
                    scr = dst.metadata.maxMemAddr.value

                    def job(src=src, dst=dst, lo=lo, ln=ln, scr=scr, r_dst=(r + 1) % n):
                        self._transfer(src, dst, base[src.rank] + lo, scr, ln,
                                       reduce_op=(base[r_dst] + lo, op.dtype, op.op))
                    jobs.append(job)
                self._parallel(jobs)
        # All-gather: step s, rank r sends segment (r + 1 - s) straight into place.
        for s in range(n - 1):
            jobs = []
            for r in range(n):
                si = (r + 1 - s) % n
                ln = off[si + 1] - off[si]
                if ln == 0:
                    continue
                src, dst = devs[r], devs[(r + 1) % n]
                jobs.append(lambda src=src, dst=dst, si=si, ln=ln, rd=(r + 1) % n: self._transfer(
                    src, dst, base[src.rank] + off[si], base[rd] + off[si], ln))
            self._parallel(jobs)
        del scratch

    # --------------------------------------------------------- NaiveAllReduce --
    def NaiveAllReduce(self, request, context):
        """Gather to the coordinator, reduce, broadcast — with `latencyMs`
        injected before every device operation, as in the reference benchmark
        (gpu_coordinator_server.go:610-717): init (untimed) writes 0x01 bytes at
        0x1000 on every device; the timed part gathers from 0x1000, sums
        byte-wise and broadcasts to 0x2000."""
        c = self._get(request.commId, context)
        with c.lock:
            if c.status == FAILED:
                context.abort(grpc.StatusCode.FAILED_PRECONDITION, f"communicator {c.id} is FAILED")
            devs = list(c.devices)
        size = int(request.dataSize)
        lat = request.latencyMs / 1000.0
        payload = bytes([1]) * size
        try:
            for d in devs:
                self._sleep(lat)
                d.stub.Memcpy(pb.MemcpyRequest(hostToDevice=pb.MemcpyHostToDeviceRequest(
                    hostSrcData=payload, dstDeviceId=pb.DeviceId(value=d.device_id),
                    dstMemAddr=pb.MemAddr(value=0x1000))), timeout=self.rpc_timeout)
            t0 = time.perf_counter()
            acc = np.zeros(size, dtype=np.uint8)
            for d in devs:
                self._sleep(lat)
                r = d.stub.Memcpy(pb.MemcpyRequest(deviceToHost=pb.MemcpyDeviceToHostRequest(
                    srcDeviceId=pb.DeviceId(value=d.device_id), srcMemAddr=pb.MemAddr(value=0x1000),
                    numBytes=size)), timeout=self.rpc_timeout)
                acc += np.frombuffer(r.deviceToHost.dstData, dtype=np.uint8)
            out = acc.tobytes()
            for d in devs:
                self._sleep(lat)
                d.stub.Memcpy(pb.MemcpyRequest(hostToDevice=pb.MemcpyHostToDeviceRequest(
                    hostSrcData=out, dstDeviceId=pb.DeviceId(value=d.device_id),
                    dstMemAddr=pb.MemAddr(value=0x2000))), timeout=self.rpc_timeout)
            dt = time.perf_counter() - t0
        except grpc.RpcError as e:
            self._fail(c, f"NaiveAllReduce: {e.code().name}: {e.details()}")
            context.abort(grpc.StatusCode.INTERNAL, f"NaiveAllReduce failed: {e.details()}")
        log.info("Naive AllReduce completed: DataSize=%d, Latency=%dms, TotalTime=%dms, "
                 "TotalDataTransferred=%d bytes", size, request.latencyMs, int(dt * 1000),
                 2 * len(devs) * size)
        return pb.NaiveAllReduceResponse(success=True, totalTimeMs=int(dt * 1000),
                                         totalDataTransferred=2 * len(devs) * size,
                                         totalTimeUs=dt * 1e6)

    # ------------------------------------------------------------------ Memcpy --
    def Memcpy(self, request, context):
        """Forward to the owning device (one source of truth: device memory)."""
        which = request.WhichOneof("either")
        if which == "hostToDevice":
            dev_id = request.hostToDevice.dstDeviceId.value
        elif which == "deviceToHost":
            dev_id = request.deviceToHost.srcDeviceId.value
        else:
            context.abort(grpc.StatusCode.INVALID_ARGUMENT, "invalid Memcpy request")
        d = self._device_by_id(dev_id)
        if d is None:
            context.abort(grpc.StatusCode.NOT_FOUND, f"device {dev_id} is not part of any communicator")
        try:
            return d.stub.Memcpy(request, timeout=self.rpc_timeout)
        except grpc.RpcError as e:
            context.abort(e.code(), e.details())

    # ------------------------------------------------------------ health loop --
    def _health_loop(self) -> None:
        while not self._stop.wait(self.health_interval):
            self.check_health()

    def check_health(self) -> None:
        """Probe every device of every live communicator (outside the global
        lock); a dead device marks its communicator FAILED (terminal, like the
        reference) and the survivors are told to abort their RCCL comms."""
        with self._mu:
            comms = list(self.comms.values())
        for c in comms:
            with c.lock:
                if c.status == FAILED:
                    continue
                devices = list(c.devices)
            dead = []
            for d in devices:
                try:
                    d.stub.GetDeviceMetadata(pb.GetDeviceMetadataRequest(), timeout=self.health_timeout)
                    d.last_health = time.time()
                except Exception as e:
                    log.warning("Device %d at %s unreachable: %s", d.device_id, d.address, e)
                    dead.append(d)
            if dead:
                with c.lock:
                    c.devices = [d for d in c.devices if d not in dead]
                self._fail(c, "lost devices " + ", ".join(str(d.device_id) for d in dead))


def start_coordinator(address: str = "127.0.0.1:0", health_interval: float = 5.0, **kw):
    from .stubs import serve

    svc = GPUCoordinatorServicer(health_interval=health_interval, **kw)
    server, addr = serve("GPUCoordinator", svc, address, max_workers=32)
    log.info("GPU Coordinator server listening on %s", addr)
    return server, addr, svc

"""GPUDevice servicer: one process (or in-process server) per GPU.

MI355X-native replacement of ``DSML/gpu_device_service/gpu_device_server.go``:
the memory is a real HBM arena (HipDevice) or a host buffer (HostDevice, for
the CPU plumbing config), transfers between devices are pushed by the sending
device itself (BeginSend with ``dstAddress``), reductions run on the device
(HIP kernels), and the extension RPCs let the coordinator bootstrap an RCCL
communicator and run collectives / whole training steps on the GPU.
"""
from __future__ import annotations

import socket as _socket
import json
import logging
import threading
import time
from typing import Dict, Optional

import grpc
import torch

from ..runtime.device import (DT_SIZE, STATUS_FAILED, STATUS_IN_PROGRESS, STATUS_SUCCESS,
                              TORCH_DTYPES, OutOfRange, _Device, make_device)
from .proto import DT_FLOAT32, SUM, pb
from .stubs import GPUDeviceStub, connect, serve

log = logging.getLogger("hipdsml.device")

CHUNK = 1 << 20  # StreamSend chunk size


class GPUDeviceServicer:
    def __init__(self, device: _Device, name: str = ""):
        self.dev = device
        self.name = name or f"device-{device.device_id}"
        self.comms: Dict[int, object] = {}      # commId -> native RcclComm
        self.comm_meta: Dict[int, dict] = {}    # commId -> {"rank", "nranks", "peers"}
        self.pg_comm: Optional[int] = None      # commId whose process group this process joined
        self.pg_node_local = False              # every rank of that group on this node
        # RingChannel: per commId, the outgoing queue to the successor (one
        # long-lived client stream) and the inbox of the predecessor's messages
        self._ring_out: Dict[int, "queue.Queue"] = {}
        self._ring_in: Dict[int, dict] = {}
        self._ring_cv = threading.Condition()
        self._xgmi_ar: Dict[int, object] = {}   # commId -> XgmiAllReduce (pg comms on GPUs)
        self._ring_chunks: Dict[int, Dict[int, int]] = {}  # commId -> size class -> tuned chunk
        self._aborted_comms: set = set()        # Abort is sticky for its communicator
        self._peer_stubs: Dict[str, GPUDeviceStub] = {}
        self._lock = threading.Lock()
        self.trainer = None
        self._fwd_cache = None
        self.counters = {"h2d_bytes": 0, "d2h_bytes": 0, "stream_bytes_in": 0,
                         "stream_bytes_out": 0, "reduces": 0, "allreduces": 0, "train_steps": 0}
        self.server = None          # set by start_device_server (fault injection stops it)
        self._fault_left: Optional[int] = None
        self._fault_mode = "stop"
        self.failed = False

    # ------------------------------------------------------ fault injection --
    def arm_fault(self, after_rpcs: int, mode: str = "stop") -> None:
        """BASELINE config 5 hook: die on the `after_rpcs`-th data-plane RPC
        (BeginSend / BeginReceive / StreamSend / Memcpy / Reduce / DeviceAllReduce,
        and every RingChannel message).
        mode "stop": stop the gRPC server (in-process clusters, like the
        reference test's ``grpcServer.Stop()``, gpu_coordinator_server_test.go:415);
        "exit": terminate the process abruptly (a crashed device server)."""
        if mode not in ("stop", "exit"):
            raise ValueError("fault mode must be 'stop' or 'exit'")
        self._fault_left, self._fault_mode = int(after_rpcs), mode

    def _tick(self, context) -> None:
        if self.failed:
            context.abort(grpc.StatusCode.UNAVAILABLE, "device failed (fault injection)")
        if self._fault_left is None:
            return
        with self._lock:
            self._fault_left -= 1
            fire = self._fault_left <= 0
        if not fire:
            return
        self.failed = True
        self._fault_left = None
        log.warning("%s: injected fault (%s)", self.name, self._fault_mode)
        if self._fault_mode == "exit":
            import os

            os._exit(17)
        if self.server is not None:
            threading.Thread(target=self.server.stop, args=(0,), daemon=True).start()
        context.abort(grpc.StatusCode.UNAVAILABLE, "device failed (fault injection)")

    # ------------------------------------------------------------ helpers --
    def _peer(self, address: str) -> GPUDeviceStub:
        with self._lock:
            s = self._peer_stubs.get(address)
            if s is None:
                s = GPUDeviceStub(connect(address))
                self._peer_stubs[address] = s
            return s

    def _push(self, sid: int, send_addr: int, n: int, address: str) -> None:
        """Background device->device transfer of a BeginSend'd buffer."""
        try:
            data = self.dev.read(send_addr, n, internal=True)

            def chunks():
                if n == 0:
                    yield pb.DataChunk(data=b"", streamId=sid)
                for off in range(0, n, CHUNK):
                    yield pb.DataChunk(data=data[off:off + CHUNK], streamId=sid)

            resp = self._peer(address).StreamSend(chunks(), timeout=120)
            self.counters["stream_bytes_out"] += n
            self.dev.set_status(sid, STATUS_SUCCESS if resp.success else STATUS_FAILED)
        except Exception as e:  # peer died / transport error
            log.warning("stream %d push to %s failed: %s", sid, address, e)
            self.dev.set_status(sid, STATUS_FAILED)

    # ---------------------------------------------------------- reference API --
    def GetDeviceMetadata(self, request, context):
        md = pb.DeviceMetadata(deviceId=pb.DeviceId(value=self.dev.device_id),
                               minMemAddr=pb.MemAddr(value=self.dev.min_addr),
                               maxMemAddr=pb.MemAddr(value=self.dev.max_addr),
                               name=self.name, backend=self.dev.backend,
                               host=_socket.gethostname())
        return pb.GetDeviceMetadataResponse(metadata=md)

    def BeginSend(self, request, context):
        self._tick(context)
        addr, n = request.sendBuffAddr.value, request.numBytes
        sid = self.dev.begin_send(addr, n, request.dstRank.value)
        if request.dstAddress:
            try:
                self.dev.check(addr, n, internal=True)
            except OutOfRange as e:
                context.abort(grpc.StatusCode.INVALID_ARGUMENT, str(e))
            threading.Thread(target=self._push, args=(sid, addr, n, request.dstAddress),
                             daemon=True).start()
        return pb.BeginSendResponse(initiated=True, streamId=pb.StreamId(value=sid))

    def BeginReceive(self, request, context):
        self._tick(context)
        sid = request.streamId.value
        own = (sid >> 32) == self.dev.device_id
        if own and self.dev.stream(sid) is None:
            context.abort(grpc.StatusCode.NOT_FOUND, f"stream ID {sid} not found")
        try:
            self.dev.begin_receive(sid, request.recvBuffAddr.value, request.numBytes,
                                   request.srcRank.value, create=True)
        except OutOfRange as e:
            context.abort(grpc.StatusCode.INVALID_ARGUMENT, str(e))
        return pb.BeginReceiveResponse(initiated=True)

    def StreamSend(self, request_iterator, context):
        self._tick(context)
        first = next(request_iterator, None)
        if first is None or first.streamId == 0:
            context.abort(grpc.StatusCode.INVALID_ARGUMENT, "stream ID not provided")
        sid = first.streamId
        nbytes = [0]

        def gen():
            nbytes[0] += len(first.data)
            yield first.data
            for c in request_iterator:
                nbytes[0] += len(c.data)
                yield c.data

        ok = self.dev.receive_chunks(sid, gen(), abort=lambda: self._sid_aborted(sid))
        self.counters["stream_bytes_in"] += nbytes[0]
        return pb.StreamSendResponse(success=ok)

    def GetStreamStatus(self, request, context):
        return pb.GetStreamStatusResponse(status=self.dev.stream_status(request.streamId.value))

    def Memcpy(self, request, context):
        self._tick(context)
        which = request.WhichOneof("either")
        if which == "hostToDevice":
            r = request.hostToDevice
            try:
                self.dev.write(r.dstMemAddr.value, r.hostSrcData)
            except OutOfRange as e:
                context.abort(grpc.StatusCode.INVALID_ARGUMENT, str(e))
            self.counters["h2d_bytes"] += len(r.hostSrcData)
            return pb.MemcpyResponse(hostToDevice=pb.MemcpyHostToDeviceResponse(success=True))
        if which == "deviceToHost":
            r = request.deviceToHost
            addr = r.srcMemAddr.value
            n = r.numBytes or self.dev.extent(addr)
            if n == 0:
                if not self.dev.in_range(addr):
                    context.abort(grpc.StatusCode.INVALID_ARGUMENT, f"memory address {addr:#x} out of range")
                context.abort(grpc.StatusCode.INTERNAL, f"no data found at memory address {addr:#x}")
            try:
                data = self.dev.read(addr, n)
            except OutOfRange as e:
                context.abort(grpc.StatusCode.INVALID_ARGUMENT, str(e))
            self.counters["d2h_bytes"] += n
            return pb.MemcpyResponse(deviceToHost=pb.MemcpyDeviceToHostResponse(dstData=data))
        context.abort(grpc.StatusCode.INVALID_ARGUMENT, "invalid Memcpy request")

    # ---------------------------------------------------------- collectives --
    def WaitStream(self, request, context):
        tmo = (request.timeoutMs or 120000) / 1000.0
        return pb.WaitStreamResponse(status=self.dev.wait_stream(request.streamId.value, tmo))

    def Reduce(self, request, context):
        self._tick(context)
        if request.waitStreamId:
            st = self.dev.wait_stream(request.waitStreamId, 120.0)
            if st != STATUS_SUCCESS:
                context.abort(grpc.StatusCode.ABORTED, f"stream {request.waitStreamId} did not complete")
            self.dev.drop_stream(request.waitStreamId)
        try:
            self.dev.reduce(request.dstAddr, request.srcAddr, request.numBytes, request.dtype, request.op)
            if request.scale not in (0.0, 1.0):
                self.dev.scale(request.dstAddr, request.numBytes, request.dtype, request.scale)
            self.dev.synchronize()
        except OutOfRange as e:
            context.abort(grpc.StatusCode.INVALID_ARGUMENT, str(e))
        except ValueError as e:
            context.abort(grpc.StatusCode.INVALID_ARGUMENT, str(e))
        self.counters["reduces"] += 1
        return pb.ReduceResponse(success=True)

    def GetCommUniqueId(self, request, context):
        if self.dev.backend != "hip":
            context.abort(grpc.StatusCode.FAILED_PRECONDITION, "RCCL needs a GPU device")
        from ..ops.native import require_native

        return pb.GetCommUniqueIdResponse(uniqueId=require_native().rccl_unique_id())

    def CommSetup(self, request, context):
        cid = request.commId
        meta = {"rank": request.rank, "nranks": request.nranks, "peers": list(request.peerAddresses)}
        backend = "rpc"
        if request.uniqueId:
            if self.dev.backend != "hip":
                context.abort(grpc.StatusCode.FAILED_PRECONDITION, "RCCL needs a GPU device")
            from ..ops.native import require_native

            C = require_native()
            try:
                # blocking unless HIPDSML_RCCL_NONBLOCKING=1 (parallel/dist.py);
                # either way the coordinator's Abort fan-out (ncclCommAbort)
                # makes in-flight RCCL kernels return
                from ..parallel.dist import rccl_blocking_default

                comm = C.RcclComm(request.uniqueId, request.rank, request.nranks, self.dev.gpu,
                                  rccl_blocking_default())
            except Exception as e:  # init failure (peer died during bootstrap)
                context.abort(grpc.StatusCode.INTERNAL, f"RCCL init failed: {e}")
            self.comms[cid] = comm
            backend = "rccl"
        if request.storeAddress:
            backend = self._join_process_group(cid, request, context)
            if self.dev.backend == "hip" and self.pg_node_local:
                backend += "+xgmi"  # GPU peers on one node: the xGMI peer all-reduce applies
        self.comm_meta[cid] = meta
        return pb.CommSetupResponse(success=True, backend=backend)

    def _join_process_group(self, cid: int, request, context) -> str:
        """CommInit backend "pg": join a torch.distributed process group (gloo:
        control-plane collectives only) on the coordinator's TCP store, then
        -- when every rank owns a distinct GPU -- an RCCL communicator for the
        gradient all-reduce candidates.  ConfigureModel can then build the
        framework's data-parallel trainer (fused xGMI exchanges / persistent
        steps, self-tested and timed) exactly as a torchrun job would.
        Collective: the coordinator calls every device at once."""
        import datetime
        import socket

        import torch.distributed as dist

        if dist.is_initialized():
            context.abort(grpc.StatusCode.FAILED_PRECONDITION,
                          f"this device server already belongs to process group of comm {self.pg_comm}")
        host, port = request.storeAddress.rsplit(":", 1)
        tmo = datetime.timedelta(seconds=120)
        try:
            store = dist.TCPStore(host, int(port), request.nranks, is_master=False, timeout=tmo)
            dist.init_process_group("gloo", store=store, rank=request.rank, world_size=request.nranks,
                                    timeout=tmo)
        except Exception as e:
            context.abort(grpc.StatusCode.INTERNAL, f"process group rendezvous failed: {e}")
        self.pg_comm = cid
        self.pg_node_local = False
        if self.dev.backend != "hip":
            return "pg"
        from ..parallel.dist import DistContext, make_native_comm

        ctx = DistContext(rank=request.rank, world_size=request.nranks, device=self._torch_device(),
                          backend="gloo")
        err = None
        try:
            props = torch.cuda.get_device_properties(self.dev.gpu)
            ident = f"{socket.gethostname()}/{getattr(props, 'uuid', '')}/{self.dev.gpu}".encode()
            gpus = ctx.all_gather_bytes(f"hipdsml/pg{cid}/gpu", ident)
            # the xGMI exchanges need every rank on this node (IPC peer memory)
            self.pg_node_local = len({g.split(b"/", 1)[0] for g in gpus}) == 1
            if len(set(gpus)) < request.nranks:
                return "pg"  # ranks share a GPU: RCCL refuses; exchanges + gloo fallback only
            self.comms[cid] = make_native_comm(ctx)
        except Exception as e:
            err = e
        if err is not None:
            # leave the group again, or every later CommInit('pg') on this server
            # would fail with "already belongs to process group" 
            self._leave_process_group()
            context.abort(grpc.StatusCode.INTERNAL, f"RCCL init failed: {err}")
        return "rccl+pg"

    def _leave_process_group(self) -> None:
        import torch.distributed as dist

        try:
            if dist.is_initialized():
                dist.destroy_process_group()
        except Exception:  # pragma: no cover
            pass
        self.pg_comm = None
        self.pg_node_local = False

    @staticmethod
    def _ring_sid(cid: int, seq: int, step: int, src: int) -> int:
        """Deterministic stream id of a device-ring transfer (bit 62 tags ring streams)."""
        return ((1 << 62) | ((cid & 0xFFFF) << 44) | ((seq & 0xFFFFF) << 24) | ((step & 0xFFF) << 12)
                | (src & 0xFFF))

    def _sid_aborted(self, sid: int) -> bool:
        return bool((sid >> 62) & 1) and ((sid >> 44) & 0xFFFF) in {
            c & 0xFFFF for c in self._aborted_comms}

    def _wait_ring_stream(self, cid: int, sid: int, timeout: float = 120.0) -> int:
        """wait_stream in short slices, giving up as soon as the communicator is
        aborted (a peer failed): an Abort that lands between two ring steps must
        not leave this device blocked on a receive no one will send."""
        t_end = time.monotonic() + timeout
        while True:
            st = self.dev.wait_stream(sid, 0.05)
            if st != STATUS_IN_PROGRESS:
                return st
            if cid in self._aborted_comms:
                raise RuntimeError(f"communicator {cid} aborted")
            if time.monotonic() > t_end:
                return STATUS_FAILED

    # ---- RingChannel: one stream per neighbour pair, one message per ring step --
    def RingChannel(self, request_iterator, context):
        """Receiving end of a neighbour's long-lived ring stream: every message
        (comm, call sequence, step) lands in this comm's inbox until the ring
        step that needs it takes it."""
        for msg in request_iterator:
            self._tick(context)  # every ring step counts as a data-plane RPC (fault injection)
            with self._ring_cv:
                self._ring_in.setdefault(msg.commId, {})[(msg.seq, msg.step)] = msg.data
                self._ring_cv.notify_all()
            self.counters["stream_bytes_in"] += len(msg.data)
        return pb.RingAck(success=True)

    # an idle ring stream is closed after this many seconds (the next ring step
    # reopens it): each open stream holds one of the successor's gRPC workers
    RING_IDLE_S = 60.0

    def _ring_send(self, cid: int, nxt: str, msg) -> None:
        """Queue `msg` on this comm's stream to the successor, opening the
        stream (a background client call fed by the queue) on first use.  The
        stream ends when the comm is torn down or aborted, or after
        RING_IDLE_S without traffic, so a client that never destroys its
        communicator cannot pin the successor's worker threads."""
        import queue

        with self._lock:
            q = self._ring_out.get(cid)
            if q is None:
                q = queue.Queue()
                self._ring_out[cid] = q

                def gen(q=q):
                    while True:
                        try:
                            m = q.get(timeout=self.RING_IDLE_S)
                        except queue.Empty:
                            with self._lock:  # _ring_send enqueues under this lock
                                if not q.empty():
                                    continue
                                if self._ring_out.get(cid) is q:
                                    del self._ring_out[cid]
                            return
                        if m is None:
                            return
                        yield m

                def run(gen=gen):
                    try:
                        # the deadline only bounds a pathological stream; the
                        # idle close above ends it long before
                        self._peer(nxt).RingChannel(gen(), timeout=3600)
                    except Exception as e:  # peer gone: the waiting step times out / aborts
                        log.warning("ring channel of comm %d to %s closed: %s", cid, nxt, e)

                threading.Thread(target=run, daemon=True).start()
            q.put(msg)

    def _ring_recv(self, cid: int, seq: int, step: int, timeout: float = 120.0) -> bytes:
        t_end = time.monotonic() + timeout
        with self._ring_cv:
            while True:
                box = self._ring_in.get(cid, {})
                if (seq, step) in box:
                    return box.pop((seq, step))
                if cid in self._aborted_comms:
                    raise RuntimeError(f"communicator {cid} aborted")
                left = t_end - time.monotonic()
                if left <= 0:
                    raise RuntimeError(f"ring step {step} of call {seq}: nothing from the predecessor")
                self._ring_cv.wait(min(left, 0.05))

    def _ring_close(self, cid: int) -> None:
        with self._lock:
            q = self._ring_out.pop(cid, None)
        if q is not None:
            q.put(None)
        with self._ring_cv:
            self._ring_in.pop(cid, None)

    def _stream_ring(self, cid: int, addr: int, count: int, dtype: int, op: int) -> None:
        """Device-driven ring all-reduce over the neighbour streams: 2(n-1)
        steps, each ONE message on the long-lived stream to the successor (no
        per-step stream setup, no per-step thread), the predecessor's segment
        reduced in place on the device.  Same segments and order as _rpc_ring."""
        meta = self.comm_meta[cid]
        r, n, peers = meta["rank"], meta["nranks"], meta["peers"]
        seq = meta.setdefault("seq", 0)
        meta["seq"] = seq + 1
        es = DT_SIZE[dtype]
        elems = count // es
        al = 16 // es
        seg = (-(-elems // n) + al - 1) // al * al
        off = [min(i * seg, elems) * es for i in range(n + 1)]
        nxt = peers[(r + 1) % n]
        for step in range(2 * (n - 1)):
            if cid in self._aborted_comms:
                raise RuntimeError(f"communicator {cid} aborted")
            s_ = step if step < n - 1 else step - (n - 1)
            if step < n - 1:  # reduce-scatter
                si, ri = (r - s_) % n, (r - s_ - 1) % n
            else:             # all-gather, straight into place
                si, ri = (r + 1 - s_) % n, (r - s_) % n
            sl, rl = off[si + 1] - off[si], off[ri + 1] - off[ri]
            self._ring_send(cid, nxt, pb.RingChunk(commId=cid, seq=seq, step=step, srcRank=r,
                                                   data=self.dev.read(addr + off[si], sl, internal=True)
                                                   if sl else b""))
            self.counters["stream_bytes_out"] += sl
            data = self._ring_recv(cid, seq, step)
            if len(data) != rl:
                raise RuntimeError(f"ring step {step}: {len(data)} B from the predecessor, expected {rl}")
            if rl:
                if step < n - 1:
                    self.dev.reduce_bytes(addr + off[ri], data, dtype, op)
                else:
                    self.dev.write(addr + off[ri], data, internal=True, record=False)
        self.dev.synchronize()

    def _rpc_ring(self, cid: int, addr: int, count: int, dtype: int, op: int, chunk: int) -> None:
        """Device-driven ring all-reduce over gRPC streams (CPU / no-RCCL path).

        Every device runs the same 2(n-1) steps; in each it binds the receive of
        its predecessor's segment locally, pushes its own segment to its
        successor (StreamSend), waits for the incoming one and reduces it in
        place.  Stream ids are deterministic (comm, call sequence, step, sender)
        so no coordinator round trip is needed per step."""
        meta = self.comm_meta[cid]
        r, n, peers = meta["rank"], meta["nranks"], meta["peers"]
        seq = meta.setdefault("seq", 0)
        meta["seq"] = seq + 1
        es = DT_SIZE[dtype]
        elems = count // es
        al = 16 // es  # 16 B aligned segments keep the HIP reduce on its vector path
        seg = (-(-elems // n) + al - 1) // al * al
        off = [min(i * seg, elems) * es for i in range(n + 1)]
        nxt, prv = peers[(r + 1) % n], (r - 1) % n
        scratch = self.dev.scratch_addr

        def sid_of(step, src):
            return self._ring_sid(cid, seq, step, src)

        def push(sid, lo, ln):
            data = self.dev.read(addr + lo, ln, internal=True)

            def chunks():
                for o in range(0, max(ln, 1), CHUNK):
                    yield pb.DataChunk(data=data[o:o + CHUNK], streamId=sid, srcRank=r)
            ok = self._peer(nxt).StreamSend(chunks(), timeout=120).success
            self.counters["stream_bytes_out"] += ln
            if not ok:
                raise RuntimeError(f"push of stream {sid} to {nxt} failed")

        step = 0
        for s_ in range(n - 1):  # reduce-scatter
            si, ri = (r - s_) % n, (r - s_ - 1) % n
            sl, rl = off[si + 1] - off[si], off[ri + 1] - off[ri]
            sid_in = sid_of(step, prv)
            if cid in self._aborted_comms:
                raise RuntimeError(f"communicator {cid} aborted")
            if rl:
                self.dev.begin_receive(sid_in, scratch, rl, prv)
            err = []
            t = None
            if sl:
                t = threading.Thread(target=_capture, args=(err, push, sid_of(step, r), off[si], sl))
                t.start()
            if rl:
                if self._wait_ring_stream(cid, sid_in) != STATUS_SUCCESS:
                    raise RuntimeError(f"ring step {step}: receive from rank {prv} failed")
                self.dev.drop_stream(sid_in)
                self.dev.reduce(addr + off[ri], scratch, rl, dtype, op)
                self.dev.synchronize()
            if t:
                t.join()
            if err:
                raise err[0]
            step += 1
        for s_ in range(n - 1):  # all-gather, straight into place
            si, ri = (r + 1 - s_) % n, (r - s_) % n
            sl, rl = off[si + 1] - off[si], off[ri + 1] - off[ri]
            sid_in = sid_of(step, prv)
            if cid in self._aborted_comms:
                raise RuntimeError(f"communicator {cid} aborted")
            if rl:
                self.dev.begin_receive(sid_in, addr + off[ri], rl, prv)
            err = []
            t = None
            if sl:
                t = threading.Thread(target=_capture, args=(err, push, sid_of(step, r), off[si], sl))
                t.start()
            if rl:
                if self._wait_ring_stream(cid, sid_in) != STATUS_SUCCESS:
                    raise RuntimeError(f"ring step {step}: receive from rank {prv} failed")
                self.dev.drop_stream(sid_in)
            if t:
                t.join()
            if err:
                raise err[0]
            step += 1
        del chunk

    def _xgmi_allreduce(self, request, context) -> float:
        """fp32 sum over xGMI peer memory (parallel/xchg.py XgmiAllReduce,
        two-shot: reduce-scatter + all-gather in one launch) between the GPU
        device servers of a "pg" communicator: the exchange buffers' IPC handles
        travel through the process group's store.  Collective (the coordinator
        calls every device at once); returns the device time in us."""
        from ..parallel.dist import DistContext
        from ..parallel.xchg import XgmiAllReduce

        cid = request.commId
        if cid != self.pg_comm or self.dev.backend != "hip":
            context.abort(grpc.StatusCode.FAILED_PRECONDITION, "algo 'xgmi' needs GPU devices in a 'pg' comm")
        if request.dtype != DT_FLOAT32 or request.op != SUM or request.count % 16:
            context.abort(grpc.StatusCode.INVALID_ARGUMENT, "algo 'xgmi' sums fp32 buffers of 16-B multiples")
        n = request.count // 4
        ar = self._xgmi_ar.get(cid)
        if ar is None or ar.max_floats < n:
            meta = self.comm_meta[cid]
            ctx = DistContext(rank=meta["rank"], world_size=meta["nranks"], device=self._torch_device(),
                              backend="gloo")
            with torch.cuda.device(self.dev.gpu):
                ar = XgmiAllReduce(ctx, max(n, 1 << 18), algo="twoshot")
            self._xgmi_ar[cid] = ar
        t = self.dev.tensor(request.addr, request.count, torch.float32, internal=False)
        torch.cuda.synchronize(self.dev.gpu)
        t0 = time.perf_counter()
        with torch.cuda.device(self.dev.gpu):
            for _ in range(max(1, request.repeat)):
                ar(t)
            torch.cuda.synchronize(self.dev.gpu)
        us = (time.perf_counter() - t0) * 1e6 / max(1, request.repeat)
        ar.check()
        return us

    def DeviceAllReduce(self, request, context):
        self._tick(context)
        if request.algo == "xgmi":
            try:
                us = self._xgmi_allreduce(request, context)
            except RuntimeError as e:
                context.abort(grpc.StatusCode.INTERNAL, f"xGMI all-reduce failed: {e}")
            self.counters["allreduces"] += max(1, request.repeat)
            return pb.DeviceAllReduceResponse(success=True, elapsedUs=us, algo="xgmi")
        comm = self.comms.get(request.commId)
        if comm is None and request.commId in self.comm_meta:
            es = DT_SIZE.get(request.dtype, 0)
            if es == 0 or request.count % es:
                context.abort(grpc.StatusCode.INVALID_ARGUMENT, "bad dtype / count")
            try:
                self.dev.check(request.addr, request.count)
            except OutOfRange as e:
                context.abort(grpc.StatusCode.INVALID_ARGUMENT, str(e))
            t0 = time.perf_counter()
            try:
                for _ in range(max(1, request.repeat)):
                    if request.algo == "stream-ring":
                        self._stream_ring(request.commId, request.addr, request.count, request.dtype,
                                          request.op)
                    else:
                        self._rpc_ring(request.commId, request.addr, request.count, request.dtype,
                                       request.op, request.chunkBytes)
            except Exception as e:
                context.abort(grpc.StatusCode.INTERNAL, f"device ring failed: {e}")
            self.counters["allreduces"] += max(1, request.repeat)
            return pb.DeviceAllReduceResponse(success=True, elapsedUs=(time.perf_counter() - t0) * 1e6,
                                              algo=request.algo if request.algo == "stream-ring" else "rpc-ring",
                                              chunkBytes=request.chunkBytes)
        if comm is None:
            context.abort(grpc.StatusCode.FAILED_PRECONDITION, f"no communicator {request.commId} on this device")
        if comm.aborted:
            context.abort(grpc.StatusCode.ABORTED, "communicator aborted")
        es = DT_SIZE[request.dtype]
        if request.count % es:
            context.abort(grpc.StatusCode.INVALID_ARGUMENT, "count is not a multiple of the element size")
        try:
            t = self.dev.tensor(request.addr, request.count, TORCH_DTYPES[request.dtype], internal=False)
        except OutOfRange as e:
            context.abort(grpc.StatusCode.INVALID_ARGUMENT, str(e))
        algo = request.algo or "ring"
        reps = max(1, request.repeat)
        chunk = int(request.chunkBytes)
        if algo != "rccl" and chunk <= 0:
            # the in-house ring's chunk (and schedule), measured once per comm
            # and size class on this very buffer (parallel/ring_tune.py), not
            # a fixed 1 MiB: collective, every device gets the same call
            try:
                chunk = self._tuned_chunk(request.commId, comm, t)
            except Exception as e:  # noqa: BLE001
                context.abort(grpc.StatusCode.INTERNAL, f"ring chunk tuning failed: {e}")
        torch.cuda.synchronize(self.dev.gpu)
        t0 = time.perf_counter()
        try:
            with torch.cuda.device(self.dev.gpu):
                for _ in range(reps):
                    if algo == "rccl":
                        comm.allreduce_(t, request.op)
                    else:
                        comm.ring_allreduce_(t, request.op, chunk)
                torch.cuda.synchronize(self.dev.gpu)
        except Exception as e:
            context.abort(grpc.StatusCode.INTERNAL, f"all-reduce failed: {e}")
        if comm.aborted:  # an Abort landed mid-collective: the kernels returned early
            context.abort(grpc.StatusCode.ABORTED, "communicator aborted during the all-reduce")
        err = comm.async_error()
        if err not in ("", "in-progress"):
            context.abort(grpc.StatusCode.INTERNAL, f"RCCL error: {err}")
        us = (time.perf_counter() - t0) * 1e6 / reps
        self.counters["allreduces"] += reps
        return pb.DeviceAllReduceResponse(success=True, elapsedUs=us, algo=algo,
                                          chunkBytes=0 if algo == "rccl" else chunk)

    def _tuned_chunk(self, cid: int, comm, t) -> int:
        """Chunk of the in-house ring for `t`'s size class (the power of two
        at or above its byte size) on comm `cid`: tuned on the first call of
        that class with ring_tune.tune_ring_chunk (max over ranks, the
        pipelined schedule only where HIPDSML_RING_PIPELINE=1 opts in) and
        cached for the comm's life.  A 1-element class keeps RCCL's scratch
        sane: nothing below 4 KiB is tuned."""
        from ..parallel.dist import DistContext
        from ..parallel.ring_tune import tune_ring_chunk

        nbytes = t.numel() * t.element_size()
        cls = max(4096, 1 << max(0, (nbytes - 1).bit_length()))
        cache = self._ring_chunks.setdefault(cid, {})
        if cls not in cache:
            meta = self.comm_meta[cid]
            ctx = DistContext(rank=meta["rank"], world_size=meta["nranks"], device=self._torch_device(),
                              backend="gloo")
            with torch.cuda.device(self.dev.gpu):
                res = tune_ring_chunk(ctx, comm, t.view(-1), iters=10)  # restores t
            cache[cls] = int(res["best"])
            log.info("%s: comm %d ring chunk for <= %d B: %d B (%s)", self.name, cid, cls, cache[cls],
                     res.get("sweep_us"))
        return cache[cls]

    def Abort(self, request, context):
        # unblock any device-driven ring step waiting on a peer that died, and
        # keep failing that communicator's later ring steps (sticky)
        if request.commId in self.comm_meta or request.commId in self.comms:
            self._aborted_comms.add(request.commId)
            # the comm is dead for good: release the successor's stream worker
            self._ring_close(request.commId)
        self.dev.fail_pending_streams()
        ids = [request.commId] if request.commId in self.comms else list(self.comms)
        for cid in ids:
            try:
                self.comms[cid].abort()
            except Exception:  # pragma: no cover
                pass
        log.warning("%s: abort comm(s) %s: %s", self.name, ids, request.reason)
        return pb.AbortResponse(success=True)

    def CommTeardown(self, request, context):
        self._ring_close(request.commId)
        self._xgmi_ar.pop(request.commId, None)
        self.comms.pop(request.commId, None)
        self.comm_meta.pop(request.commId, None)
        if request.commId == self.pg_comm:
            if self.trainer is not None and getattr(self.trainer, "ctx", None) is not None \
                    and self.trainer.ctx.is_distributed:
                self.trainer = None  # its exchanges and self-tests belong to this group
            torch.cuda.synchronize() if self.dev.backend == "hip" else None
            self._leave_process_group()
        return pb.CommTeardownResponse(success=True)

    # -------------------------------------------------------------- training --
    def _torch_device(self) -> torch.device:
        return torch.device("cuda", self.dev.gpu) if self.dev.backend == "hip" else torch.device("cpu")

    def ConfigureModel(self, request, context):
        from ..data.mnist import load_mnist, mnist_available, synthetic_mnist
        from ..engine.trainer import MlpTrainer
        from ..models.mlp import MlpLayout, MlpSpec
        from ..parallel.dist import DistContext

        try:
            spec = MlpSpec(tuple(request.dims) or (784, 128, 64, 10))
        except ValueError as e:
            context.abort(grpc.StatusCode.INVALID_ARGUMENT, str(e))
        batch = request.batch or 64
        world = max(1, request.worldSize)
        rank = request.rank
        n = request.numSamples or 60032
        if request.dataset in ("", "synthetic"):
            ds = synthetic_mnist(n, seed=request.dataSeed + rank, dim=spec.dims[0])
        elif request.dataset.startswith("mnist") and mnist_available():
            ds = load_mnist(split="t10k").shard(rank, world)
        else:
            context.abort(grpc.StatusCode.INVALID_ARGUMENT, f"dataset {request.dataset!r} unavailable")
        layout = MlpLayout(spec, batch, max(1, len(ds) // batch))
        params = None
        if request.weightsAddr:
            nb = spec.num_params * 4
            raw = self.dev.read(request.weightsAddr, nb)
            import numpy as np

            params = layout.from_reference(np.frombuffer(raw, dtype=np.float32))
        pg = world > 1 and request.commId == self.pg_comm
        ctx = DistContext(rank=rank, world_size=world, device=self._torch_device(),
                          backend="gloo" if pg else "none")
        comm = self.comms.get(request.commId) if world > 1 else None
        host_ar = None
        if pg:
            import torch.distributed as dist

            if dist.get_world_size() != world or dist.get_rank() != rank:
                context.abort(grpc.StatusCode.FAILED_PRECONDITION,
                              f"comm {request.commId}'s process group is rank {dist.get_rank()} of "
                              f"{dist.get_world_size()}, not {rank} of {world}")
        elif world > 1 and comm is None:
            if self.dev.backend == "hip":
                context.abort(grpc.StatusCode.FAILED_PRECONDITION,
                              "data-parallel TrainSteps needs an RCCL comm (CommInit backend=rccl)")
            meta = self.comm_meta.get(request.commId)
            if meta is None or meta["nranks"] != world or meta["rank"] != rank:
                context.abort(grpc.StatusCode.FAILED_PRECONDITION,
                              f"data-parallel TrainSteps on host devices needs comm {request.commId} "
                              f"set up with rank {rank} of {world} (CommInit backend=rpc)")
            try:
                host_ar = self._host_grad_allreduce(request.commId, world, layout.nparams * 4)
            except ValueError as e:  # the gradient does not fit the ring scratch window
                context.abort(grpc.StatusCode.INVALID_ARGUMENT, str(e))
        try:
            # a process group runs the framework's own data-parallel choice
            # (sync "auto": every fused exchange self-tested and timed, RCCL
            # or a gloo all-reduce as the fallback)
            sync = request.sync or ("auto" if pg else "rccl")
            if pg and self.dev.backend != "hip":
                sync = "rccl"  # host replicas: the torch step's all-reduce over the group
            self.trainer = MlpTrainer(spec, ds, batch=batch, lr=request.lr or 0.01, ctx=ctx,
                                      seed=request.seed, momentum=request.momentum,
                                      graph_steps=request.graphSteps, params=params,
                                      external_comm=comm, sync=sync, grad_allreduce=host_ar,
                                      auto_fallback="rccl" if (comm is not None or not pg) else "torch",
                                      # the exchanges need every server on this node, whatever
                                      # the group's backend (RCCL stays the fallback candidate)
                                      node_local=self.pg_node_local if pg else None)
        except (ValueError, RuntimeError) as e:
            context.abort(grpc.StatusCode.INVALID_ARGUMENT, str(e))
        return pb.ConfigureModelResponse(success=True, numParams=spec.num_params,
                                         batchesPerEpoch=self.trainer.nbatches,
                                         paramBytes=layout.nparams * 4,
                                         sync=self.trainer.sync_active,
                                         syncTimesJson=json.dumps(self.trainer.sync_times or {}))

    def _host_grad_allreduce(self, cid: int, n: int, nbytes: int):
        """Gradient sum for host replicas trained by TrainSteps: each step's flat
        fp32 gradient is staged in this device's private scratch window, summed
        over the communicator by the device-driven gRPC ring (`_rpc_ring`, the
        same transfers as DeviceAllReduce) and read back.  The ring's receive
        segment sits at the bottom of the window, the gradient right above it.
        Every replica applies the same summed gradient, so they stay identical
        (the reference instead broadcast weights after each step,
        client.go:596-647)."""
        seg = (-(-(nbytes // 4) // n) + 3) // 4 * 16
        gaddr = self.dev.scratch_addr + (seg + 255) // 256 * 256
        if gaddr + nbytes > self.dev.max_addr + self.dev.scratch_size:
            need = gaddr + nbytes - self.dev.max_addr
            raise ValueError(f"gradient of {nbytes} B does not fit the {self.dev.scratch_size} B "
                             f"ring scratch window (needs {need} B: start the device server with "
                             f"a larger --scratch-bytes)")

        def allreduce(g: torch.Tensor) -> None:
            self.dev.write(gaddr, g.detach().float().contiguous().numpy().tobytes(), internal=True,
                           record=False)
            self._rpc_ring(cid, gaddr, nbytes, DT_FLOAT32, SUM, 0)
            g.copy_(torch.frombuffer(bytearray(self.dev.read(gaddr, nbytes, internal=True)),
                                     dtype=torch.float32).view_as(g))
            self.counters["allreduces"] += 1

        return allreduce

    def _need_trainer(self, context):
        if self.trainer is None:
            context.abort(grpc.StatusCode.FAILED_PRECONDITION, "ConfigureModel first")
        return self.trainer

    def TrainSteps(self, request, context):
        tr = self._need_trainer(context)
        t0 = time.perf_counter()
        try:
            tr.train_steps(int(request.steps))
            tr.synchronize()
        except Exception as e:
            context.abort(grpc.StatusCode.INTERNAL, f"train step failed: {e}")
        us = (time.perf_counter() - t0) * 1e6
        st = tr.read_stats()
        self.counters["train_steps"] += int(request.steps)
        return pb.TrainStepsResponse(success=True, lossSum=st.loss_sum, correct=st.correct,
                                     count=st.count, elapsedUs=us, stepsDone=tr.steps_done)

    def Evaluate(self, request, context):
        from ..data.mnist import load_mnist, mnist_available, synthetic_mnist

        tr = self._need_trainer(context)
        if request.dataset.startswith("mnist") and mnist_available():
            ds = load_mnist(split="t10k", limit=request.numSamples or None)
        else:
            ds = synthetic_mnist(request.numSamples or 10000, seed=request.seed or 777,
                                 dim=tr.spec.dims[0])
        ev = tr.evaluate(ds)
        return pb.EvaluateResponse(success=True, accuracy=ev["accuracy"], loss=ev["loss"], count=ev["n"])

    def RunForward(self, request, context):
        tr = self._need_trainer(context)
        rows = request.numRows or tr.batch
        d0 = tr.spec.dims[0]
        try:
            X = self.dev.tensor(request.inputAddr, rows * d0 * 4, torch.float32).view(rows, d0)
            y = (self.dev.tensor(request.labelsAddr, rows * 4, torch.int32)
                 if request.labelsAddr else None)
        except OutOfRange as e:
            context.abort(grpc.StatusCode.INVALID_ARGUMENT, str(e))
        X = X.clone()
        y = y.clone() if y is not None else None
        # GPU: the fused HIP forward kernels (K_A + row chain, logits kept);
        # host devices: the fp32 torch reference
        logits, loss_sum, corr = tr.forward_logits(X, y)
        loss = correct = 0.0
        if y is not None:
            loss, correct = float(loss_sum) / rows, int(corr)
        if request.outputAddr:
            self.dev.write(request.outputAddr, logits.detach().float().cpu().numpy().tobytes(),
                           internal=True)
        self._fwd_cache = (X, y)
        return pb.RunForwardResponse(success=True, loss=loss, correct=int(correct))

    def RunBackward(self, request, context):
        tr = self._need_trainer(context)
        if self._fwd_cache is None or self._fwd_cache[1] is None:
            context.abort(grpc.StatusCode.FAILED_PRECONDITION, "RunForward with labels first")
        X, y = self._fwd_cache
        g = tr.batch_gradients(X, y)
        data = g.detach().float().cpu().numpy().tobytes()
        try:
            self.dev.write(request.gradientAddr, data, internal=True)
        except OutOfRange as e:
            context.abort(grpc.StatusCode.INVALID_ARGUMENT, str(e))
        return pb.RunBackwardResponse(success=True, numBytes=len(data))

    def ApplyGradients(self, request, context):
        tr = self._need_trainer(context)
        nb = tr.layout.nparams * 4
        try:
            g = self.dev.tensor(request.gradientAddr, nb, torch.float32).to(tr.device)
        except OutOfRange as e:
            context.abort(grpc.StatusCode.INVALID_ARGUMENT, str(e))
        tr.apply_gradients(g, request.scale or 1.0)
        return pb.ApplyGradientsResponse(success=True)

    def GetStats(self, request, context):
        d = dict(self.counters)
        d.update({"device_id": self.dev.device_id, "backend": self.dev.backend,
                  "comms": sorted(self.comms), "steps_done": getattr(self.trainer, "steps_done", 0)})
        d["rpc_latency"] = {m: h.summary() for m, h in getattr(self, "rpc_latency", {}).items()
                            if h.n}
        return pb.GetStatsResponse(json=json.dumps(d))


def _capture(err, fn, *args):
    try:
        fn(*args)
    except Exception as e:  # surfaced by the caller after join()
        err.append(e)


def start_device_server(device_id: int, mem_size: int, address: str = "127.0.0.1:0",
                        backend: str = "auto", gpu: int = 0, max_workers: int = 32,
                        scratch_size: Optional[int] = None):
    """Start one device server; returns (grpc_server, address, servicer).
    `scratch_size` sizes the private ring window above max_addr (None: 64 MiB
    on a GPU, 1 MiB on the host)."""
    dev = make_device(device_id, mem_size, backend, gpu=gpu, scratch_size=scratch_size)
    svc = GPUDeviceServicer(dev)
    server, addr = serve("GPUDevice", svc, address, max_workers=max_workers)
    svc.server = server
    log.info("GPU Device server listening on %s with device ID %d (%s)", addr, device_id, dev.backend)
    return server, addr, svc

"""Device memory + stream runtimes behind the GPUDevice servicer.

``HipDevice``  — a real MI355X: HBM arena, pinned copy engine and stream table
                 from the native extension (csrc/runtime/device_runtime.cpp);
                 reductions run as HIP kernels on the GPU.
``HostDevice`` — the CPU simulation used by the plumbing tests (BASELINE
                 config 1: "3 simulated CPU device-servers"), numpy-backed.

Both expose the reference's MemAddr space ``[0x1000, 0x1000 + mem_size)``
(``gpu_device_server.go:39-62``) and, directly above it, a private scratch
window ``[max_addr, max_addr + scratch)`` used by the device-to-device ring as
its receive buffer, so collectives never clobber user memory.

Fixes vs the reference: memory is linear (not a map of blobs),
writes may update part of a previous write, D2H returns exactly ``numBytes``
(``numBytes == 0`` keeps the "whole last write" behaviour, Q12), streams are
freed after completion (Q11).
"""
from __future__ import annotations

import threading
import time
from dataclasses import dataclass, field
from typing import Dict, Optional

import numpy as np
import torch

BASE_ADDR = 0x1000
STATUS_IN_PROGRESS, STATUS_SUCCESS, STATUS_FAILED = 0, 1, 2

# gpu_sim DataType -> numpy / torch / native dtype ids
NP_DTYPES = {0: np.float32, 1: np.uint8, 2: None, 3: np.float16, 4: np.int32}
TORCH_DTYPES = {0: torch.float32, 1: torch.uint8, 2: torch.bfloat16, 3: torch.float16, 4: torch.int32}
NATIVE_DTYPE = {0: 0, 1: 3, 2: 1, 3: 2, 4: 4}  # -> dsml::DType
DT_SIZE = {0: 4, 1: 1, 2: 2, 3: 2, 4: 4}


class OutOfRange(IndexError):
    pass


@dataclass
class _Stream:
    send_addr: int = 0
    num_bytes: int = 0
    dst_rank: int = 0
    recv_addr: int = 0
    src_rank: int = 0
    initiated_recv: bool = False
    received: int = 0
    status: int = STATUS_IN_PROGRESS
    bound: threading.Event = field(default_factory=threading.Event)
    done: threading.Event = field(default_factory=threading.Event)


class _Device:
    """Shared bookkeeping: address checks, extents, stream table."""

    backend = "abstract"

    def __init__(self, device_id: int, mem_size: int, scratch_size: int):
        self.device_id = int(device_id)
        self.mem_size = int(mem_size)
        self.scratch_size = int(scratch_size)
        self.min_addr = BASE_ADDR
        self.max_addr = BASE_ADDR + self.mem_size
        self.scratch_addr = self.max_addr
        self._extents: Dict[int, int] = {}
        self._lock = threading.Lock()
        self._streams: Dict[int, _Stream] = {}
        self._next_sid = 1

    # -- address checks -------------------------------------------------------
    def check(self, addr: int, n: int, internal: bool = False) -> None:
        hi = self.max_addr + (self.scratch_size if internal else 0)
        if addr < self.min_addr or addr > hi or n > hi - addr:
            raise OutOfRange(f"memory address out of range: addr={addr:#x} bytes={n} "
                             f"valid=[{self.min_addr:#x},{hi:#x})")

    def in_range(self, addr: int) -> bool:
        return self.min_addr <= addr < self.max_addr

    # -- streams (BeginSend / BeginReceive / StreamSend / GetStreamStatus) -----
    def new_stream_id(self) -> int:
        with self._lock:
            sid = (self.device_id << 32) | self._next_sid
            self._next_sid += 1
            return sid

    def begin_send(self, send_addr: int, num_bytes: int, dst_rank: int) -> int:
        sid = self.new_stream_id()
        with self._lock:
            self._streams[sid] = _Stream(send_addr=send_addr, num_bytes=num_bytes, dst_rank=dst_rank)
        return sid

    def begin_receive(self, sid: int, recv_addr: int, num_bytes: int, src_rank: int,
                      create: bool = True) -> None:
        with self._lock:
            st = self._streams.get(sid)
            if st is None:
                if not create:
                    raise KeyError(f"stream not found: {sid}")
                st = _Stream(num_bytes=num_bytes)
                self._streams[sid] = st
            n = num_bytes or st.num_bytes
            st.num_bytes = n
            self.check(recv_addr, n, internal=True)
            st.recv_addr, st.src_rank, st.initiated_recv = recv_addr, src_rank, True
            st.bound.set()

    def stream(self, sid: int) -> Optional[_Stream]:
        with self._lock:
            return self._streams.get(sid)

    def set_status(self, sid: int, status: int) -> None:
        with self._lock:
            st = self._streams.get(sid)
            if st is not None:
                st.status = status
                if status != STATUS_IN_PROGRESS:
                    st.done.set()

    def wait_stream(self, sid: int, timeout: float) -> int:
        """Block until stream `sid` completes (event-driven, no polling)."""
        with self._lock:
            st = self._streams.setdefault(sid, _Stream())
        st.done.wait(timeout)
        return st.status

    def stream_status(self, sid: int) -> int:
        st = self.stream(sid)
        return STATUS_FAILED if st is None else st.status

    def receive_chunks(self, sid: int, chunks, wait_s: float = 30.0, abort=None) -> bool:
        """Write streamed chunks at the bound receive address.  A sender that
        races ahead of BeginReceive waits (bounded, and no longer than until
        `abort()` turns true) for the binding."""
        st = self.stream(sid)
        if st is None:
            with self._lock:
                st = self._streams.setdefault(sid, _Stream())
        t_end = time.monotonic() + wait_s
        while not st.bound.wait(0.05):
            if time.monotonic() > t_end or (abort is not None and abort()):
                st.status = STATUS_FAILED
                st.done.set()
                return False
        off = 0
        ok = True
        for data in chunks:
            if off + len(data) > st.num_bytes:
                ok = False
                break
            self.write(st.recv_addr + off, data, internal=True, record=False)
            off += len(data)
        ok = ok and off == st.num_bytes and st.initiated_recv
        st.received = off
        st.status = STATUS_SUCCESS if ok else STATUS_FAILED
        st.done.set()
        if ok:
            self.record_extent(st.recv_addr, off)
        return ok

    def gc_streams(self, keep_last: int = 4096) -> None:
        with self._lock:
            done = [k for k, v in self._streams.items() if v.status != STATUS_IN_PROGRESS]
            for k in done[:-keep_last] if len(done) > keep_last else []:
                del self._streams[k]

    def fail_pending_streams(self) -> None:
        with self._lock:
            for st in self._streams.values():
                if st.status == STATUS_IN_PROGRESS:
                    st.status = STATUS_FAILED
                    st.bound.set()
                    st.done.set()

    def drop_stream(self, sid: int) -> None:
        with self._lock:
            self._streams.pop(sid, None)

    # -- extents ---------------------------------------------------------------
    def record_extent(self, addr: int, n: int) -> None:
        with self._lock:
            self._extents[addr] = n

    def extent(self, addr: int) -> int:
        with self._lock:
            return self._extents.get(addr, 0)

    # -- to implement ------------------------------------------------------------
    def write(self, addr: int, data: bytes, internal: bool = False, record: bool = True) -> None:
        raise NotImplementedError

    def read(self, addr: int, n: int, internal: bool = False) -> bytes:
        raise NotImplementedError

    def reduce(self, dst: int, src: int, nbytes: int, dtype: int, op: int) -> None:
        raise NotImplementedError

    def scale(self, addr: int, nbytes: int, dtype: int, alpha: float) -> None:
        raise NotImplementedError

    def reduce_bytes(self, dst: int, data: bytes, dtype: int, op: int) -> None:
        """dst <- dst (op) data for bytes that arrived off the wire (a ring
        step's segment); default: through the private scratch window."""
        self.write(self.scratch_addr, data, internal=True, record=False)
        self.reduce(dst, self.scratch_addr, len(data), dtype, op)

    def tensor(self, addr: int, nbytes: int, dtype: torch.dtype, internal: bool = True) -> torch.Tensor:
        raise NotImplementedError

    def synchronize(self) -> None:
        pass


class HostDevice(_Device):
    backend = "host"

    def __init__(self, device_id: int, mem_size: int, scratch_size: int = 1 << 20):
        super().__init__(device_id, mem_size, scratch_size)
        self._mem = torch.zeros(mem_size + scratch_size, dtype=torch.uint8)
        self._np = self._mem.numpy()

    def _off(self, addr: int) -> int:
        return addr - self.min_addr

    def write(self, addr, data, internal=False, record=True):
        self.check(addr, len(data), internal)
        o = self._off(addr)
        self._np[o:o + len(data)] = np.frombuffer(data, dtype=np.uint8)
        if record:
            self.record_extent(addr, len(data))

    def read(self, addr, n, internal=False):
        self.check(addr, n, internal)
        o = self._off(addr)
        return self._np[o:o + n].tobytes()

    def tensor(self, addr, nbytes, dtype, internal=True):
        self.check(addr, nbytes, internal)
        o = self._off(addr)
        return self._mem[o:o + nbytes].view(dtype)

    def reduce(self, dst, src, nbytes, dtype, op):
        from ..ops.functional import reduce_ref

        td = TORCH_DTYPES[dtype]
        if nbytes % DT_SIZE[dtype]:
            raise ValueError("byte count is not a multiple of the element size")
        a = self.tensor(dst, nbytes, td)
        b = self.tensor(src, nbytes, td)
        a.copy_(reduce_ref(a, b, op))

    def scale(self, addr, nbytes, dtype, alpha):
        t = self.tensor(addr, nbytes, TORCH_DTYPES[dtype])
        t.copy_((t.float() * alpha).to(t.dtype))

    def reduce_bytes(self, dst, data, dtype, op):
        # host memory: reduce straight from the received buffer (no scratch copy)
        from ..ops.functional import reduce_ref

        td = TORCH_DTYPES[dtype]
        if len(data) % DT_SIZE[dtype]:
            raise ValueError("byte count is not a multiple of the element size")
        a = self.tensor(dst, len(data), td)
        b = torch.frombuffer(bytearray(data) if isinstance(data, bytes) else data, dtype=td)
        if op == 0 and td not in (torch.uint8, torch.bfloat16, torch.float16):  # SUM
            a.add_(b)
        else:
            a.copy_(reduce_ref(a, b, op))


class _CudaArrayView:
    """__cuda_array_interface__ shim so torch can alias arena memory."""

    def __init__(self, ptr: int, nbytes: int):
        self.__cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1",
                                         "data": (ptr, False), "version": 2}


class HipDevice(_Device):
    backend = "hip"

    def __init__(self, device_id: int, mem_size: int, scratch_size: int = 64 << 20,
                 gpu: int = 0, staging_bytes: int = 16 << 20):
        super().__init__(device_id, mem_size, scratch_size)
        from ..ops.native import require_native

        C = require_native()
        self.gpu = int(gpu)
        torch.cuda.set_device(self.gpu)
        self.arena = C.DeviceArena(self.gpu, mem_size + scratch_size, BASE_ADDR)
        self.copy = C.CopyEngine(self.gpu, staging_bytes)
        self._views: dict = {}

    def write(self, addr, data, internal=False, record=True):
        self.check(addr, len(data), internal)
        self.copy.h2d(self.arena, addr, bytes(data))
        if record:
            self.record_extent(addr, len(data))

    def read(self, addr, n, internal=False):
        self.check(addr, n, internal)
        return self.copy.d2h(self.arena, addr, n)

    def reduce(self, dst, src, nbytes, dtype, op):
        if nbytes % DT_SIZE[dtype]:
            raise ValueError("byte count is not a multiple of the element size")
        self.check(dst, nbytes, True)
        self.check(src, nbytes, True)
        self.arena.reduce(dst, src, nbytes, NATIVE_DTYPE[dtype], op)

    def tensor(self, addr, nbytes, dtype, internal=True):
        self.check(addr, nbytes, internal)
        # views of the (never moving) arena are cached: building one through
        # __cuda_array_interface__ costs tens of us of Python per RPC
        key = (addr, nbytes, dtype)
        t = self._views.get(key)
        if t is not None:
            return t
        ptr = self.arena.ptr(addr, nbytes)
        with torch.cuda.device(self.gpu):
            raw = torch.as_tensor(_CudaArrayView(ptr, nbytes), device=f"cuda:{self.gpu}")
        t = raw.view(dtype)
        if len(self._views) >= 256:
            self._views.clear()
        self._views[key] = t
        return t

    def scale(self, addr, nbytes, dtype, alpha):
        from ..ops.functional import scale_

        scale_(self.tensor(addr, nbytes, TORCH_DTYPES[dtype]), alpha)
        torch.cuda.synchronize(self.gpu)

    def synchronize(self) -> None:
        torch.cuda.synchronize(self.gpu)


def make_device(device_id: int, mem_size: int, backend: str = "auto", gpu: int = 0,
                scratch_size: Optional[int] = None) -> _Device:
    if backend == "auto":
        backend = "hip" if torch.cuda.is_available() else "host"
    if backend == "hip":
        return HipDevice(device_id, mem_size, scratch_size or (64 << 20), gpu=gpu)
    if backend == "host":
        return HostDevice(device_id, mem_size, scratch_size or (1 << 20))
    raise ValueError(f"unknown device backend {backend}")

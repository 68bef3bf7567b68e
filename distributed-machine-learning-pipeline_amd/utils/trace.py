"""Tracing: roctx ranges around training / RPC phases.

The reference has no tracing (only log timestamps and ``time.Now()``
around NaiveAllReduce, ``gpu_coordinator_server.go:658,706-707``).  Ranges go
through the native extension's roctx bindings (``librocprofiler-sdk-roctx``),
so ``rocprofv3 --marker-trace`` shows them on the same timeline as the HIP
kernels.  Enabled by ``HIPDSML_TRACE=1`` or :func:`enable`; when disabled,
or on a host without the extension, every call is a cheap no-op.
"""
from __future__ import annotations

import contextlib
import functools
import os
import threading
import time
from typing import Callable, Dict, List, Optional, Tuple

_enabled = os.environ.get("HIPDSML_TRACE", "0") not in ("", "0", "false")
_native = None
_lock = threading.Lock()
# host-side record of ranges (name, start, duration) when recording is on
_records: List[Tuple[str, float, float]] = []
_recording = False


def _lib():
    global _native
    if _native is None:
        try:
            from ..ops.native import load_native

            _native = load_native() or False
        except Exception:
            _native = False
    return _native or None


def enable(on: bool = True, record: bool = False) -> None:
    global _enabled, _recording
    _enabled, _recording = on, record


def enabled() -> bool:
    return _enabled


@contextlib.contextmanager
def trace_range(name: str):
    if not _enabled:
        yield
        return
    lib = _lib()
    t0 = time.perf_counter()
    if lib is not None:
        lib.roctx_push(name)
    try:
        yield
    finally:
        if lib is not None:
            lib.roctx_pop()
        if _recording:
            with _lock:
                _records.append((name, t0, time.perf_counter() - t0))


def traced(name: Optional[str] = None) -> Callable:
    def deco(fn):
        label = name or fn.__qualname__

        @functools.wraps(fn)
        def wrapper(*a, **k):
            with trace_range(label):
                return fn(*a, **k)
        return wrapper
    return deco


def mark(name: str) -> None:
    if _enabled:
        lib = _lib()
        if lib is not None:
            lib.roctx_mark(name)


def records(clear: bool = False) -> List[Tuple[str, float, float]]:
    with _lock:
        out = list(_records)
        if clear:
            _records.clear()
    return out


def summary() -> Dict[str, Dict[str, float]]:
    agg: Dict[str, Dict[str, float]] = {}
    for name, _, dt in records():
        a = agg.setdefault(name, {"n": 0, "total_s": 0.0})
        a["n"] += 1
        a["total_s"] += dt
    return agg

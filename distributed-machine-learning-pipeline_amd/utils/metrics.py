"""Metrics / logging / observability.

Reference: ``log.Printf`` at 44 sites, the epoch line
``Epoch %d complete: Avg Loss: %.4f, Accuracy: %.2f%%`` (``client.go:650-652``),
a progress bar with it/s (``client.go:584-590``) and ``totalTimeMs`` in the
NaiveAllReduce response (``gpu_sim.proto:240-244``) — SURVEY §5.

Here:
  * :class:`MetricsLogger` — JSON-lines records (one object per line, with
    wall time, rank and an event name) to a file or stdout, rank-0 only by
    default so a DP job writes one stream.
  * :class:`Progress` — a terminal progress line with it/s and samples/s
    (throttled; never on the hot path: it only reads host counters).
  * :class:`StepTimer` — host wall-clock timer, and :class:`GpuTimer`, which
    brackets work with hip events (torch.cuda.Event) so GPU time is measured
    without synchronising inside the loop.
  * :class:`Histogram` — fixed log2 buckets for RPC / collective latencies.
"""
from __future__ import annotations

import json
import math
import os
import sys
import threading
import time
from typing import IO, Any, Dict, List, Optional


class MetricsLogger:
    def __init__(self, path: str = "", rank: int = 0, all_ranks: bool = False,
                 static: Optional[Dict[str, Any]] = None):
        self.rank = rank
        self.enabled = bool(path) and (all_ranks or rank == 0)
        self.static = dict(static or {})
        self._fh: Optional[IO[str]] = None
        self._own = False
        self._lock = threading.Lock()
        if self.enabled:
            if path == "-":
                self._fh = sys.stdout
            else:
                d = os.path.dirname(os.path.abspath(path))
                os.makedirs(d, exist_ok=True)
                self._fh = open(path, "a", buffering=1)
                self._own = True
        self.records = 0

    def log(self, event: str, **values: Any) -> None:
        if not self.enabled:
            return
        rec = {"ts": round(time.time(), 6), "rank": self.rank, "event": event, **self.static}
        for k, v in values.items():
            if isinstance(v, float):
                v = v if math.isfinite(v) else None
            rec[k] = v
        line = json.dumps(rec, default=str)
        with self._lock:
            self._fh.write(line + "\n")
            self._fh.flush()
            self.records += 1

    def close(self) -> None:
        if self._own and self._fh is not None:
            self._fh.close()
        self._fh = None
        self.enabled = False

    def __enter__(self) -> "MetricsLogger":
        return self

    def __exit__(self, *exc) -> None:
        self.close()


def read_jsonl(path: str) -> List[Dict[str, Any]]:
    with open(path) as fh:
        return [json.loads(line) for line in fh if line.strip()]


class Progress:
    """``[=====>    ] 412/937 (1234.5 it/s, 79008 samples/s)`` on a tty-like stream."""

    def __init__(self, total: int, desc: str = "", samples_per_it: int = 0, stream=None,
                 min_interval: float = 0.5, width: int = 30, enabled: bool = True):
        self.total, self.desc, self.spi = total, desc, samples_per_it
        self.stream = stream or sys.stderr
        self.min_interval, self.width, self.enabled = min_interval, width, enabled
        self.n = 0
        self.t0 = time.perf_counter()
        self._last = 0.0
        self._shown = -1

    def rate(self) -> float:
        dt = time.perf_counter() - self.t0
        return self.n / dt if dt > 0 else 0.0

    def render(self) -> str:
        frac = min(1.0, self.n / self.total) if self.total else 1.0
        fill = int(frac * self.width)
        bar = "=" * fill + (">" if fill < self.width else "") + " " * max(0, self.width - fill - 1)
        r = self.rate()
        extra = f", {r * self.spi:.0f} samples/s" if self.spi else ""
        return f"{self.desc}[{bar}] {self.n}/{self.total} ({r:.1f} it/s{extra})"

    def update(self, k: int = 1) -> None:
        self.n += k
        now = time.perf_counter()
        if self.enabled and (now - self._last >= self.min_interval or self.n >= self.total):
            self._last = now
            self._shown = self.n
            self.stream.write("\r" + self.render())
            self.stream.flush()

    def close(self) -> None:
        if self.enabled:
            self.stream.write(("" if self._shown == self.n else "\r" + self.render()) + "\n")
            self.stream.flush()


class StepTimer:
    def __init__(self):
        self.t0 = time.perf_counter()

    def lap(self) -> float:
        t = time.perf_counter()
        dt, self.t0 = t - self.t0, t
        return dt


class GpuTimer:
    """Elapsed GPU time between two points of a stream (hip events)."""

    def __init__(self, device=None):
        import torch

        self._torch = torch
        self.device = device
        self.start_ev = torch.cuda.Event(enable_timing=True)
        self.end_ev = torch.cuda.Event(enable_timing=True)

    def start(self, stream=None) -> None:
        self.start_ev.record(stream)

    def stop(self, stream=None) -> None:
        self.end_ev.record(stream)

    def elapsed_ms(self) -> float:
        self.end_ev.synchronize()
        return self.start_ev.elapsed_time(self.end_ev)


class Histogram:
    """Latency histogram with log2 buckets (µs); thread-safe."""

    def __init__(self, name: str = ""):
        self.name = name
        self.counts: Dict[int, int] = {}
        self.n = 0
        self.total = 0.0
        self.min = math.inf
        self.max = 0.0
        self._lock = threading.Lock()

    def add(self, seconds: float) -> None:
        us = seconds * 1e6
        b = 0 if us < 1 else int(math.log2(us)) + 1
        with self._lock:
            self.counts[b] = self.counts.get(b, 0) + 1
            self.n += 1
            self.total += us
            self.min = min(self.min, us)
            self.max = max(self.max, us)

    def quantile(self, q: float) -> float:
        """Upper bucket edge (µs) containing quantile q."""
        with self._lock:
            if not self.n:
                return 0.0
            target = q * self.n
            acc = 0
            for b in sorted(self.counts):
                acc += self.counts[b]
                if acc >= target:
                    return float(2 ** b)
            return self.max

    def summary(self) -> Dict[str, Any]:
        return {"name": self.name, "n": self.n, "mean_us": self.total / self.n if self.n else 0.0,
                "min_us": self.min if self.n else 0.0, "max_us": self.max,
                "p50_us": self.quantile(0.5), "p99_us": self.quantile(0.99)}

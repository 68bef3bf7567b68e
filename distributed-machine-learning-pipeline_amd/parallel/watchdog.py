"""Failure detector for the data plane of a data-parallel job.

The reference detects failures only in its control plane: a 5 s ticker pings
every device with GetDeviceMetadata (2 s timeout) and marks the communicator
FAILED on the first miss (``gpu_coordinator_server.go:57,69-119``).  Its
"collectives" are gRPC calls with deadlines, so nothing can hang in a kernel.

Here gradients move GPU<->GPU inside RCCL kernels and xGMI exchange kernels,
where a dead or stalled peer would leave the survivors spinning.  Three layers
keep a fault from turning into a hang:

* xGMI exchange kernels bound every flag wait (``kernels/common.h``
  ``poll_flag_ge``) and set an error word the host checks after each sync;
* this watchdog thread polls ``ncclCommGetAsyncError`` of every registered
  RCCL communicator every ``interval`` seconds (communicators are blocking by
  default, ``HIPDSML_RCCL_NONBLOCKING=1`` makes them non-blocking so no RCCL
  host call can wait unboundedly either);
* every blocking host section of the job (stream syncs, collectives on the
  process group) runs under :meth:`Watchdog.guard`.  A section that exceeds
  ``timeout`` seconds — or any RCCL async error — makes the watchdog abort
  every registered communicator (``ncclCommAbort``: in-flight RCCL kernels
  return) and record the fault; the guarded call then raises
  :class:`CommFault` in the main thread.  If the main thread is still stuck
  ``grace`` seconds later the watchdog ends the process with exit code
  :data:`EXIT_CODE` (``os._exit``: no re-exec, nothing else runs).

The process exits non-zero in every case; the coordinator / launcher sees the
rank die, exactly like the reference's FAILED-is-terminal semantics.
"""
from __future__ import annotations

import contextlib
import logging
import os
import sys
import threading
import time
from typing import Callable, List, Optional

log = logging.getLogger("hipdsml.watchdog")

EXIT_CODE = 70  # EX_SOFTWARE: the watchdog ended the process


class CommFault(RuntimeError):
    """A collective / peer failed or stalled; the communicators are aborted."""


class Watchdog:
    def __init__(self, timeout: float = 300.0, interval: float = 0.1, grace: float = 10.0,
                 name: str = "", exit_on_stuck: bool = True):
        if timeout <= 0:
            raise ValueError("watchdog timeout must be > 0")
        self.timeout = float(timeout)
        self.interval = float(interval)
        self.grace = float(grace)
        self.name = name
        self.exit_on_stuck = exit_on_stuck
        self._comms: List[object] = []
        self._aborters: List[Callable[[], None]] = []
        self._lock = threading.Lock()
        self._section: Optional[str] = None
        self._since = 0.0
        self._fault: Optional[str] = None
        self._fault_at = 0.0
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._run, name=f"hipdsml-watchdog{name}", daemon=True)
        self._thread.start()

    # -- registration ---------------------------------------------------------
    def watch_comm(self, comm) -> None:
        """A native RCCL communicator (``_C.RcclComm``): polled for async
        errors and aborted on any fault."""
        with self._lock:
            self._comms.append(comm)

    def unwatch_comm(self, comm) -> None:
        """Stop polling / aborting `comm` (before it is destroyed)."""
        with self._lock:
            self._comms = [c for c in self._comms if c is not comm]

    def on_fault(self, fn: Callable[[], None]) -> None:
        """Extra abort action (e.g. a process-group abort)."""
        with self._lock:
            self._aborters.append(fn)

    # -- guarded sections ---------------------------------------------------------
    @contextlib.contextmanager
    def guard(self, what: str):
        """Run a blocking section under the stall timeout; raises CommFault if
        the watchdog declared a fault during (or before) it."""
        self.check()
        with self._lock:
            outer = self._section
            if outer is None:
                self._section, self._since = what, time.monotonic()
        try:
            yield
        except Exception as e:  # the section itself failed (e.g. a peer closed the socket)
            self.check()
            raise CommFault(f"{what} failed: {e}") from e
        finally:
            with self._lock:
                if outer is None:
                    self._section = None
        self.check()

    def check(self) -> None:
        if self._fault is not None:
            raise CommFault(self._fault)

    @property
    def fault(self) -> Optional[str]:
        return self._fault

    def declare(self, reason: str) -> None:
        """Record a fault and abort every registered communicator (idempotent)."""
        with self._lock:
            if self._fault is not None:
                return
            self._fault = reason
            self._fault_at = time.monotonic()
            comms, aborters = list(self._comms), list(self._aborters)
        log.error("watchdog%s: %s — aborting %d communicator(s)", self.name, reason, len(comms))
        print(f"[hipdsml watchdog] {reason}", file=sys.stderr, flush=True)
        for c in comms:
            try:
                c.abort()
            except Exception as e:  # noqa: BLE001
                log.error("abort failed: %s", e)
        for fn in aborters:
            try:
                fn()
            except Exception as e:  # noqa: BLE001
                log.error("abort hook failed: %s", e)

    def stop(self) -> None:
        self._stop.set()
        if self._thread is not threading.current_thread():
            self._thread.join(timeout=2.0)

    # -- the thread --------------------------------------------------------------
    def _run(self) -> None:
        while not self._stop.wait(self.interval):
            now = time.monotonic()
            if self._fault is None:
                with self._lock:
                    comms = list(self._comms)
                    section, since = self._section, self._since
                for c in comms:
                    try:
                        err = c.async_error()
                    except Exception as e:  # noqa: BLE001
                        err = str(e)
                    if err not in ("", "in-progress", "aborted"):
                        self.declare(f"RCCL async error: {err}")
                        break
                if self._fault is None and section is not None and now - since > self.timeout:
                    self.declare(f"'{section}' made no progress for {now - since:.1f} s "
                                 f"(timeout {self.timeout:.0f} s): a peer died or stalled")
            elif self.exit_on_stuck and self._section is not None and \
                    now - self._fault_at > self.grace:
                print(f"[hipdsml watchdog] main thread still blocked in '{self._section}' "
                      f"{self.grace:.0f} s after the abort; exiting with code {EXIT_CODE}",
                      file=sys.stderr, flush=True)
                os._exit(EXIT_CODE)


def timeout_from_env(default: float = 300.0) -> float:
    """HIPDSML_WATCHDOG_S: stall timeout in seconds (0 disables the watchdog)."""
    try:
        return float(os.environ.get("HIPDSML_WATCHDOG_S", default))
    except ValueError:
        return default

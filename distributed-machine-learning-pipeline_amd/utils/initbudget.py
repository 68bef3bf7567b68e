"""Wall-clock phases of a job's initialisation, and a total budget for the
optional ones.

The reference has one init step worth timing -- dial three device servers and
read their metadata (``gpu_coordinator_server.go:121-192``) -- and nothing
optional.  A data-parallel job here does much more before its first timed
step: RCCL bootstrap, self-tests of every gradient-sync candidate, timing of
the candidates, the hand-off buffer placement search, the ring chunk sweep,
and (bench.py) diagnostic probes after the timed steps.  On a node nobody has
run on yet, each of those can cost more than expected, so:

* every phase is timed and reported (``report()`` -> the bench JSON's
  ``init_phases_s``), so the first multi-GPU run says where its init went;
* the optional phases ask :meth:`InitPhases.allow` first.  Once the slowest
  rank's elapsed init exceeds the budget (``HIPDSML_INIT_BUDGET_S``, default
  240 s), every remaining optional phase is skipped and recorded in
  ``skipped``.  The timed steps, the self-test of the candidate that will run
  and the cross-rank replica check are never optional.

``allow`` is collective in a distributed job (the max elapsed time over the
ranks decides), so every rank takes the same branch.
"""
from __future__ import annotations

import contextlib
import os
import time
from typing import Callable, Dict, List, Optional

DEFAULT_BUDGET_S = 240.0


def budget_from_env(default: float = DEFAULT_BUDGET_S) -> float:
    try:
        return float(os.environ.get("HIPDSML_INIT_BUDGET_S", default))
    except ValueError:
        return default


class InitPhases:
    def __init__(self, ctx=None, budget_s: Optional[float] = None,
                 clock: Callable[[], float] = time.perf_counter, t0: Optional[float] = None):
        self.ctx = ctx
        self.budget_s = budget_from_env() if budget_s is None else float(budget_s)
        self.clock = clock
        self.t0 = clock() if t0 is None else t0
        self.phases: Dict[str, float] = {}
        self.skipped: List[str] = []

    def elapsed(self) -> float:
        return self.clock() - self.t0

    @contextlib.contextmanager
    def phase(self, name: str):
        """Time a phase (repeated names accumulate)."""
        t = self.clock()
        try:
            yield
        finally:
            self.phases[name] = round(self.phases.get(name, 0.0) + self.clock() - t, 4)

    def allow(self, name: str) -> bool:
        """Whether optional phase `name` may run: the slowest rank's elapsed
        init is still under the budget.  Collective when distributed."""
        e = self.elapsed()
        ctx = self.ctx
        if ctx is not None and getattr(ctx, "is_distributed", False):
            e = ctx.all_reduce_scalars(e, op="max")[0]
        if e < self.budget_s:
            return True
        self.skipped.append(name)
        return False

    def report(self) -> dict:
        return {"total_s": round(self.elapsed(), 4), "budget_s": self.budget_s,
                "phases_s": dict(self.phases), "skipped": list(self.skipped)}

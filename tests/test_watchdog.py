"""Data-plane failure detection (BASELINE config 5; the
reference's health monitor: gpu_coordinator_server.go:69-119).  Two ranks of
the real fit job on CPU (gloo), launched as plain processes (no torchrun agent
that would kill the survivor for us): when rank 1 dies or stalls mid-job,
rank 0 must exit non-zero within 30 s instead of waiting out the 600 s
process-group timeout."""
import os
import socket
import subprocess
import sys
import time

import pytest

from hipdsml.parallel.watchdog import EXIT_CODE, CommFault, Watchdog

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _launch(fault, extra_env=None):
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r),
                   LOCAL_WORLD_SIZE="2", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   HIPDSML_FAULT=fault, HIPDSML_WATCHDOG_S="4", HIPDSML_WATCHDOG_GRACE_S="3",
                   HIPDSML_PROGRESS="0", OMP_NUM_THREADS="1", PYTHONPATH=ROOT)
        env.update(extra_env or {})
        cmd = [sys.executable, "-m", "hipdsml", "fit", "--device", "cpu", "--backend", "gloo",
               "--model", "784-32-10", "--batch", "16", "--samples", "512", "--steps", "100000",
               "--log-every", "1", "--eval", "false"]
        procs.append(subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    return procs


def _finish(procs, timeout):
    t0 = time.monotonic()
    p0 = procs[0]
    try:
        out, err = p0.communicate(timeout=timeout)
        rc = p0.returncode
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
            p.wait(timeout=30)
    return rc, time.monotonic() - t0, out, err


@pytest.mark.parametrize("mode", ["exit", "hang"])
def test_survivor_exits_when_peer_dies_or_stalls(mode):
    procs = _launch(f"1:20:{mode}")
    rc, dt, out, err = _finish(procs, timeout=60)
    assert rc != 0, (out[-2000:], err[-2000:])
    # 30 s from the fault, measured loosely from launch (the import alone is a few s)
    assert dt < 45, dt
    if mode == "hang":  # only the watchdog can end this one: gloo waits 600 s by itself
        assert "watchdog" in err, err[-3000:]
        assert rc in (1, EXIT_CODE), rc


def test_watchdog_unit_timeout_and_abort():
    class FakeComm:
        aborted = False
        err = ""

        def abort(self):
            self.aborted = True

        def async_error(self):
            return self.err

    wd = Watchdog(timeout=0.3, interval=0.02, grace=60.0, exit_on_stuck=False)
    c = FakeComm()
    wd.watch_comm(c)
    with wd.guard("fast"):
        pass
    with pytest.raises(CommFault, match="no progress"):
        with wd.guard("stalled collective"):
            time.sleep(1.0)
    assert c.aborted
    with pytest.raises(CommFault):  # sticky
        wd.check()
    wd.stop()

    wd2 = Watchdog(timeout=30, interval=0.02, exit_on_stuck=False)
    c2 = FakeComm()
    wd2.watch_comm(c2)
    c2.err = "remote process exited or there was a network error"
    time.sleep(0.2)
    assert c2.aborted and "RCCL async error" in wd2.fault
    wd2.stop()

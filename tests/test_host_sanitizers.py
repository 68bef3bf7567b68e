"""Sanitizer builds of the host-side native runtime (SURVEY
§5 "race detection / sanitizers").  GPU sanitizers (ASan with xnack) are not
available on this pool, so the host logic is compiled against a host-only HIP
stand-in (csrc/hostshim) by g++ and run under:

* AddressSanitizer + UndefinedBehaviorSanitizer: ring_plan.h schedules for
  n = 1..8 simulated over all ranks, DeviceArena bounds, CopyEngine staging
  pipelines at every chunk boundary, the StreamTable state machine;
* ThreadSanitizer: 8 threads driving the StreamTable (+ CopyEngine) at once,
  as the gRPC servicer threads do.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "distributed-machine-learning-pipeline_amd", "csrc")
SRCS = [os.path.join(ROOT, "tests", "native", "host_runtime_test.cpp"),
        os.path.join(CSRC, "runtime", "device_runtime.cpp"),
        os.path.join(CSRC, "hostshim", "hostshim.cpp")]

pytestmark = pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")


def _build(tmp_path, name, san):
    exe = str(tmp_path / name)
    cmd = ["g++", "-std=c++17", "-g", "-O1", "-fno-omit-frame-pointer", "-pthread",
           "-I", os.path.join(CSRC, "hostshim"), "-I", CSRC, *san, *SRCS, "-o", exe]
    p = subprocess.run(cmd, capture_output=True, text=True)
    assert p.returncode == 0, p.stderr[-4000:]
    return exe


def _run(exe, arg, env_extra):
    env = dict(os.environ, **env_extra)
    p = subprocess.run([exe, arg], capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-6000:])
    assert "host runtime OK" in p.stdout


def test_asan_ubsan(tmp_path):
    exe = _build(tmp_path, "rt_asan", ["-fsanitize=address,undefined", "-fno-sanitize-recover=all"])
    _run(exe, "all", {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0",
                      "UBSAN_OPTIONS": "print_stacktrace=1:halt_on_error=1"})


def test_tsan_stream_table_threads(tmp_path):
    exe = _build(tmp_path, "rt_tsan", ["-fsanitize=thread"])
    _run(exe, "threads", {"TSAN_OPTIONS": "halt_on_error=1:second_deadlock_stack=1"})

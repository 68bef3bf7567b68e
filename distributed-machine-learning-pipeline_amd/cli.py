"""Command-line entry points (``python -m hipdsml <command>``).

Reference launchers: ``DSML/cmd/gpu_device_server/main.go`` (3 device servers on
ports 5003-5005, ids 1-3, memSize 0x3000) and ``DSML/cmd/gpu_coordinator_server/main.go``
(port 50051); client ``go run client/client.go``.  Everything that was a
compile-time constant there is a flag here (SURVEY §5 "Config / flag system").

  device-server  start device servers (one per --ports entry; --gpus maps them to GPUs)
  coordinator    start the coordinator (health-check interval configurable)
  train          run the training client (device / rpc mode)
  fit            data-parallel training job (torchrun-compatible; config, checkpoints, metrics)
  local          spawn device servers (one process per GPU) + coordinator + client
  bench-allreduce  ring vs naive all-reduce latency through the gpu_sim API
"""
from __future__ import annotations

import argparse
import logging
import os
import signal
import subprocess
import sys
import threading
import time


def _serve_forever(stop_fns):
    ev = threading.Event()
    signal.signal(signal.SIGINT, lambda *_: ev.set())
    signal.signal(signal.SIGTERM, lambda *_: ev.set())
    ev.wait()
    for f in stop_fns:
        f()


def cmd_device_server(a) -> int:
    from .rpc.device_server import start_device_server

    ports = [p for p in a.ports.split(",") if p]
    gpus = [int(g) for g in a.gpus.split(",")] if a.gpus else [0] * len(ports)
    ids = [int(i) for i in a.device_ids.split(",")] if a.device_ids else list(range(1, len(ports) + 1))
    servers = []
    for port, gpu, did in zip(ports, gpus, ids):
        server, addr, svc = start_device_server(did, a.mem_size, f"{a.host}:{port}", backend=a.backend, gpu=gpu,
                                              scratch_size=a.scratch_bytes or None)
        if a.fail_after and did == (a.fail_device or did):
            svc.arm_fault(a.fail_after, a.fail_mode)
        print(f"GPU Device server listening on port {addr.rsplit(':', 1)[1]} with device ID {did}", flush=True)
        servers.append(server)
    _serve_forever([lambda s=s: s.stop(1) for s in servers])
    return 0


def cmd_coordinator(a) -> int:
    from .rpc.coordinator import start_coordinator

    # the "pg" communicators' TCP store: devices on other hosts must reach it,
    # so it binds to the coordinator's own address unless told otherwise
    store_host = a.store_host or (a.host if a.host not in ("", "0.0.0.0", "::") else "127.0.0.1")
    server, addr, svc = start_coordinator(f"{a.host}:{a.port}", health_interval=a.health_interval,
                                          health_timeout=a.health_timeout, store_host=store_host)
    print(f"GPU Coordinator server listening on port {addr.rsplit(':', 1)[1]}", flush=True)
    _serve_forever([svc.stop, lambda: server.stop(1)])
    return 0


def cmd_train(rest) -> int:
    from .rpc.client import main as client_main

    return client_main(rest)


def child_env() -> dict:
    """Environment for spawned server processes: the repo root on PYTHONPATH so
    `python -m hipdsml` resolves from any cwd; dmabuf IPC for RCCL."""
    env = dict(os.environ)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env["PYTHONPATH"] = root + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return env


def _wait_port(addr: str, timeout: float = 300.0) -> None:
    from .rpc.stubs import connect

    t0 = time.time()
    while True:
        try:
            connect(addr, timeout=5).close()
            return
        except Exception:
            if time.time() - t0 > timeout:
                raise
            time.sleep(0.5)


def cmd_local(a) -> int:
    """One device-server PROCESS per GPU (own HIP context, own RCCL rank), a
    coordinator process, then the client in this process."""
    env = child_env()
    procs = []
    try:
        devs = []
        for i in range(a.gpus):
            port = a.base_port + i
            devs.append(f"127.0.0.1:{port}")
            procs.append(subprocess.Popen(
                [sys.executable, "-m", "hipdsml", "device-server", "--ports", str(port), "--gpus",
                 str(i if a.backend == "hip" else 0), "--device-ids", str(i + 1), "--backend",
                 a.backend, "--mem-size", str(a.mem_size)], env=env))
        procs.append(subprocess.Popen([sys.executable, "-m", "hipdsml", "coordinator", "--port",
                                       str(a.coord_port), "--health-interval", str(a.health_interval)],
                                      env=env))
        coord = f"127.0.0.1:{a.coord_port}"
        for d in devs + [coord]:
            _wait_port(d)
        args = ["--coordinator", coord, "--devices", ",".join(devs), "--mode", a.mode,
                "--epochs", str(a.epochs), "--model", a.model, "--samples", str(a.samples)]
        return cmd_train(args)
    finally:
        for p in procs:
            p.terminate()
        for p in procs:
            try:
                p.wait(timeout=10)
            except subprocess.TimeoutExpired:
                p.kill()


def cmd_bench_allreduce(rest) -> int:
    from .bench.allreduce import main as bench_main

    return bench_main(rest)


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(name)s %(message)s")
    if argv and argv[0] == "train":
        return cmd_train(argv[1:])
    if argv and argv[0] == "fit":
        from .engine.fit import main as fit_main

        return fit_main(argv[1:])
    if argv and argv[0] == "bench-allreduce":
        return cmd_bench_allreduce(argv[1:])
    ap = argparse.ArgumentParser(prog="hipdsml")
    sub = ap.add_subparsers(dest="cmd", required=True)
    d = sub.add_parser("device-server")
    d.add_argument("--host", default="127.0.0.1")
    d.add_argument("--ports", default="5003,5004,5005")
    d.add_argument("--gpus", default="")
    d.add_argument("--device-ids", default="")
    d.add_argument("--backend", default="auto", choices=["auto", "host", "hip"])
    d.add_argument("--mem-size", type=int, default=64 << 20)
    d.add_argument("--scratch-bytes", type=int, default=0,
                   help="private ring scratch window per device (0: 64 MiB GPU, 1 MiB host); "
                        "host data-parallel TrainSteps stages the whole gradient there")
    d.add_argument("--fail-after", type=int, default=0,
                   help="fault injection: die on the N-th data-plane RPC (0 = never)")
    d.add_argument("--fail-device", type=int, default=0, help="only this device id (0 = all)")
    d.add_argument("--fail-mode", default="exit", choices=["exit", "stop"])
    c = sub.add_parser("coordinator")
    c.add_argument("--host", default="127.0.0.1")
    c.add_argument("--port", type=int, default=50051)
    c.add_argument("--health-interval", type=float, default=5.0)
    c.add_argument("--health-timeout", type=float, default=2.0)
    c.add_argument("--store-host", default="",
                   help="address the process-group store of CommInit backend 'pg' binds to and "
                        "the device servers connect to (default: --host, or 127.0.0.1 when "
                        "--host is a wildcard)")
    lo = sub.add_parser("local")
    lo.add_argument("--gpus", type=int, default=1)
    lo.add_argument("--backend", default="hip", choices=["host", "hip"])
    lo.add_argument("--mode", default="device", choices=["device", "rpc"])
    lo.add_argument("--epochs", type=int, default=1)
    lo.add_argument("--model", default="784-128-64-10")
    lo.add_argument("--samples", type=int, default=60032)
    lo.add_argument("--mem-size", type=int, default=64 << 20)
    lo.add_argument("--base-port", type=int, default=5003)
    lo.add_argument("--coord-port", type=int, default=50051)
    lo.add_argument("--health-interval", type=float, default=5.0)
    a = ap.parse_args(argv)
    return {"device-server": cmd_device_server, "coordinator": cmd_coordinator,
            "local": cmd_local}[a.cmd](a)


if __name__ == "__main__":
    sys.exit(main())

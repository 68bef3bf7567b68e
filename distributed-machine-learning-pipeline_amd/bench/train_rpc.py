"""BASELINE config 2 through the reference's topology: the MLP trained on ONE
device-server process (own GPU, or the host backend on a CPU box) driven by a
client through the coordinator, exactly the process layout of the reference
(coordinator :50051, device servers :5003+, client; ``client.go:516-659``,
wall time ``README.md:199-203``).

Two client flows are timed:

* ``device`` — ConfigureModel once, then TrainSteps(k) RPCs (the fused HIP
  step, persistent on the GPU; only loss / accuracy scalars return).  For
  k in {1, 50, 937} it reports samples/s at the client and the per-RPC
  overhead = client wall - the device's own elapsedUs of the call.
* ``rpc`` — the reference's per-step pipeline, made correct: Memcpy of the
  batch, Memcpy of the labels, RunForward, RunBackward, AllReduceRing (n = 1:
  trivially SUCCESS, ``gpu_coordinator_server.go:289-295``), ApplyGradients:
  six RPCs per step.

With ``--devices N`` (N > 1) the client drives N device-server processes
(one per visible GPU, or all on GPU 0 of a one-GPU box) through CommInit
backend "pg": the coordinator hosts the TCP store the devices' process group
meets on, every device's ConfigureModel self-tests and times the
data-parallel candidates together (the persistent step's xGMI exchanges, the
fused exchanges, RCCL or gloo), and TrainSteps(k) runs on all devices at
once; samples/s counts every device's batches.

Synthetic 28x28 data and random-init weights (no dataset on the box).  Prints
one JSON line; ``--out`` also writes it to a file."""
from __future__ import annotations

import argparse
import json
import os
import statistics
import subprocess
import sys
import time


def _free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run(a) -> dict:
    from ..cli import _wait_port, child_env
    from ..data.mnist import synthetic_mnist
    from ..models.mlp import MlpSpec
    from ..rpc.client import TrainingClient
    from ..rpc.coordinator import start_coordinator
    from ..rpc.proto import pb

    n = a.devices
    gpus = 0
    if a.backend == "hip":
        import torch

        gpus = max(1, torch.cuda.device_count())  # counting does not initialise the GPU
    addrs, procs = [], []
    for i in range(n):
        port = (a.port + i) if a.port else _free_port()
        addrs.append(f"127.0.0.1:{port}")
        procs.append(subprocess.Popen(
            [sys.executable, "-m", "hipdsml", "device-server", "--ports", str(port),
             "--gpus", str(i % gpus if gpus else 0), "--device-ids", str(i + 1), "--backend", a.backend,
             "--mem-size", str(64 << 20)],
            env=child_env(), stdout=subprocess.DEVNULL, stderr=subprocess.PIPE))
    server = svc = None
    out = {"metric": "MNIST MLP samples/sec via coordinator + device server",
           "config": {"model": f"MLP {a.model} SGD", "batch": a.batch, "device_servers": n,
                      "physical_gpus": min(n, gpus) if gpus else 0,
                      "backend": a.backend, "data": "synthetic 28x28 (random-init weights)"}}
    try:
        server, caddr, svc = start_coordinator("127.0.0.1:0", health_interval=60.0)
        for ad in addrs:
            _wait_port(ad, timeout=600.0)
        spec = MlpSpec.parse(a.model)
        cl = TrainingClient(caddr, addrs, spec.dims, a.batch, 0.01, out=lambda s: None)
        try:
            cl.comm_init("pg" if n > 1 else "rpc")
            out["config"]["comm_backend"] = "pg" if n > 1 else "rpc"
            t0 = time.perf_counter()
            rs = cl._all(lambda i, s: s.ConfigureModel(pb.ConfigureModelRequest(
                dims=list(spec.dims), batch=a.batch, lr=0.01, seed=0, commId=cl.comm_id, rank=i,
                worldSize=n, dataset="synthetic", numSamples=a.samples, dataSeed=1000,
                graphSteps=50, sync=a.sync if n > 1 else "rccl"), timeout=600))
            out["configure_ms"] = round(1e3 * (time.perf_counter() - t0), 2)
            out["batches_per_epoch"] = rs[0].batchesPerEpoch
            out["config"]["sync"] = rs[0].sync
            if n > 1:
                out["config"]["sync_candidates_us"] = json.loads(rs[0].syncTimesJson or "{}") or None
            cl._all(lambda i, s: s.TrainSteps(pb.TrainStepsRequest(steps=max(a.warmup, 1)), timeout=600))
            dflow = {}
            for k in [int(x) for x in a.steps.split(",")]:
                walls, devs = [], []
                for _ in range(a.reps):
                    t0 = time.perf_counter()
                    rr = cl._all(lambda i, s: s.TrainSteps(pb.TrainStepsRequest(steps=k), timeout=600))
                    walls.append(time.perf_counter() - t0)
                    devs.append(max(x.elapsedUs for x in rr) * 1e-6)
                w, d = statistics.median(walls), statistics.median(devs)
                dflow[str(k)] = {"samples_per_s": round(k * a.batch * n / w, 1),
                                 "us_per_step": round(1e6 * w / k, 2),
                                 "device_us_per_step": round(1e6 * d / k, 2),
                                 "rpc_overhead_us": round(1e6 * (w - d), 1)}
            out["device_flow"] = dflow
            if n == 1:
                # the reference's per-step pipeline (six RPCs per step)
                ds = synthetic_mnist(a.batch * max(a.rpc_steps, 1), seed=1000)
                res = cl.train_rpc_mode(1, ds.X.numpy(), ds.y.numpy(), steps_per_epoch=a.rpc_steps)
                out["rpc_flow"] = {"steps": a.rpc_steps, "rpcs_per_step": 6,
                                   "samples_per_s": round(res["samples_per_s"], 1),
                                   "ms_per_step": round(1e3 * res["wall_s"] / max(a.rpc_steps, 1), 3)}
        finally:
            cl.close()
        best = max(v["samples_per_s"] for v in out["device_flow"].values())
        out["value"] = best
        out["unit"] = "samples/s"
        out["vs_baseline"] = round(best / 819.0, 2)  # ~819 samples/s
        return out
    finally:
        if svc is not None:
            svc.stop()
        if server is not None:
            server.stop(1)
        for proc in procs:
            proc.terminate()
        for proc in procs:
            try:
                proc.wait(timeout=30)
            except subprocess.TimeoutExpired:
                proc.kill()


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--backend", default="auto", choices=["auto", "hip", "host"])
    ap.add_argument("--model", default="784-128-64-10")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--samples", type=int, default=60032)
    ap.add_argument("--steps", default="1,50,937", help="TrainSteps(k) sizes to time")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--rpc-steps", type=int, default=50, help="steps of the per-step RPC flow")
    ap.add_argument("--port", type=int, default=0)
    ap.add_argument("--devices", type=int, default=1, help="device-server processes (one per GPU, "
                    "all on GPU 0 when fewer are visible)")
    ap.add_argument("--sync", default="", help="N > 1: the devices' sync mode ('' = auto)")
    ap.add_argument("--out", default="")
    a = ap.parse_args(argv)
    if a.backend == "auto":
        import torch

        a.backend = "hip" if torch.cuda.device_count() > 0 else "host"
    res = run(a)
    line = json.dumps(res)
    print(line, flush=True)
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        with open(a.out, "w") as f:
            f.write(line + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())

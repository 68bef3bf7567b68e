"""BASELINE config 2 through the reference topology (bench/train_rpc.py):
coordinator + one device-server PROCESS + client, TrainSteps(k) and the
per-step five-RPC flow.  Exercised here with the host (CPU) device backend;
the GPU run is recorded under profiles/r3_bench_rpc_device_n1.json."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_train_rpc_bench_host_backend(tmp_path):
    out = tmp_path / "rpc.json"
    env = dict(os.environ, PYTHONPATH=ROOT)
    p = subprocess.run([sys.executable, "-m", "hipdsml.bench.train_rpc", "--backend", "host",
                        "--steps", "1,5", "--reps", "2", "--warmup", "1", "--rpc-steps", "3",
                        "--samples", "640", "--out", str(out)],
                       capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    res = json.loads(out.read_text())
    assert res["config"]["backend"] == "host" and res["batches_per_epoch"] == 10
    for k in ("1", "5"):
        d = res["device_flow"][k]
        assert d["samples_per_s"] > 0 and d["rpc_overhead_us"] >= 0
        assert d["device_us_per_step"] > 0
    assert res["rpc_flow"]["steps"] == 3 and res["rpc_flow"]["samples_per_s"] > 0
    assert res["value"] == max(v["samples_per_s"] for v in res["device_flow"].values())

"""Host wait latency of one launch + synchronize under HIP's device schedule
flags (argv[1]: default | spin | yield | blocking, set through
hipSetDeviceFlags before torch creates its context), for an empty torch op and
for the persistent step's driver-shaped call (train_steps(20) + synchronize).
Prints one JSON line."""
import ctypes
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

mode = sys.argv[1] if len(sys.argv) > 1 else "default"
flags = {"default": None, "spin": 1, "yield": 2, "blocking": 4}[mode]
rc = None
if flags is not None:
    hip = ctypes.CDLL("libamdhip64.so")
    rc = hip.hipSetDeviceFlags(ctypes.c_uint(flags))

import torch  # noqa: E402

from hipdsml.data.mnist import synthetic_mnist  # noqa: E402
from hipdsml.engine.trainer import MlpTrainer  # noqa: E402
from hipdsml.models.mlp import MlpSpec  # noqa: E402
from hipdsml.parallel.dist import DistContext  # noqa: E402

dev = torch.device("cuda", 0)
x = torch.zeros(4, device=dev)
d = []
for _ in range(50):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    x.add_(1)
    torch.cuda.synchronize()
    d.append((time.perf_counter() - t0) * 1e6)
empty = statistics.median(d)

t = MlpTrainer(MlpSpec((784, 128, 64, 10)), synthetic_mnist(64 * 100, seed=1), batch=64, lr=0.01,
               ctx=DistContext(device=dev))
t.train_steps(5)
t.synchronize()
res = {}
for n in (1, 20, 200):
    d = []
    for _ in range(25):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        t.train_steps(n)
        t.synchronize()
        torch.cuda.synchronize()
        d.append((time.perf_counter() - t0) * 1e6)
    res[str(n)] = round(statistics.median(d), 2)
print(json.dumps({"mode": mode, "hipSetDeviceFlags_rc": rc, "empty_launch_sync_us": round(empty, 2),
                  "persistent_call_us": res, "us_per_step_n20": round(res["20"] / 20, 3)}))

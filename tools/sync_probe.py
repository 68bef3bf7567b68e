"""How much of the driver-form headline (bench.py --steps 20: one persistent
launch, synchronize on both sides) is the host's wait for the GPU, with the HIP
runtime's default scheduling vs hipDeviceScheduleSpin (SPIN=1: set through the
runtime torch loaded, before the device is first used).  Prints one JSON line:
median us of a 1-element op + synchronize, and the median us/step of 30 timed
20-step runs of the config-2 trainer, exactly as bench.py times them."""
import ctypes
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
spin = os.environ.get("SPIN", "0") == "1"
rc = None
if spin:
    lib = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
    rc = lib.hipSetDeviceFlags(ctypes.c_uint(1))  # hipDeviceScheduleSpin
from hipdsml.data.mnist import synthetic_mnist  # noqa: E402
from hipdsml.engine.trainer import MlpTrainer  # noqa: E402
from hipdsml.models.mlp import MlpSpec  # noqa: E402
from hipdsml.parallel.dist import DistContext  # noqa: E402

x = torch.zeros(1, device="cuda")
torch.cuda.synchronize()
lat = []
for _ in range(2000):
    t0 = time.perf_counter()
    x.add_(1)
    torch.cuda.synchronize()
    lat.append((time.perf_counter() - t0) * 1e6)
ctx = DistContext(device=torch.device("cuda", 0))
tr = MlpTrainer(MlpSpec((784, 128, 64, 10)), synthetic_mnist(60032, seed=1000), batch=64, lr=0.01, ctx=ctx, seed=0,
                graph_steps=50)
tr.train_steps(200)
tr.synchronize()
runs = []
for _ in range(30):
    tr.prepare(20)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tr.train_steps(20)
    torch.cuda.synchronize()
    runs.append((time.perf_counter() - t0) * 1e6 / 20)
    tr.synchronize()
print(json.dumps({"spin": spin, "set_flags_rc": rc, "op_sync_us_median": round(statistics.median(lat), 2),
                  "driver_form_us_per_step_median": round(statistics.median(runs), 3),
                  "driver_form_us_per_step_min": round(min(runs), 3)}))

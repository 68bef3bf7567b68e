"""Spread of the driver-form call (20 persistent steps): per repetition the
host wall time of train_steps(20) + torch.cuda.synchronize() and the kernel's
own span (launch-edge stamps: first block start -> last block end), to tell
host-side jitter from device-side.  Writes JSON to argv[1]."""
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hipdsml.data.mnist import synthetic_mnist  # noqa: E402
from hipdsml.engine.trainer import MlpTrainer  # noqa: E402
from hipdsml.models.mlp import MlpSpec  # noqa: E402
from hipdsml.ops.native import require_native  # noqa: E402
from hipdsml.parallel.dist import DistContext  # noqa: E402

C = require_native()
dev = torch.device("cuda", 0)
t = MlpTrainer(MlpSpec((784, 128, 64, 10)), synthetic_mnist(64 * 938, seed=1), batch=64, lr=0.01,
               ctx=DistContext(device=dev))
t.train_steps(5)
t.synchronize()
reps = int(os.environ.get("REPS", "40"))
walls, spans = [], []
C.mlp_persist_set_stamping(True)
for _ in range(reps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    t.train_steps(20)
    torch.cuda.synchronize()
    walls.append((time.perf_counter() - t0) * 1e6)
    v = C.mlp_persist_stamps()
    e = [v[(3 * 8 + 0) * 8 + p] for p in range(6)]
    spans.append((max(e[2], e[5]) - min(e[0], e[3])) / 100.0)
C.mlp_persist_set_stamping(False)
q = lambda xs: {"min": round(min(xs), 2), "median": round(statistics.median(xs), 2),  # noqa: E731
                "max": round(max(xs), 2), "stdev": round(statistics.pstdev(xs), 2)}
out = {"reps": reps, "wall_us": q(walls), "kernel_span_us": q(spans),
       "outside_kernel_us": q([w - s for w, s in zip(walls, spans)]),
       "walls": [round(w, 1) for w in walls], "spans": [round(s, 1) for s in spans]}
print(json.dumps({k: out[k] for k in ("wall_us", "kernel_span_us", "outside_kernel_us")}))
if len(sys.argv) > 1:
    json.dump(out, open(sys.argv[1], "w"), indent=1)

"""Does the single-replica persistent step's speed depend on WHERE its hand-off
buffer lands in memory?  One process, one trainer; the hand-off buffer is
re-allocated K times (earlier ones kept alive, so every one has a new address)
and each is timed over 2000 steps, plus a repeat of the first.  JSON to stdout."""
import json
import os
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
K = int(sys.argv[1]) if len(sys.argv) > 1 else 6
steps = 2000
ctx = DistContext(device=torch.device("cuda", 0))
spec = MlpSpec.parse("784-128-64-10")
tr = MlpTrainer(spec, synthetic_mnist(60032, seed=1000, dim=784), batch=64, lr=0.01, ctx=ctx, seed=0)
assert tr.pk_buf is not None


def timed():
    tr.train_steps(200)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tr.train_steps(steps)
    torch.cuda.synchronize()
    return round((time.perf_counter() - t0) / steps * 1e6, 3)


bufs = [tr.pk_buf]
pad = []
out = []
for k in range(K + 1):
    if k > 0:
        pad.append(torch.empty((k * 7919 + 1) * 4096, dtype=torch.uint8, device=ctx.device))  # shift the next address
        b = torch.zeros_like(bufs[0]) if k < K else bufs[0]
        if k < K:
            bufs.append(b)
        tr.pk_buf = b
        tr.runner.set_persist(b, tr.pk_err, 2000.0)
    out.append({"buf": k if k < K else 0, "addr_hex": hex(tr.pk_buf.data_ptr()), "us_per_step": [timed(), timed()]})
    print(json.dumps(out[-1]), flush=True)
print(json.dumps({"runs": out}))

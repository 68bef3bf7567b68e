"""Wide step (784-4096-4096-10, batch 64): does its time depend on where the
skinny GEMMs' split-K workspace (slabs + tickets) lands?  One process; the
workspace is re-allocated K times (earlier ones kept alive), the captured
graph dropped each time, each timed over 200 steps twice.  JSON lines."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hipdsml.data.mnist import synthetic_mnist  # noqa: E402
from hipdsml.engine.wide import WideMlpTrainer  # noqa: E402
from hipdsml.models.mlp import MlpSpec  # noqa: E402
from hipdsml.parallel.dist import DistContext  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 6
ctx = DistContext(device=torch.device("cuda", 0))
spec = MlpSpec.parse("784-4096-4096-10")
tr = WideMlpTrainer(spec, synthetic_mnist(64 * 50, seed=5, dim=784), batch=64, lr=0.01, ctx=ctx)


def timed(n=200):
    tr.train_steps(tr.nbatches)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tr.train_steps(n)
    torch.cuda.synchronize()
    return round((time.perf_counter() - t0) / n * 1e6, 2)


keep = []
for k in range(K):
    if k:
        keep.append(torch.empty((k * 7919 + 1) * 4096, dtype=torch.uint8, device=ctx.device))
        tr.Cp = torch.zeros_like(tr.Cp)
        tr.tctr = torch.zeros_like(tr.tctr)
        keep += [tr.Cp, tr.tctr]
        tr._graph = None
    print(json.dumps({"ws": k, "cp": hex(tr.Cp.data_ptr()), "ctr": hex(tr.tctr.data_ptr()),
                      "us_per_step": [timed(), timed()]}), flush=True)

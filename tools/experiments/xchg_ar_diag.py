"""Diagnose the standalone in-process xGMI all-reduce on dedicated streams."""
import sys

import torch

sys.path.insert(0, ".")
from hipdsml.ops.native import require_native  # noqa: E402
from hipdsml.parallel.xchg import make_local_group  # noqa: E402

DEV = torch.device("cuda", 0)
C = require_native()
mode = sys.argv[1]
n = int(sys.argv[2])
world = 2
if mode == "dedicated":
    streams = [torch.cuda.ExternalStream(C.dedicated_stream(0), device=DEV) for _ in range(world)]
else:
    streams = [torch.cuda.Stream(DEV) for _ in range(world)]
side = torch.cuda.Stream(DEV)
with torch.cuda.stream(side):
    xs = make_local_group(None, [0] * world, 2000.0, half_floats=2 << 20, ntiles=256)
    for it in range(3):
        host = [torch.arange(n, dtype=torch.float32) + 100 * r + 1 for r in range(world)]
        ins = [h.to(DEV) for h in host]
        outs = [torch.full_like(i, -7.0) for i in ins]
        torch.cuda.synchronize()
        for r in range(world):
            with torch.cuda.stream(streams[r]):
                xs[r].allreduce(ins[r], outs[r], 0)
        torch.cuda.synchronize()
        print(mode, n, it, [x.error() for x in xs], [o[:4].tolist() for o in outs],
              (host[0] + host[1])[:4].tolist(), flush=True)

"""In-process exchange replica groups (graph replay): bit-identical replicas?
Variant = stream kind; repeated R times."""
import sys

import torch

sys.path.insert(0, ".")
from hipdsml.data.mnist import synthetic_mnist  # noqa: E402
from hipdsml.engine.trainer import MlpTrainer  # noqa: E402
from hipdsml.models.mlp import MlpSpec  # noqa: E402
from hipdsml.ops.native import require_native  # noqa: E402
from hipdsml.parallel.dist import DistContext  # noqa: E402
from hipdsml.parallel.xchg import make_local_group  # noqa: E402

DEV = torch.device("cuda", 0)
C = require_native()
mode, world, gs, reps = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
pool = []
if mode == "dedicated":
    pool = [torch.cuda.ExternalStream(C.dedicated_stream(0), device=DEV) for _ in range(world)]
elif mode == "torchpool":
    pool = [torch.cuda.Stream(DEV) for _ in range(world)]
else:
    pool = [None] * world
side = torch.cuda.Stream(DEV)
res = []
with torch.cuda.stream(side):
    for rep in range(reps):
        trs = [MlpTrainer(MlpSpec((784, 128, 64, 10)), synthetic_mnist(256, seed=300 + r), batch=64,
                          lr=0.05, seed=7, ctx=DistContext(device=DEV), graph_steps=gs, stream=pool[r])
               for r in range(world)]
        xs = make_local_group(trs[0].layout, [0] * world, 5000.0)
        for t, x in zip(trs, xs):
            t.runner.set_exchange(x)
            t.xchg = x
        for chunk in (5, 5):
            for t in trs:
                t.train_steps(chunk)
            for t in trs:
                t.synchronize()
        Ps = [t.P.cpu() for t in trs]
        ndiff = [int((P != Ps[0]).sum()) for P in Ps]
        res.append(ndiff)
        del trs, xs
print(mode, world, gs, res, flush=True)

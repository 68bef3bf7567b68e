"""Diagnose in-process xGMI exchange replicas on one GPU: which stream setup
lets two spinning replicas run concurrently.  Prints one line per variant."""
import sys
import time

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


def run(name, streams, world=2, steps=10):
    trs = [MlpTrainer(MlpSpec((784, 128, 64, 10)), synthetic_mnist(256, seed=300 + r), batch=64,
                      lr=0.05, seed=7, ctx=DistContext(device=DEV), stream=streams[r])
           for r in range(world)]
    xs = make_local_group(trs[0].layout, [0] * world, 2000.0)
    for t, x in zip(trs, xs):
        t.runner.set_exchange(x)
        t.xchg = x
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for t in trs:
        t.train_steps(steps)
    for t in trs:
        t.runner.synchronize()
    dt = time.perf_counter() - t0
    errs = [x.error() for x in xs]
    print(f"{name:28s} world={world} errors={errs} wall={dt * 1e3:.1f} ms", flush=True)


which = sys.argv[1:] or ["own", "torchpool", "dedicated", "dedicated_cur"]
for w in which:
    if w == "own":
        run(w, [None, None, None])
    elif w == "torchpool":
        ss = [torch.cuda.Stream(DEV) for _ in range(3)]
        run(w, ss)
    elif w == "dedicated":
        ss = [torch.cuda.ExternalStream(C.dedicated_stream(0), device=DEV) for _ in range(3)]
        run(w, ss)
    elif w == "dedicated_cur":  # torch's current stream set to a non-null stream
        ss = [torch.cuda.ExternalStream(C.dedicated_stream(0), device=DEV) for _ in range(3)]
        with torch.cuda.stream(torch.cuda.Stream(DEV)):
            run(w, ss)

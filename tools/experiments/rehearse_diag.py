"""2-rank one-GPU rehearsal diagnosis (run under torch.distributed.run, gloo):
µs/step of sync=xgmi for 1000 steps before and after timing other sync modes,
to find which mode leaves the job slower."""
import json
import sys
import time

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))))
from hipdsml.data.mnist import synthetic_mnist  # noqa: E402
from hipdsml.engine.trainer import MlpTrainer  # noqa: E402
from hipdsml.models.mlp import MlpSpec  # noqa: E402
from hipdsml.parallel.dist import DistContext  # noqa: E402

ctx = DistContext.from_env(device="cuda", backend="gloo", device_index=0)
tr = MlpTrainer(MlpSpec((784, 128, 64, 10)), synthetic_mnist(64 * 100, seed=1000 + ctx.rank),
                batch=64, lr=0.01, ctx=ctx, seed=0, sync="auto", auto_fallback="torch")


def timed(n=1000):
    tr.train_steps(100)
    tr.synchronize()
    tr.prepare(n)
    ctx.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tr.train_steps(n)
    tr.synchronize()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / n
    ctx.barrier()
    return round(1e6 * ctx.all_reduce_scalars(dt, op="max")[0], 2)


out = {"auto_times": tr.sync_times, "auto_choice": tr.sync_active}
out["after_init"] = timed()
for m in ("xgmi", "xact", "torch"):
    tr.time_sync_modes([m])
    tr._set_mode("xgmi")
    out[f"after_{m}"] = timed()
tr._set_mode("xgmi")
out["again"] = timed()
if ctx.rank == 0:
    print(json.dumps(out), flush=True)
ctx.destroy()

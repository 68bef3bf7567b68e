"""Fixed cost of one persistent launch (kernels/mlp_persist.hip) as the
driver's bench sees it: wall time of train_steps(n) + synchronize() for a
range of n (median of reps), a least-squares fixed + per-step split, the
host-side pieces of synchronize(), and the in-kernel launch edges (prologue /
epilogue, s_memrealtime).  Writes JSON to argv[1]."""
import json
import statistics
import sys
import time

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from hipdsml.data.mnist import synthetic_mnist  # noqa: E402
from hipdsml.engine.trainer import MlpTrainer  # noqa: E402
from hipdsml.models.mlp import MlpSpec  # noqa: E402
from hipdsml.ops.native import require_native  # noqa: E402
from hipdsml.parallel.dist import DistContext  # noqa: E402

C = require_native()
dev = torch.device("cuda", 0)


def trainer(persist):
    return MlpTrainer(MlpSpec((784, 128, 64, 10)), synthetic_mnist(64 * 100, seed=1), batch=64,
                      lr=0.01, ctx=DistContext(device=dev), persist=persist)


def wall(t, n, reps=15):
    t.prepare(n)
    t.train_steps(n)
    t.synchronize()
    d = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        t.train_steps(n)
        t.synchronize()
        torch.cuda.synchronize()
        d.append((time.perf_counter() - t0) * 1e6)
    return statistics.median(d)


def fit(ns, us):
    mn, mu = statistics.mean(ns), statistics.mean(us)
    b = sum((x - mn) * (y - mu) for x, y in zip(ns, us)) / sum((x - mn) ** 2 for x in ns)
    return mu - b * mn, b


out = {}
NS = [1, 2, 5, 10, 20, 50, 200]
for name, persist in (("persistent", True), ("three_launch", False)):
    t = trainer(persist)
    assert t.persistent == persist
    us = [wall(t, n) for n in NS]
    a, b = fit(NS, us)
    out[name] = {"wall_us": dict(zip(map(str, NS), [round(u, 2) for u in us])),
                 "fixed_us": round(a, 2), "per_step_us": round(b, 3)}
    print(name, out[name], flush=True)

# the pieces of one driver-shaped call (n = 20)
t = trainer(True)
t.train_steps(20)
t.synchronize()
pieces = {"enqueue": [], "runner_sync": [], "err_read": [], "torch_sync": []}
for _ in range(15):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    t.train_steps(20)
    t1 = time.perf_counter()
    t.runner.join_into_torch()
    t.runner.synchronize()
    t2 = time.perf_counter()
    t.runner.persist_failed()
    t3 = time.perf_counter()
    torch.cuda.synchronize()
    t4 = time.perf_counter()
    for k, v in zip(pieces, (t1 - t0, t2 - t1, t3 - t2, t4 - t3)):
        pieces[k].append(v * 1e6)
out["n20_pieces_us"] = {k: round(statistics.median(v), 2) for k, v in pieces.items()}

# variants of the call: skip the torch->runner join, spin-wait stream sync
def raw(t, n, join, reps=25):
    d = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        t.runner.step(n, join)
        t.runner.synchronize()
        t.runner.persist_failed()
        d.append((time.perf_counter() - t0) * 1e6)
    return round(statistics.median(d), 2)


var = {}
for join in (True, False):
    var[f"join={int(join)}"] = {str(n): raw(t, n, join) for n in (1, 20)}
out["raw_call_variants_us"] = var
print(var, flush=True)

# empty-launch floor: one tiny torch kernel + synchronize
x = torch.zeros(4, device=dev)
d = []
for _ in range(30):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    x.add_(1)
    torch.cuda.synchronize()
    d.append((time.perf_counter() - t0) * 1e6)
out["empty_launch_sync_us"] = round(statistics.median(d), 2)

# in-kernel launch edges for n = 20
C.mlp_persist_set_stamping(True)
t.train_steps(20)
t.synchronize()
C.mlp_persist_set_stamping(False)
v = C.mlp_persist_stamps()
e = [v[(3 * 8 + 0) * 8 + p] for p in range(6)]  # role 3, row 0: the launch edges
us = lambda a_, b_: round((b_ - a_) / 100.0, 2)  # noqa: E731
out["n20_kernel_edges_us"] = {
    "l1_prologue": us(e[0], e[1]), "l1_loop_and_epilogue": us(e[1], e[2]),
    "chain_prologue": us(e[3], e[4]), "chain_loop_and_epilogue": us(e[4], e[5]),
    "chain_start_after_l1_start": us(e[0], e[3]),
    "span": us(min(e[0], e[3]), max(e[2], e[5])),
}
print(json.dumps(out, indent=1))
if len(sys.argv) > 1:
    json.dump(out, open(sys.argv[1], "w"), indent=1)

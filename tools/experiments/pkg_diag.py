"""Diagnostic: data-parallel Gram form (sync pkg) with 2 processes on one GPU,
parameter error against the fp32 reference after launch plans (1+2, 2+2, ...) (self-test
bypassed), next to sync pk.  Prints one JSON line."""
import json
import os
import sys
import tempfile

import torch
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))


def worker(rank, world, port, outdir, sync, plan):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    from hipdsml.data.mnist import synthetic_mnist
    from hipdsml.engine import trainer as T
    from hipdsml.models.mlp import MlpSpec
    from hipdsml.parallel import xchg as X
    from hipdsml.parallel.dist import DistContext

    X.verify_against_allreduce = lambda tr, steps=3: 0.0  # diagnostic: no self-test
    ctx = DistContext.from_env(device="cuda", backend="gloo")
    tr = T.MlpTrainer(MlpSpec((784, 128, 64, 10)), synthetic_mnist(64 * 4, seed=300 + rank), batch=64,
                      lr=0.05, ctx=ctx, seed=7, sync=sync, xchg_timeout_ms=5000.0, auto_fallback="torch")
    for k in plan:
        tr.train_steps(k)
    tr.synchronize()
    torch.save({"P": tr.P.cpu(), "xerr": int(tr.xchg.error()) if tr.xchg is not None else -1,
                "pk_failed": bool(tr.runner.persist_failed())}, os.path.join(outdir, f"r{rank}.pt"))
    ctx.destroy()


def main():
    from test_gpu_xchg import _reference
    from spawn_util import spawn_group

    world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    syncs = tuple(sys.argv[2].split(",")) if len(sys.argv) > 2 else ("pk", "pkg")
    out = {"world": world}
    for sync in syncs:
        for plan in ((1,), (3,), (1, 2), (2, 2)):
            steps = sum(plan)
            with tempfile.TemporaryDirectory() as d:
                spawn_group(worker, world, lambda port, d=d, sync=sync, plan=plan: (world, port, d, sync, plan))
                R = [torch.load(os.path.join(d, f"r{r}.pt"), weights_only=True) for r in range(world)]
            Ps = [x["P"] for x in R]
            err = (Ps[0] - _reference(world, steps, 0.05, 4)).abs().max().item()
            out[f"{sync}_{'+'.join(map(str, plan))}"] = {
                "err": err, "replicas_equal": all(bool(torch.equal(Ps[0], p)) for p in Ps),
                "xerr": [x["xerr"] for x in R], "pk_failed": [x["pk_failed"] for x in R]}
            print(json.dumps(out), file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    mp.set_start_method("spawn", force=True)
    main()

"""Phase timeline of the data-parallel persistent step (sync=pk) on ONE GPU:
two processes share cuda:0 through IPC (a rehearsal of two GPUs), rank 0
records the in-kernel stamps of layer-1 block 0 and chain block 0 for steps
8..15 of a launch (same phases as tools/pk_stamps.py; the replica exchange
sits inside "bwd+xchg+update" and, for the chains, is split between the
push after dW2 and the pull after the next partials).  Prints JSON; argv[1] = file."""
import json
import os
import socket
import statistics
import sys
import tempfile

import torch
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def _worker(rank, world, port, out):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK="0",
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from hipdsml.data.mnist import synthetic_mnist
    from hipdsml.engine.trainer import MlpTrainer
    from hipdsml.models.mlp import MlpSpec
    from hipdsml.ops.native import require_native
    from hipdsml.parallel.dist import DistContext

    C = require_native()
    ctx = DistContext.from_env(device="cuda", backend="gloo")
    t = MlpTrainer(MlpSpec((784, 128, 64, 10)), synthetic_mnist(64 * 100, seed=1 + rank), batch=64,
                   lr=0.01, ctx=ctx, sync="pk", auto_fallback="torch")
    assert t.persistent
    t.train_steps(100)
    t.synchronize()
    ctx.barrier()
    if rank == 0:
        C.mlp_persist_set_stamping(True)
    t.train_steps(32)
    t.synchronize()
    if rank == 0:
        C.mlp_persist_set_stamping(False)
        v = C.mlp_persist_stamps()
        st = [[[v[(r * 8 + s) * 8 + p] for p in range(8)] for s in range(8)] for r in range(3)]
        L1 = ["fwd+publish", "dZ1 wait", "bwd+xchg+update"]
        # the chain pushes its gradient after dW2 and sums + applies it after the
        # next step's partials arrived: "partials wait" includes that pull
        CH = ["partials wait + xchg pull/update", "L2/L3 fwd+softmax", "dZ2,dZ1 publish", "row exchange",
              "dW2/dW3 + xchg push"]
        res = {"layer1": {}, "chain": {}}
        for name, role, labels in (("layer1", 0, L1), ("chain", 1, CH)):
            for k, lab in enumerate(labels):
                res[name][lab] = round(statistics.median(
                    [(st[role][s][k + 1] - st[role][s][k]) / 100.0 for s in range(8)]), 3)
        res["step_us"] = round(statistics.median(
            [(st[0][s + 1][0] - st[0][s][0]) / 100.0 for s in range(7)]), 3)
        json.dump(res, open(out, "w"), indent=1)
    ctx.barrier()
    ctx.destroy()


if __name__ == "__main__":
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    with tempfile.TemporaryDirectory() as d:
        f = os.path.join(d, "st.json")
        mp.start_processes(_worker, args=(2, port, f), nprocs=2, start_method="spawn", join=True)
        res = json.load(open(f))
    print(json.dumps(res, indent=1))
    if len(sys.argv) > 1:
        json.dump(res, open(sys.argv[1], "w"), indent=1)

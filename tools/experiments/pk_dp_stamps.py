"""Phase timeline of the data-parallel persistent step (sync=pk, or argv[2] =
pkg for the Gram form, analysed like tools/pk_stamps.py) on ONE GPU:
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


def _worker(rank, world, port, out, sync="pk"):
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
                   lr=0.01, ctx=ctx, sync=sync, auto_fallback="torch")
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
        st = [[[v[(r * 8 + s) * 8 + p] for p in range(8)] for s in range(8)] for r in range(4)]
        if sync == "pkg":
            med = lambda xs: round(statistics.median(xs), 3)  # noqa: E731
            res = {"sync": sync, "layer1": {}, "chain": {}, "grad": {}}
            for name, role, labels in (
                    ("layer1", 0, ["fwd+publish", "dZ1 wait (+ peers' dZ1)", "bwd+slot sum+update"]),
                    ("chain", 1, ["Z1 wait", "H1, W wait+load", "fwd+softmax", "bwd+dZ1 publish+push",
                                  "rows publish"]),
                    ("grad", 2, ["rows wait+load", "dW/db MFMAs", "slot sum+update", "publish"])):
                for k, lab in enumerate(labels):
                    res[name][lab] = med([(st[role][s][k + 1] - st[role][s][k]) / 100.0 for s in range(8)])
            res["step_us"] = med([(st[0][s + 1][0] - st[0][s][0]) / 100.0 for s in range(7)])
            res["chain_dz1_publish_to_l1_ready_us"] = med([(st[0][s][2] - st[1][s][4]) / 100.0 for s in range(8)])
            res["l1_dz1_ready_to_z1_stored_us"] = med([(st[0][s][4] - st[0][s][2]) / 100.0 for s in range(8)])
            res["z1_stored_to_chain_seen_us"] = med([(st[1][s + 1][1] - st[0][s][4]) / 100.0 for s in range(7)])
            json.dump(res, open(out, "w"), indent=1)
            ctx.barrier()
            ctx.destroy()
            return
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
        sync = sys.argv[2] if len(sys.argv) > 2 else "pk"
        mp.start_processes(_worker, args=(2, port, f, sync), nprocs=2, start_method="spawn", join=True)
        res = json.load(open(f))
    print(json.dumps(res, indent=1))
    if len(sys.argv) > 1:
        json.dump(res, open(sys.argv[1], "w"), indent=1)

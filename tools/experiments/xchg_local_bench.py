#!/usr/bin/env python3
"""N replicas of the flagship MLP in ONE process on one GPU, synchronised by a
fused xGMI exchange (one-shot gradient exchange or activation exchange; peers
referenced directly).  Prints us/step; meant
to run under rocprofv3 --kernel-trace --stats (single process, no launcher)."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--replicas", type=int, default=2)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--graph-steps", type=int, default=50)
    ap.add_argument("--mode", default="xgmi", choices=["xgmi", "xact"],
                    help="xgmi: one-shot gradient exchange; xact: activation exchange")
    a = ap.parse_args()
    import torch

    from hipdsml.data.mnist import synthetic_mnist
    from hipdsml.engine.trainer import MlpTrainer
    from hipdsml.models.mlp import MlpSpec
    from hipdsml.parallel.dist import DistContext
    from hipdsml.parallel.xchg import make_local_act_group, make_local_group, swizzle_inputs

    dev = torch.device("cuda", 0)
    trs = [MlpTrainer(MlpSpec((784, 128, 64, 10)), synthetic_mnist(64 * 100, seed=r), batch=64,
                      lr=0.01, seed=0, ctx=DistContext(device=dev), graph_steps=a.graph_steps)
           for r in range(a.replicas)]
    if a.mode == "xgmi":
        xs = make_local_group(trs[0].layout, [0] * a.replicas)
        for t, x in zip(trs, xs):
            t.runner.set_exchange(x)
            t.xchg = x
    else:
        rows = trs[0].nbatches * 64
        Xall = swizzle_inputs(torch.stack([t.X[:rows] for t in trs]), 64)
        xs = make_local_act_group(trs[0].layout, [0] * a.replicas)
        for t, x in zip(trs, xs):
            t.runner.set_act_exchange(x, Xall, Xall[0].numel())
            t.xchg = x

    def run(n):
        for t in trs:
            t.train_steps(n)
        for t in trs:
            t.synchronize()

    run(a.graph_steps * 2)
    t0 = time.perf_counter()
    run(a.steps)
    dt = (time.perf_counter() - t0) / a.steps
    same = all(torch.equal(trs[0].P, t.P) for t in trs[1:])
    print(json.dumps({"mode": a.mode, "replicas": a.replicas, "us_per_step": round(dt * 1e6, 2),
                      "samples_per_s": round(64 * a.replicas / dt, 1), "replicas_identical": same}))
    return 0


if __name__ == "__main__":
    sys.exit(main())

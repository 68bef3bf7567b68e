#!/usr/bin/env python3
"""Compute-side cost of the two fused xGMI sync modes on ONE GPU, with no peer
to wait for: one replica runs the N-rank kernels while the other N-1 ranks'
exchange buffers live on the same device and every flag it would wait on is
preset.  The step time then holds the kernels' own work (N-rank weight-gradient
MFMAs and uncached-HBM reads for xact; peer-tile reads for xgmi) but no link
transfer and no peer skew.  Prints one JSON line per (mode, N)."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--graph-steps", type=int, default=50)
    a = ap.parse_args()
    import torch

    from hipdsml.data.mnist import synthetic_mnist
    from hipdsml.engine.trainer import MlpTrainer
    from hipdsml.models.mlp import MlpSpec
    from hipdsml.parallel.dist import DistContext
    from hipdsml.parallel.xchg import make_local_act_group, make_local_group, swizzle_inputs

    dev = torch.device("cuda", 0)
    for n in [int(x) for x in a.ranks.split(",")]:
        for mode in (("none",) if n == 1 else ("xgmi", "xact")):
            tr = MlpTrainer(MlpSpec((784, 128, 64, 10)), synthetic_mnist(64 * 100, seed=0),
                            batch=64, lr=0.01, seed=0, ctx=DistContext(device=dev),
                            graph_steps=a.graph_steps)
            xs = []
            if mode == "xgmi":
                xs = make_local_group(tr.layout, [0] * n)
                tr.runner.set_exchange(xs[0])
            elif mode == "xact":
                rows = tr.nbatches * 64
                Xall = swizzle_inputs(torch.stack([tr.X[:rows]] * n), 64)
                xs = make_local_act_group(tr.layout, [0] * n)
                tr.runner.set_act_exchange(xs[0], Xall, Xall[0].numel())
            for x in xs:
                x.fill_flags(1 << 62)
            torch.cuda.synchronize()
            tr.train_steps(a.graph_steps * 2)
            tr.runner.synchronize()
            t0 = time.perf_counter()
            tr.train_steps(a.steps)
            tr.runner.synchronize()
            dt = (time.perf_counter() - t0) / a.steps
            print(json.dumps({"mode": mode, "ranks": n, "us_per_step": round(dt * 1e6, 2)}),
                  flush=True)
            del tr, xs
    return 0


if __name__ == "__main__":
    sys.exit(main())

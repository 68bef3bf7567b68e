#!/usr/bin/env python3
"""BASELINE config 4: wide MLP 784-4096-4096-10, bf16 MFMA GEMMs, data-parallel.
Same launch contract as bench.py: `--gpus N` > 1 without a launcher starts N
ranks itself (bench._launch: the parent never touches the GPU, fewer visible
GPUs is rc 2); prints one JSON line."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--model", default="784-4096-4096-10")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--sync", default="xact", choices=["xact", "rccl", "ring", "torch"],
                    help="N > 1: xact = all-gather the bf16 activations (about 2 MB per replica "
                         "per step), rccl / ring = all-reduce the fp32 gradients (80 MB)")
    a = ap.parse_args()
    import bench

    if a.gpus > 1 and "WORLD_SIZE" not in os.environ and not os.environ.get(bench._LAUNCHED):
        return bench._launch(a, sys.argv[1:], script=__file__)
    if int(os.environ.get("WORLD_SIZE", "1")) != a.gpus:
        print(f"bench_wide.py: --gpus {a.gpus} but WORLD_SIZE={os.environ.get('WORLD_SIZE', '1')}",
              file=sys.stderr)
        return 2
    import torch  # noqa: F401

    from hipdsml.data.mnist import synthetic_mnist
    from hipdsml.engine.wide import WideMlpTrainer
    from hipdsml.models.mlp import MlpSpec
    from hipdsml.parallel.dist import DistContext

    ctx = DistContext.from_env(device="cuda")
    spec = MlpSpec.parse(a.model)
    ds = synthetic_mnist(a.batch * 64, seed=1000 + ctx.rank, dim=spec.dims[0])
    tr = WideMlpTrainer(spec, ds, batch=a.batch, lr=0.01, ctx=ctx, sync=a.sync)
    tr.train_steps(max(a.warmup, tr.nbatches if tr.graph_enabled else 0))
    tr.synchronize()
    ctx.barrier()
    t0 = time.perf_counter()
    tr.train_steps(a.steps)
    tr.synchronize()
    t1 = time.perf_counter()
    ctx.barrier()
    el = ctx.all_reduce_scalars(t1 - t0, op="max")[0] if ctx.is_distributed else t1 - t0
    n = ctx.world_size
    identical = ctx.replicas_identical(tr.P, "bench_wide/P") if n > 1 else True
    d = spec.dims
    flops = 6 * a.batch * sum(d[i] * d[i + 1] for i in range(len(d) - 1)) * a.steps * n
    if ctx.rank == 0:
        print(json.dumps({"metric": "wide MLP samples/sec", "value": round(a.batch * n * a.steps / el, 1),
                          "unit": "samples/s", "n_gpus": n, "steps": a.steps, "warmup": a.warmup,
                          "ms_per_step": round(1e3 * el / a.steps, 4), "tflops": round(flops / el / 1e12, 2),
                          "dtype": "bf16 (fp32 master/accum)", "data": "synthetic",
                          "config": {"model": f"MLP {spec}", "global_batch": a.batch * n,
                                     "parallelism": f"dp{n}", "sync": a.sync if n > 1 else "none"},
                          "replicas_identical": identical}),
              flush=True)
    ctx.destroy()
    if not identical:
        print("bench_wide.py: replicas diverged (parameters differ across ranks)", file=sys.stderr)
        return 3
    return 0


if __name__ == "__main__":
    sys.exit(main())

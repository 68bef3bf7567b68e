#!/usr/bin/env python3
"""Compute-plus-push cost of the persistent data-parallel step (sync='pk') on
ONE GPU, per replica count N, with no peer to wait for: one replica runs the
N-rank persistent launch while the other N-1 ranks' receive buffers live on
the same device and every flag it would wait on is preset.  Each step then
holds the kernel's own work plus its pushes (into local uncached HBM instead
of over xGMI) but no link transfer and no peer skew -- the lone-replica probe
of profiles/r1_sync_probe_lone_replica.json, for pk.

Prints one JSON line per N, with the exchange bytes each replica sends per
step (to all peers) from the kernel's slot layout."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def pk_bytes_out(n: int, algo: int = 0) -> int:
    """Bytes one replica pushes per step at n ranks (kernels/mlp_persist.hip):
    each of the 224 layer-1 waves sums an 8-float-per-lane slot (2 KiB), the
    16 gradient-block waves 16 / 8 / 4 floats per lane (3 layers: wave 0 four
    float4, waves 1-3 two).  One-shot (pk): every slot to every peer; two-shot
    (pk2): (n-1)/n of each slot to its owners, then the owners' (n-1)/n share
    to every peer."""
    slot_bytes = 224 * 64 * 8 * 4 + 4 * (64 * 16 * 4 + 3 * 64 * 8 * 4)
    if algo == 0:
        return (n - 1) * slot_bytes
    return 2 * (n - 1) * slot_bytes // n


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--launch", type=int, default=0, help="steps per launch (0: all in one)")
    ap.add_argument("--algo", type=int, default=0, help="0: pk (one-shot), 1: pk2 (two-shot)")
    a = ap.parse_args()
    import torch

    from hipdsml.data.mnist import synthetic_mnist
    from hipdsml.engine.trainer import MlpTrainer
    from hipdsml.models.mlp import MlpSpec
    from hipdsml.ops.native import require_native
    from hipdsml.parallel.dist import DistContext
    from hipdsml.parallel.xchg import make_local_group

    C = require_native()
    dev = torch.device("cuda", 0)
    for n in [int(x) for x in a.ranks.split(",")]:
        tr = MlpTrainer(MlpSpec((784, 128, 64, 10)), synthetic_mnist(64 * 100, seed=0),
                        batch=64, lr=0.01, seed=0, ctx=DistContext(device=dev))
        assert tr.persistent
        xs = []
        if n > 1:
            half, ntiles = C.MlpRunner.persist_xchg_size(n, a.algo)
            xs = make_local_group(None, [0] * n, 5000.0, half_floats=half, ntiles=ntiles)
            for x in xs:
                x.fill_flags(1 << 62)
            tr.runner.set_world_size(n)
            tr.runner.set_persist(tr.pk_buf, tr.pk_err, 5000.0, xs[0], a.algo)
        torch.cuda.synchronize()

        def run(k):
            per = a.launch or k
            while k > 0:
                tr.train_steps(min(per, k))
                k -= per

        run(200)
        tr.synchronize()
        t0 = time.perf_counter()
        run(a.steps)
        tr.synchronize()
        dt = (time.perf_counter() - t0) / a.steps
        print(json.dumps({"mode": ("pk2" if a.algo else "pk") if n > 1 else "none", "ranks": n,
                          "us_per_step": round(dt * 1e6, 2),
                          "bytes_out_per_step": pk_bytes_out(n, a.algo),
                          "bytes_per_peer_per_step": pk_bytes_out(n, a.algo) // max(n - 1, 1)}),
              flush=True)
        del tr, xs
        torch.cuda.synchronize()
    return 0


if __name__ == "__main__":
    sys.exit(main())

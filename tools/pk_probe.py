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


def pk_bytes_out(n: int, mode: str = "pk") -> int:
    """Bytes one replica pushes per step at n ranks (kernels/mlp_persist.hip):
    layer-1 waves move only their real dW1 tiles (wave 0 four 16x16 fp32
    tiles, waves 1-3 three) to every peer; chain wave slots (40 floats per
    lane) go from chain c to the peers d with d % 4 == c."""
    l1 = 32 * (4 + 3 * 3) * 64 * 4 * 4      # per destination
    ch = 4 * 64 * 40 * 4                     # all 4 chains' slots, per destination
    return (n - 1) * (l1 + ch)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--launch", type=int, default=0, help="steps per launch (0: all in one)")
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
            half, ntiles = C.MlpRunner.persist_xchg_size(n)
            xs = make_local_group(None, [0] * n, 5000.0, half_floats=half, ntiles=ntiles)
            for x in xs:
                x.fill_flags(1 << 62)
            tr.runner.set_world_size(n)
            tr.runner.set_persist(tr.pk_buf, tr.pk_err, 5000.0, xs[0])
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
        print(json.dumps({"mode": "pk" if n > 1 else "none", "ranks": n,
                          "us_per_step": round(dt * 1e6, 2),
                          "bytes_out_per_step": pk_bytes_out(n),
                          "bytes_per_peer_per_step": pk_bytes_out(n) // max(n - 1, 1)}),
              flush=True)
        del tr, xs
        torch.cuda.synchronize()
    return 0


if __name__ == "__main__":
    sys.exit(main())

"""A/B of the wide step's weight-update schedule (one GPU, 784-4096-4096-10,
batch 64): the default (dgrad, then one launch for every layer's update)
against the gated side-stream overlap for several gate lengths, and whether
the parameters stay bit-identical to the default after the same steps.
Prints one JSON line."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from hipdsml.data.mnist import synthetic_mnist  # noqa: E402
from hipdsml.engine.wide import WideMlpTrainer  # noqa: E402
from hipdsml.models.mlp import MlpSpec  # noqa: E402


def run(steps, **kw):
    spec = MlpSpec.parse("784-4096-4096-10")
    ds = synthetic_mnist(64 * 64, seed=1000, dim=784)
    tr = WideMlpTrainer(spec, ds, batch=64, lr=0.01, **kw)
    tr.train_steps(64)
    tr.synchronize()
    t0 = time.perf_counter()
    tr.train_steps(steps)
    tr.synchronize()
    us = 1e6 * (time.perf_counter() - t0) / steps
    return us, tr.P.detach().clone()


def main():
    steps = 256
    out = {}
    ref_us, ref_P = run(steps)
    out["default"] = round(ref_us, 2)
    for name, kw in [("overlap_per_layer", dict(overlap_wgrad=True)),
                     ("gated_0", dict(overlap_wgrad=True, wgrad_gate=0)),
                     ("gated_2k", dict(overlap_wgrad=True, wgrad_gate=2000)),
                     ("gated_8k", dict(overlap_wgrad=True, wgrad_gate=8000)),
                     ("gated_32k", dict(overlap_wgrad=True, wgrad_gate=32000))]:
        us, P = run(steps, **kw)
        out[name] = {"us": round(us, 2), "bit_identical": bool(torch.equal(P, ref_P)),
                     "maxdiff": float((P - ref_P).abs().max())}
        print(json.dumps(out), file=sys.stderr, flush=True)
    again, _ = run(steps)
    out["default_again"] = round(again, 2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()

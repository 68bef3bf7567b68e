"""A/B timing of the wide step's multi-layer weight-update launch
(wgrad_sgd_multi) on the BASELINE config-4 shapes: layer order and single
layers. Prints one JSON line of µs per launch."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from hipdsml.data.mnist import synthetic_mnist  # noqa: E402
from hipdsml.engine.wide import WideMlpTrainer  # noqa: E402
from hipdsml.models.mlp import MlpSpec  # noqa: E402

t = WideMlpTrainer(MlpSpec((784, 4096, 4096, 10)), synthetic_mnist(64 * 8, seed=1), batch=64,
                   lr=1e-6, seed=0, graph=False)
t.train_steps(3)
t.synchronize()
C, d, Bt, L = t.C, t.spec.dims, t.batch, t.L
H = [t.Xb[:Bt]] + t.H[1:]


def layer(l):
    W, b = t.views[l]
    return (t.dZ[l + 1], H[l], Bt, d[l + 1], d[l], 1.0, 1e-6, W, t.Wb[l][1], None, b, None)


def timed(layers, reps=50):
    for _ in range(5):
        C.wgrad_sgd_multi(layers)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        C.wgrad_sgd_multi(layers)
    e1.record()
    torch.cuda.synchronize()
    return round(1e3 * e0.elapsed_time(e1) / reps, 2)


out = {}
for name, order in [("last_layer_first", range(L - 1, -1, -1)), ("first_layer_first", range(L)),
                    ("l0_only", [0]), ("l1_only", [1])]:
    out[name] = timed([layer(l) for l in order])
print(json.dumps(out), flush=True)

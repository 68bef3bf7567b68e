"""Roofline of the wide step's weight-update launch (wgrad_sgd_multi) on the
BASELINE config-4 shapes: the production kernel (one workgroup per 64x64 tile)
against two probes that move the same W bytes (fp32 read-modify-write + bf16
copy): the tile kernel without operand staging and MFMAs, and a plain linear
stream.  Prints one JSON line of µs per launch.  Variants tried and dropped
(see profiles/r2_wgrad_variants.json): a persistent tile walk with the next
tile's W prefetched, 2 / 4 tiles per workgroup, forced occupancy 6-8, operand
DMA ahead of the W loads."""
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


def layers(Ws):
    return [(t.dZ[l + 1], H[l], Bt, d[l + 1], d[l], 1.0, 1e-3, Ws[l][0], Ws[l][1], None, Ws[l][2], None)
            for l in range(L - 1, -1, -1)]


base = [(t.views[l][0].clone(), t.Wb[l][1].clone(), t.views[l][1].clone()) for l in range(L)]


def run_once(variant, grid):
    Ws = [(a.clone(), b.clone(), c.clone()) for a, b, c in base]
    C.wgrad_sgd_multi(layers(Ws), variant, grid)
    torch.cuda.synchronize()
    return Ws


def timed(variant, grid, reps=50):
    Ws = [(a.clone(), b.clone(), c.clone()) for a, b, c in base]
    ls = layers(Ws)
    for _ in range(5):
        C.wgrad_sgd_multi(ls, variant, grid)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        C.wgrad_sgd_multi(ls, variant, grid)
    e1.record()
    torch.cuda.synchronize()
    return round(1e3 * e0.elapsed_time(e1) / reps, 2)


ref = run_once(0, 0)
out = {"v0_production": timed(0, 0)}
# roofline probes: 20 = the same tiles without operand staging / MFMAs,
# 21 = a linear grid-stride stream of the same W bytes (fp32 RMW + bf16 copy)
for v, g in ((20, 0), (21, 8192)):
    out[f"v{v}_g{g}"] = timed(v, g)
out["v0_again"] = timed(0, 0)
print(json.dumps(out), flush=True)

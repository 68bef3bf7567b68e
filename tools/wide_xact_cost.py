"""Compute side of the wide engine's activation exchange (sync=xact) at N
replicas, measured on ONE MI355X: the fused weight-gradient + SGD launch over
the global batch (M = 64 N rows) that every replica runs instead of
all-reducing fp32 gradients, for the 784-4096-4096-10 shapes.  Also prints the
bytes each replica all-gathers per step (bf16 activations) against the bytes a
gradient all-reduce moves.  One JSON line."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hipdsml.ops.native import require_native  # noqa: E402

C = require_native()
dev = torch.device("cuda", 0)
d = (784, 4096, 4096, 10)
pd = [784, 4096, 4096, 16]
B = 64
W = [torch.randn(d[l + 1], d[l], device=dev) * 0.01 for l in range(3)]
Wb = [torch.zeros(pd[l + 1], pd[l], dtype=torch.bfloat16, device=dev) for l in range(3)]
# the engine's split masters (hi = the bf16 copy, lo = int16 remainder); HILO=0: fp32 W form
HILO = os.environ.get("HILO", "1") == "1"
Wh = [torch.zeros(pd[l + 1], pd[l], dtype=torch.bfloat16, device=dev) for l in range(3)]
Wl = [torch.zeros(pd[l + 1], pd[l], dtype=torch.int16, device=dev) for l in range(3)]
for l in range(3):
    C.hilo_split(W[l], Wh[l], Wl[l])
bias = [torch.zeros(d[l + 1], device=dev) for l in range(3)]


TILE = int(os.environ.get("WG_TILE", "0"))


def timed(n, reps=30):
    M = B * n
    g = torch.Generator(device=dev).manual_seed(n)
    H = [torch.randn(M, pd[l], device=dev, generator=g).to(torch.bfloat16) for l in range(3)]
    Z = [torch.randn(M, pd[l + 1], device=dev, generator=g).mul(1e-3).to(torch.bfloat16) for l in range(3)]
    if HILO:
        layers = [(Z[l], H[l], M, d[l + 1], d[l], 1.0 / n, 1e-6, None, Wb[l], None, bias[l], None, Wh[l], Wl[l])
                  for l in range(2, -1, -1)]
    else:
        layers = [(Z[l], H[l], M, d[l + 1], d[l], 1.0 / n, 1e-6, W[l], Wb[l], None, bias[l], None)
                  for l in range(2, -1, -1)]
    for _ in range(3):
        C.wgrad_sgd_multi(layers, tile=TILE)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        C.wgrad_sgd_multi(layers, tile=TILE)
    e1.record()
    torch.cuda.synchronize()
    return round(1e3 * e0.elapsed_time(e1) / reps, 2)


gather_per_replica = 2 * B * (pd[1] + pd[2] + pd[1] + pd[2] + pd[3])  # H1, H2, dZ1, dZ2, dZ3 bf16
grad_bytes = 4 * sum(d[l] * d[l + 1] + d[l + 1] for l in range(3))
out = {"wgrad_sgd_multi_us_by_replicas": {n: timed(n) for n in (1, 2, 4, 8)},
       "allgather_bytes_per_replica_per_step": gather_per_replica,
       "bytes_received_per_gpu_per_step_at_N8": 7 * gather_per_replica,
       "fp32_gradient_allreduce_bytes": grad_bytes,
       "ring_allreduce_bytes_sent_per_gpu_at_N8": int(2 * 7 / 8 * grad_bytes)}
print(json.dumps(out), flush=True)

"""Runs ONLY the wide global-batch weight-update launch (wgrad_sgd_multi, the
784-4096-4096-10 shapes, split masters) at N replicas' rows (M = 64 N) for a
few repetitions -- a short target for rocprofv3 --pmc / --kernel-trace.
Env: N (default 8), WG_TILE (0 auto / 64 / 128), REPS (default 10)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hipdsml.ops.native import require_native  # noqa: E402

C = require_native()
dev = torch.device("cuda", 0)
d = (784, 4096, 4096, 10)
pd = [784, 4096, 4096, 16]
n = int(os.environ.get("N", "8"))
tile = int(os.environ.get("WG_TILE", "0"))
reps = int(os.environ.get("REPS", "10"))
M = 64 * n
g = torch.Generator(device=dev).manual_seed(n)
Wh = [torch.zeros(pd[l + 1], pd[l], dtype=torch.bfloat16, device=dev) for l in range(3)]
Wl = [torch.zeros(pd[l + 1], pd[l], dtype=torch.int16, device=dev) for l in range(3)]
Wb = [torch.zeros(pd[l + 1], pd[l], dtype=torch.bfloat16, device=dev) for l in range(3)]
for l in range(3):
    C.hilo_split(torch.randn(d[l + 1], d[l], device=dev) * 0.01, Wh[l], Wl[l])
bias = [torch.zeros(d[l + 1], device=dev) for l in range(3)]
H = [torch.randn(M, pd[l], device=dev, generator=g).to(torch.bfloat16) for l in range(3)]
Z = [torch.randn(M, pd[l + 1], device=dev, generator=g).mul(1e-3).to(torch.bfloat16) for l in range(3)]
layers = [(Z[l], H[l], M, d[l + 1], d[l], 1.0 / n, 1e-6, None, Wb[l], None, bias[l], None, Wh[l], Wl[l])
          for l in range(2, -1, -1)]
for _ in range(reps):
    C.wgrad_sgd_multi(layers, tile=tile)
torch.cuda.synchronize()
print("ok", n, tile, reps)

"""Phase stamps of the row-block global-batch update (kernels/wgrad_sgd.hip
wgrad_rowblk_body, measurement build), wave 0 of each workgroup: entry, the
first segment's Z^T in registers, the end of each k tile (up to 12), exit.
The wide update at N replicas (M = 64 N, the 784-4096-4096-10 shapes).  Prints
medians over workgroups and launches (us)."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hipdsml.ops.native import require_native  # noqa: E402

C = require_native()
assert C.measure_build, "needs the measurement build"
dev = torch.device("cuda", 0)
d = (784, 4096, 4096, 10)
pd = [784, 4096, 4096, 16]
n = int(os.environ.get("N", "8"))
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
for _ in range(5):
    C.wgrad_sgd_multi(layers)
torch.cuda.synchronize()
zph, tiles, total, first_tile = [], [], [], []
for _ in range(10):
    C.wgrad_rowblk_set_stamping(True)
    C.wgrad_sgd_multi(layers)
    torch.cuda.synchronize()
    C.wgrad_rowblk_set_stamping(False)
    v = C.wgrad_rowblk_stamps()
    st = [v[16 * b:16 * b + 16] for b in range(256)]
    t0 = min(x[0] for x in st if x[0])
    for x in st:
        if not (x[0] and x[1] and x[14]):
            continue
        zph.append((x[1] - x[0]) / 100.0)
        total.append((x[14] - t0) / 100.0)
        ts = [x[k] for k in range(2, 14) if x[k]]
        if ts:
            first_tile.append((ts[0] - x[1]) / 100.0)
            tiles += [(b - a) / 100.0 for a, b in zip(ts, ts[1:])]
med = lambda xs: round(statistics.median(xs), 2) if xs else None  # noqa: E731
print(json.dumps({"N": n, "z_phase_us": med(zph), "first_tile_us": med(first_tile), "tile_us": med(tiles),
                  "tile_us_p90": round(sorted(tiles)[int(0.9 * len(tiles))], 2) if tiles else None,
                  "exit_since_launch_us_median": med(total), "exit_max": round(max(total), 2)}))

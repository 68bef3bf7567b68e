"""Time the fused classifier head (gemm_bf16.hip head_softmax_xent) variants."""
import json
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))))
from hipdsml.ops.native import require_native  # noqa: E402

C = require_native()
assert C.measure_build, "head_set_debug needs the measurement build: python -m hipdsml._build --measure"
dev = torch.device("cuda", 0)
B, K, Cn = 64, 4096, 10
H = torch.randn(B, K, device=dev).to(torch.bfloat16)
W = (0.05 * torch.randn(16, K, device=dev)).to(torch.bfloat16)
b = torch.randn(Cn, device=dev)
y = torch.randint(0, Cn, (B,), device=dev, dtype=torch.int32)
logits = torch.empty(B, Cn, device=dev)
dz = torch.zeros(B, 16, dtype=torch.bfloat16, device=dev)
dzp = torch.zeros(B, K, dtype=torch.bfloat16, device=dev)
stats = torch.zeros(4, device=dev)
rstats = torch.zeros(4 * B, device=dev)  # per-row accumulators, as the wide engine runs it
nostats = torch.zeros(4, device=dev)
rstats = torch.zeros(4 * B, device=dev)  # per-row accumulators, as the wide engine runs it


def t(fn, iters=50):
    for _ in range(5):
        fn()
    ts = []
    for _ in range(iters):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    ts.sort()
    return round(ts[len(ts) // 2], 2)


out = {
    "full_row_stats": t(lambda: C.head_softmax_xent(H, W, b, B, K, Cn, y, 1.0 / B, logits, dz, None, rstats,
                                                    dzp=dzp, row_stats=True)),
    "no_dzp_row_stats": t(lambda: C.head_softmax_xent(H, W, b, B, K, Cn, y, 1.0 / B, logits, dz, None, rstats,
                                                      row_stats=True)),
    "full": t(lambda: C.head_softmax_xent(H, W, b, B, K, Cn, y, 1.0 / B, logits, dz, None, stats, dzp=dzp)),
    "no_dzp": t(lambda: C.head_softmax_xent(H, W, b, B, K, Cn, y, 1.0 / B, logits, dz, None, stats)),
    "no_logits_no_dzp": t(lambda: C.head_softmax_xent(H, W, b, B, K, Cn, y, 1.0 / B, None, dz, None, stats)),
    "empty_torch_op": t(lambda: logits.zero_()),
}
for dbg in (1, 2, 3):
    C.head_set_debug(dbg)
    out[f"dbg{dbg}"] = t(lambda: C.head_softmax_xent(H, W, b, B, K, Cn, y, 1.0 / B, logits, dz, None, stats,
                                                     dzp=dzp))
C.head_set_debug(0)
print(json.dumps(out))

C.head_set_stamping(True)
C.head_softmax_xent(H, W, b, B, K, Cn, y, 1.0 / B, logits, dz, None, stats, dzp=dzp)
torch.cuda.synchronize()
C.head_set_stamping(False)
v = C.head_stamps()
st = [v[6 * r: 6 * r + 6] for r in range(64)]
t0 = min(s[0] for s in st)
import statistics  # noqa: E402
print(json.dumps({f"ph{k}": round(statistics.median((s[k + 1] - s[k]) / 100.0 for s in st), 2) for k in range(4)}
                 | {"entry_spread": (max(s[0] for s in st) - t0) / 100.0,
                    "span": (max(s[4] for s in st) - t0) / 100.0}))

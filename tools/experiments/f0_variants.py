"""Kernel-trace the first-layer forward (64 x 4096 x 784) variants: full-K
batch-row kernel vs the split-K skinny kernel at 1..4 slices."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from hipdsml.ops.native import require_native  # noqa: E402

C = require_native()
dev = torch.device("cuda", 0)
B, N, K = 64, 4096, 784
A = torch.randn(B, K, device=dev).to(torch.bfloat16)
W = torch.randn(N, K, device=dev).to(torch.bfloat16)
bias = torch.randn(N, device=dev)
H = torch.empty(B, N, dtype=torch.bfloat16, device=dev)
tiles = (N + 63) // 64
ws = torch.zeros(8 * tiles * 4096, device=dev)
ctr = torch.zeros(tiles, dtype=torch.int32, device=dev)
for _ in range(30):
    C.gemm_bf16_nt_fused(A, W, B, N, K, bias=bias, relu=True, obf=H, splits=0)
for sp in (1, 2, 3, 4):
    for _ in range(30):
        C.gemm_skinny(A, W, B, N, K, bias=bias, relu=True, obf=H, splits=sp, ws=ws, ctr=ctr)
torch.cuda.synchronize()

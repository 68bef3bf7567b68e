#!/usr/bin/env python3
"""Run ONE wide-MLP GEMM variant back to back (for rocprofv3 --pmc passes):
gemm_one.py rows64|splitk4|dwsgd|skinny_nt|skinny_nn|wgrad [N K iters]."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main() -> int:
    import torch

    from hipdsml.ops.native import require_native

    kind = sys.argv[1]
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    K = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
    iters = int(sys.argv[4]) if len(sys.argv) > 4 else 20
    C = require_native()
    dev = torch.device("cuda", 0)
    B = 64
    A = torch.randn(B, K, device=dev).to(torch.bfloat16)
    W = torch.randn(N, K, device=dev).to(torch.bfloat16)
    H = torch.empty(B, N, dtype=torch.bfloat16, device=dev)
    ws = torch.zeros(4 * ((N + 63) // 64) * 4096, device=dev)
    ctr = torch.zeros((N + 63) // 64, dtype=torch.int32, device=dev)
    dZT = torch.randn(N, B, device=dev).to(torch.bfloat16)
    HT = torch.randn(K, B, device=dev).to(torch.bfloat16)
    Wf = torch.randn(N, K, device=dev)
    Wb = torch.empty(N, K, dtype=torch.bfloat16, device=dev)
    WbT = torch.empty(K, N, dtype=torch.bfloat16, device=dev)
    bb = torch.zeros(N, device=dev)
    Wt = torch.randn(K, N, device=dev).to(torch.bfloat16)  # dgrad operand: W stored [K rows][N]
    Zr = torch.randn(B, N, device=dev).to(torch.bfloat16)  # row-major dZ
    Xr = torch.randn(B, K, device=dev).to(torch.bfloat16)  # row-major H
    for _ in range(iters):
        if kind == "rows64":
            C.gemm_bf16_nt_fused(A, W, B, N, K, obf=H, splits=0)
        elif kind == "skinny_nt":
            C.gemm_skinny(A, W, B, N, K, obf=H, ws=ws, ctr=ctr)
        elif kind == "skinny_nn":
            C.gemm_skinny(A, Wt, B, N, K, nn=True, obf=H, ws=ws, ctr=ctr)
        elif kind == "wgrad":
            C.wgrad_sgd(Zr, Xr, B, N, K, lr=1e-6, W=Wf, Wb=Wb, bias=bb)
        elif kind == "splitk4":
            C.gemm_bf16_nt_fused(A, W, B, N, K, obf=H, splits=4, ws=ws, ctr=ctr)
        else:
            C.gemm_bf16_nt_fused(dZT, HT, N, K, B, sgdW=Wf, lr=1e-6, obf=Wb, obfT=WbT, bsgd=bb)
    torch.cuda.synchronize()
    return 0


if __name__ == "__main__":
    sys.exit(main())

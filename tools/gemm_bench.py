#!/usr/bin/env python3
"""Time the wide-MLP GEMM shapes in isolation (median of N launches, hip events)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    import torch

    from hipdsml.ops.native import require_native

    C = require_native()
    dev = torch.device("cuda", 0)
    bf = dict(dtype=torch.bfloat16, device=dev)
    out = {}

    def timeit(name, fn, nbytes=0, flops=0):
        for _ in range(5):
            fn()
        ts = []
        for _ in range(a.iters):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        ts.sort()
        us = ts[len(ts) // 2]
        out[name] = {"us": round(us, 2), "TB/s": round(nbytes / us / 1e6, 2) if nbytes else None,
                     "TFLOP/s": round(flops / us / 1e6, 1) if flops else None}

    B = 64
    for (N, K) in [(4096, 4096), (4096, 784)]:
        A = torch.randn(B, K, device=dev).to(torch.bfloat16)
        W = torch.randn(N, K, device=dev).to(torch.bfloat16)
        bias = torch.randn(N, device=dev)
        H = torch.empty(B, N, **bf)
        HT = torch.empty(N, B, **bf)
        timeit(f"fwd_rows64_{N}x{K}", lambda: C.gemm_bf16_nt_fused(A, W, B, N, K, bias=bias, relu=True, obf=H, obfT=HT, splits=0),
               nbytes=N * K * 2, flops=2 * B * N * K)
        tiles = (N + 63) // 64
        ws = torch.zeros(8 * tiles * 4096, device=dev)
        ctr = torch.zeros(tiles, dtype=torch.int32, device=dev)
        for sp in (2, 4, 8):
            timeit(f"fwd_splitk{sp}_{N}x{K}", lambda sp=sp: C.gemm_bf16_nt_fused(
                A, W, B, N, K, bias=bias, relu=True, obf=H, obfT=HT, splits=sp, ws=ws, ctr=ctr),
                nbytes=N * K * 2, flops=2 * B * N * K)
    # library reference (hipBLASLt via torch) and K scaling of the batch-row kernel
    for (N, K) in [(4096, 4096), (4096, 1024), (4096, 784), (16384, 1024)]:
        A = torch.randn(B, K, device=dev).to(torch.bfloat16)
        W = torch.randn(N, K, device=dev).to(torch.bfloat16)
        H = torch.empty(B, N, **bf)
        timeit(f"torch_mm_{N}x{K}", lambda: torch.mm(A, W.t(), out=H), nbytes=N * K * 2,
               flops=2 * B * N * K)
        timeit(f"rows64_{N}x{K}", lambda: C.gemm_bf16_nt_fused(A, W, B, N, K, obf=H, splits=0),
               nbytes=N * K * 2, flops=2 * B * N * K)
    # skinny split-K kernels (kernels/gemm_skinny.hip): forward (NT) and dgrad (NN, W untransposed)
    for (N, K) in [(4096, 4096), (4096, 784)]:
        A = torch.randn(B, K, device=dev).to(torch.bfloat16)
        W = torch.randn(N, K, device=dev).to(torch.bfloat16)
        bias = torch.randn(N, device=dev)
        H = torch.empty(B, N, **bf)
        HT = torch.empty(N, B, **bf)
        wsw, ctw = C.gemm_skinny_ws(B, N, K, 8)
        ws = torch.zeros(wsw, device=dev)
        ctr = torch.zeros(ctw, dtype=torch.int32, device=dev)
        timeit(f"skinny_nt_{N}x{K}", lambda: C.gemm_skinny(A, W, B, N, K, bias=bias, relu=True, obf=H, obfT=HT,
                                                             ws=ws, ctr=ctr), nbytes=N * K * 2, flops=2 * B * N * K)
    for (N, K) in [(4096, 4096)]:
        A = torch.randn(B, K, device=dev).to(torch.bfloat16)
        W = torch.randn(K, N, device=dev).to(torch.bfloat16)
        mask = torch.randn(B, N, device=dev).to(torch.bfloat16)
        H = torch.empty(B, N, **bf)
        HT = torch.empty(N, B, **bf)
        wsw, ctw = C.gemm_skinny_ws(B, N, K, 8)
        ws = torch.zeros(wsw, device=dev)
        ctr = torch.zeros(ctw, dtype=torch.int32, device=dev)
        timeit(f"skinny_nn_{N}x{K}", lambda: C.gemm_skinny(A, W, B, N, K, nn=True, mask=mask, obf=H, obfT=HT,
                                                             ws=ws, ctr=ctr), nbytes=N * K * 2, flops=2 * B * N * K)
        for sp in (2, 4, 8):
            ws8 = ws
            timeit(f"skinny_nn_{N}x{K}_s{sp}", lambda sp=sp, ws8=ws8: C.gemm_skinny(
                A, W, B, N, K, nn=True, mask=mask, obf=H, obfT=HT, splits=sp, ws=ws8, ctr=ctr),
                nbytes=N * K * 2, flops=2 * B * N * K)
    M, N = 4096, 4096
    dZT = torch.randn(M, B, device=dev).to(torch.bfloat16)
    HT = torch.randn(N, B, device=dev).to(torch.bfloat16)
    Wf = torch.randn(M, N, device=dev)
    Wb = torch.empty(M, N, **bf)
    WbT = torch.empty(N, M, **bf)
    b = torch.zeros(M, device=dev)
    timeit("dw_sgd_4096x4096", lambda: C.gemm_bf16_nt_fused(dZT, HT, M, N, B, sgdW=Wf, lr=1e-6, obf=Wb, obfT=WbT, bsgd=b),
           nbytes=M * N * (4 + 4 + 2 + 2), flops=2 * B * M * N)
    timeit("dw_sgd_noT_4096x4096", lambda: C.gemm_bf16_nt_fused(dZT, HT, M, N, B, sgdW=Wf, lr=1e-6, obf=Wb, bsgd=b),
           nbytes=M * N * (4 + 4 + 2), flops=2 * B * M * N)
    Zr = torch.randn(B, N, device=dev).to(torch.bfloat16)
    Xr = torch.randn(B, N, device=dev).to(torch.bfloat16)
    bb = torch.zeros(M, device=dev)
    timeit("wgrad_sgd_4096x4096", lambda: C.wgrad_sgd(Zr, Xr, B, M, N, lr=1e-6, W=Wf, Wb=Wb, bias=bb),
           nbytes=M * N * (4 + 4 + 2), flops=2 * B * M * N)
    x = torch.empty(64 << 20, device=dev)
    timeit("copy_256MB", lambda: x[: 32 << 20].copy_(x[32 << 20:]), nbytes=2 * (32 << 20) * 4)
    print(json.dumps({"flags": os.environ.get("HIPDSML_R64_FLAGS", "3"), **out}))
    return 0


if __name__ == "__main__":
    sys.exit(main())

#!/usr/bin/env python3
"""Which operand limits the batch-row GEMM?  Time it with the activations or
the weights broadcast (stride 0: every block re-reads one cached row)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main() -> int:
    import torch

    from hipdsml.ops.native import require_native

    C = require_native()
    dev = torch.device("cuda", 0)
    B, N, K = 64, 4096, 4096
    A = torch.randn(B, K, device=dev).to(torch.bfloat16)
    W = torch.randn(N, K, device=dev).to(torch.bfloat16)
    Ab = A[:1].expand(B, K)
    Wb = W[:1].expand(N, K)
    H = torch.empty(B, N, dtype=torch.bfloat16, device=dev)
    out = {}
    for name, a, w in [("normal", A, W), ("A_bcast", Ab, W), ("W_bcast", A, Wb), ("both_bcast", Ab, Wb)]:
        f = lambda: C.gemm_bf16_nt_fused(a, w, B, N, K, obf=H, splits=0)  # noqa: E731
        for _ in range(5):
            f()
        ts = []
        for _ in range(30):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(); f(); e1.record(); e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        ts.sort()
        out[name] = round(ts[len(ts) // 2], 2)
    print(json.dumps({"rows64_us": out, "flags": os.environ.get("HIPDSML_R64_FLAGS", "3")}))
    return 0


if __name__ == "__main__":
    sys.exit(main())

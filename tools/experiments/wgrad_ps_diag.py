"""Diagnose the persistent wgrad form (tile 129) against per-layer launches."""
import sys
import torch
sys.path.insert(0, ".")
from hipdsml.ops.native import require_native

C = require_native()
DEV = torch.device("cuda", 0)
for M in [int(x) for x in sys.argv[1:]] or [64]:
    g = torch.Generator(device="cpu").manual_seed(77 + M)
    shapes = [(10, 4096), (4096, 4096), (4096, 784)]
    A, B = [], []
    for N, K in shapes:
        pn, pk = (N + 15) // 16 * 16, (K + 15) // 16 * 16
        Z = torch.zeros(M, pn, dtype=torch.bfloat16); X = torch.zeros(M, pk, dtype=torch.bfloat16)
        Z[:, :N] = torch.randn(M, N, generator=g).to(torch.bfloat16)
        X[:, :K] = torch.randn(M, K, generator=g).to(torch.bfloat16)
        W = torch.randn(N, K, generator=g); b = torch.randn(N, generator=g)
        for lst in (A, B):
            lst.append((Z.to(DEV), X.to(DEV), M, N, K, 1.0, 0.01, W.to(DEV),
                        torch.zeros(N, pk, dtype=torch.bfloat16, device=DEV), None, b.to(DEV), None))
    W0 = [a[7].clone() for a in A]
    C.wgrad_sgd_multi(A, tile=129)
    for (Z, X, M_, N, K, al, lr, W, Wb, G, b, bg) in B:
        C.wgrad_sgd(Z, X, M_, N, K, alpha=al, lr=lr, W=W, Wb=Wb, bias=b)
    torch.cuda.synchronize()
    for li, (a, bb) in enumerate(zip(A, B)):
        d = (a[7] - bb[7]).abs()
        bad = (d > 0)
        nb = int(bad.sum())
        info = {"layer": li, "M": M, "W_bad": nb, "W_maxdiff": float(d.max()),
                "Wb_bad": int((a[8] != bb[8]).sum()), "b_bad": int((a[10] != bb[10]).sum()),
                "unchanged": int((a[7] == W0[li]).sum())}
        if nb:
            r, c = bad.nonzero(as_tuple=True)
            info["rows"] = sorted(set((r // 128).tolist()))[:10]
            info["cols"] = sorted(set((c // 128).tolist()))[:10]
            info["row_mod"] = sorted(set((r % 128).tolist()))[:20]
            info["col_mod"] = sorted(set((c % 128).tolist()))[:20]
            info["ref_upd_absmax"] = float((bb[7] - W0[li]).abs().max())
        print(info, flush=True)

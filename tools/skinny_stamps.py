"""Per-workgroup phase timeline of the skinny GEMMs (kernels/gemm_skinny.hip):
entry skew, K loop, wave reduction, split-K combine, epilogue (s_memrealtime,
100 MHz -> us), for the wide-MLP shapes.  JSON to argv[1]."""
import json
import statistics
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from hipdsml.ops.native import require_native  # noqa: E402

C = require_native()
dev = torch.device("cuda", 0)
out = {}
CASES = (("nt_4096x4096", False, 4096, 4096, 0), ("nn_4096x4096", True, 4096, 4096, 0),
         ("nt_4096x784", False, 4096, 784, 0), ("nt_4096x4096_s1", False, 4096, 4096, 1),
         ("nt_4096x4096_s8", False, 4096, 4096, 8),
         # the wide step's own epilogues: NT bias + ReLU + bf16 rows, NN ReLU'-mask + bf16 rows
         ("wide_f1_nt", False, 4096, 4096, 0), ("wide_b1_nn", True, 4096, 4096, 0))
for name, nn, N, K, sp in CASES:
    M = 64
    A = torch.randn(M, K, device=dev).to(torch.bfloat16)
    B = torch.randn(K, N, device=dev).to(torch.bfloat16) if nn else torch.randn(N, K, device=dev).to(torch.bfloat16)
    S = C.gemm_skinny_splits(M, N, K, sp)
    tiles = (N + 63) // 64
    wsw, ctw = C.gemm_skinny_ws(M, N, K, sp)
    ws = torch.zeros(max(wsw, 1), device=dev)
    ctr = torch.zeros(max(ctw, 1), dtype=torch.int32, device=dev)
    H = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    HT = torch.empty(N, M, dtype=torch.bfloat16, device=dev)
    if name.startswith("wide_"):
        bias = torch.randn(N, device=dev)
        mask = torch.randn(M, N, device=dev).to(torch.bfloat16)
        epi = dict(mask=mask, obf=H) if nn else dict(bias=bias, relu=True, obf=H)
    else:
        epi = dict(relu=True, obf=H, obfT=HT)
    for _ in range(3):
        C.gemm_skinny(A, B, M, N, K, nn=nn, splits=sp, ws=ws, ctr=ctr, **epi)
    torch.cuda.synchronize()
    C.gemm_skinny_set_stamping(True)
    C.gemm_skinny(A, B, M, N, K, nn=nn, splits=sp, ws=ws, ctr=ctr, **epi)
    torch.cuda.synchronize()
    C.gemm_skinny_set_stamping(False)
    v = C.gemm_skinny_stamps()
    nb = tiles * S
    st = [v[5 * b: 5 * b + 5] for b in range(nb)]
    t0 = min(s[0] for s in st)
    us = lambda x: round(x / 100.0, 2)  # noqa: E731
    rec = {"blocks": nb, "splits": S,
           "entry_spread": us(max(s[0] for s in st) - t0),
           "loop_med": us(statistics.median(s[1] - s[0] for s in st)),
           "loop_max": us(max(s[1] - s[0] for s in st)),
           "wave_red_med": us(statistics.median(s[2] - s[1] for s in st)),
           "combine_med": us(statistics.median(s[3] - s[2] for s in st)),
           "combine_max": us(max(s[3] - s[2] for s in st)),
           "epi_max": us(max(s[4] - s[3] for s in st)),
           "span": us(max(s[4] for s in st) - t0)}
    # per slice (the combiners are slice S-1): entry, loop end and exit, relative to the first entry
    tx = (N + 63) // 64
    for zz in sorted({0, S - 1}):
        ss = [st[b] for b in range(nb) if (b // tx) % S == zz]
        rec[f"z{zz}"] = {"entry_med": us(statistics.median(x[0] - t0 for x in ss)),
                         "entry_max": us(max(x[0] - t0 for x in ss)),
                         "loop_end_med": us(statistics.median(x[1] - t0 for x in ss)),
                         "loop_end_max": us(max(x[1] - t0 for x in ss)),
                         "red_med": us(statistics.median(x[2] - x[1] for x in ss)),
                         "comb_med": us(statistics.median(x[3] - x[2] for x in ss)),
                         "comb_max": us(max(x[3] - x[2] for x in ss)),
                         "epi_med": us(statistics.median(x[4] - x[3] for x in ss)),
                         "epi_max": us(max(x[4] - x[3] for x in ss)),
                         "exit_med": us(statistics.median(x[4] - t0 for x in ss)),
                         "exit_max": us(max(x[4] - t0 for x in ss))}
    out[name] = rec
    print(name, rec, flush=True)
if len(sys.argv) > 1:
    json.dump(out, open(sys.argv[1], "w"), indent=1)

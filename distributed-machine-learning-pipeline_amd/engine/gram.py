"""Gram tables of the persistent step's Gram form (kernels/mlp_persist.hip,
"Gram form"), as pure tensor functions so the layout the kernel indexes is
tested on its own (tests/test_gram_form.py).

With plain SGD, the next step's first-layer pre-activation needs the updated
W1 only through one product, so it can be computed before the update lands:

    Z1(s+1) = X(s+1) W1(s+1)^T + b1(s+1)
            = [X(s+1) W1(s)^T + b1(s)] - (lr/N) sum_r' (X(s+1) X_r'(s)^T + 1) dZ1_r'(s)

(dZ1 already carries the 1/batch factor; N replicas average their gradients).
The bracket is computed by the layer-1 blocks while dZ1(s) is still being
produced; the correction is a [64 x 64] . [64 x 128] product per replica over
a Gram block that depends on the data only, so it is tabulated once.

Layout: T[b][r'][m'][m] = X_r'(b-1)[m'] . X_rank(b)[m] + 1 with b - 1
wrapping over the shard's batches, i.e. the TRANSPOSE of the Gram block
G[m][m'] (the kernel reads column m' of G as one contiguous row).  Rows past
a short batch repeat its last row, as the kernel's X tiles do.  The single
replica's table is the N = 1 case with the replica axis dropped.

Reference: the per-step weight update this reorders is client.go:112-202
(forward, backward, SGD per sample)."""
from typing import Optional

import torch

ROWS = 64  # the persistent step's row tile


def _pad_rows(Xb: torch.Tensor) -> torch.Tensor:
    """[..., B, d0] -> [..., 64, d0], rows past B repeating row B - 1."""
    B = Xb.shape[-2]
    if B == ROWS:
        return Xb
    if B > ROWS:
        raise ValueError("the persistent step takes batches of <= 64 rows")
    idx = torch.clamp(torch.arange(ROWS, device=Xb.device), max=B - 1)
    return Xb.index_select(Xb.dim() - 2, idx)


def _bmm64(A: torch.Tensor, Bt: torch.Tensor) -> torch.Tensor:
    """A . Bt accumulated in float64, rounded once to fp32 (+ 1 added first):
    the table never depends on the process's matmul precision flags (a TF32 /
    xf32 GEMM would move the correction off the fp32 reference)."""
    return (torch.bmm(A.double(), Bt.double()) + 1.0).float()


def gram_table(Xb: torch.Tensor, step: int = 256, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Single replica: Xb [nb][B][d0] (the shard's batches in step order) ->
    T [nb][64][64], T[b][m'][m] = X(b-1)[m'] . X(b)[m] + 1 (fp32 of a float64
    product)."""
    Xp = _pad_rows(Xb.float())
    nb = Xp.shape[0]
    T = out if out is not None else torch.empty((nb, ROWS, ROWS), dtype=torch.float32, device=Xb.device)
    for b0 in range(0, nb, step):  # bounded temporaries for large shards
        b1 = min(nb, b0 + step)
        prev = Xp[torch.arange(b0 - 1, b1 - 1, device=Xp.device) % nb]
        T[b0:b1] = _bmm64(prev, Xp[b0:b1].transpose(1, 2))
    return T


def gram_table_dp(Xall: torch.Tensor, rank: int, step: int = 128) -> torch.Tensor:
    """Data parallel: Xall [N][nb][B][d0] (every replica's shard, rank order)
    -> T [nb][N][64][64], T[b][r'][m'][m] = X_r'(b-1)[m'] . X_rank(b)[m] + 1."""
    Xp = _pad_rows(Xall.float())
    N, nb = Xp.shape[0], Xp.shape[1]
    me = Xp[rank]
    T = torch.empty((nb, N, ROWS, ROWS), dtype=torch.float32, device=Xall.device)
    for b0 in range(0, nb, step):
        b1 = min(nb, b0 + step)
        prev_idx = torch.arange(b0 - 1, b1 - 1, device=Xp.device) % nb
        cur_t = me[b0:b1].transpose(1, 2)
        for r2 in range(N):
            T[b0:b1, r2] = _bmm64(Xp[r2][prev_idx], cur_t)
    return T.contiguous()


def gram_correction(T_b: torch.Tensor, dZ1: torch.Tensor, lr: float) -> torch.Tensor:
    """The correction the gk = 0 layer-1 blocks add, in the kernel's
    indexing: T_b [N][64 m'][64 m] (one batch's table rows), dZ1 [N][64][n]
    (every replica's activation gradient, rank order) -> C [64][n] =
    -lr sum_r' sum_m' T_b[r'][m'][m] dZ1[r'][m'][:] (lr already / N)."""
    return -lr * torch.einsum("rpm,rpn->mn", T_b, dZ1)

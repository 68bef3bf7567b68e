"""The Gram form of the persistent step (engine/gram.py, kernels/mlp_persist.hip):
the tables' layout as the kernel indexes it, and the identity the kernel relies
on -- the next step's first-layer pre-activation from the OLD weights plus the
tabulated correction equals the one from the updated weights -- for one
replica and for N replicas (their gradients averaged), with full and short
batches.  CPU only (float64, so a layout slip cannot hide in rounding)."""
import pytest
import torch

from hipdsml.engine.gram import ROWS, gram_correction, gram_table, gram_table_dp


def _pad(xb, B):
    idx = torch.clamp(torch.arange(ROWS), max=B - 1)
    return xb[idx]


@pytest.mark.parametrize("B", [64, 48])
def test_single_table_layout(B):
    g = torch.Generator().manual_seed(1)
    nb, d0 = 3, 40
    X = torch.rand(nb, B, d0, generator=g, dtype=torch.float64)
    T = gram_table(X)
    assert T.shape == (nb, ROWS, ROWS) and T.dtype == torch.float32
    for b in range(nb):
        prev, cur = _pad(X[(b - 1) % nb], B), _pad(X[b], B)
        want = prev @ cur.T + 1.0  # [m'][m]
        torch.testing.assert_close(T[b].double(), want, rtol=1e-6, atol=1e-5)


def test_dp_table_layout_and_single_case():
    g = torch.Generator().manual_seed(2)
    N, nb, B, d0 = 3, 4, 64, 24
    Xall = torch.rand(N, nb, B, d0, generator=g)
    for rank in range(N):
        T = gram_table_dp(Xall, rank)
        assert T.shape == (nb, N, ROWS, ROWS) and T.is_contiguous()
        for b in range(nb):
            for r2 in range(N):
                want = Xall[r2][(b - 1) % nb] @ Xall[rank][b].T + 1.0
                torch.testing.assert_close(T[b, r2], want, rtol=1e-5, atol=1e-4)
    # one replica: the data-parallel table is the single-replica one
    torch.testing.assert_close(gram_table_dp(Xall[:1], 0)[:, 0], gram_table(Xall[0]))


@pytest.mark.parametrize("N,B", [(1, 64), (2, 64), (3, 48)])
def test_gram_identity(N, B):
    """Z1(s+1) = X(s+1) W1(s+1)^T + b1(s+1), with W1(s+1) = W1(s) - (lr/N) sum_r
    dZ1_r^T X_r(s) and b1(s+1) = b1(s) - (lr/N) sum_r colsum(dZ1_r), equals the
    bracket from the old weights plus gram_correction over the table."""
    g = torch.Generator().manual_seed(10 * N + B)
    nb, d0, d1, lr = 3, 56, 32, 0.05
    Xall = torch.rand(N, nb, B, d0, generator=g, dtype=torch.float64)
    W1 = torch.randn(d1, d0, generator=g, dtype=torch.float64) * 0.1
    b1 = torch.randn(d1, generator=g, dtype=torch.float64) * 0.1
    s = 4
    b_s, b_n = s % nb, (s + 1) % nb
    # dZ1 of step s per replica: padded rows (past a short batch) carry none
    dZ1 = torch.randn(N, ROWS, d1, generator=g, dtype=torch.float64) / B
    dZ1[:, B:] = 0.0
    Xs = torch.stack([_pad(Xall[r][b_s], B) for r in range(N)])  # [N][64][d0]
    W1n = W1 - (lr / N) * sum(dZ1[r].T @ Xs[r] for r in range(N))
    b1n = b1 - (lr / N) * dZ1.sum(dim=(0, 1))
    for rank in range(N):
        Xn = _pad(Xall[rank][b_n], B)
        direct = Xn @ W1n.T + b1n
        T = gram_table_dp(Xall, rank).double()
        gram = (Xn @ W1.T + b1) + gram_correction(T[b_n], dZ1, lr / N)
        torch.testing.assert_close(gram[:B], direct[:B], rtol=1e-4, atol=1e-5)

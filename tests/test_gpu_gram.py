"""kernels/gram.hip: the Gram tables of the persistent step's Gram form,
against engine/gram.py (the float64 torch oracle): single replica and
data-parallel layouts, full and short batches, K with and without a 16-tail.
Reference data path these tables reorder: client.go:112-202."""
import pytest
import torch

from hipdsml.engine.gram import gram_table, gram_table_dp

pytestmark = pytest.mark.gpu


def _C():
    from hipdsml.ops.native import require_native

    return require_native()


@pytest.mark.parametrize("nb,B,K", [(5, 64, 784), (3, 48, 784), (4, 64, 40), (1, 17, 56)])
def test_gram_table_single_matches_float64_oracle(nb, B, K):
    g = torch.Generator().manual_seed(nb * 100 + B + K)
    X = torch.rand(nb * B, K, generator=g)
    want = gram_table(X.view(nb, B, K))
    got = _C().gram_table(X.cuda(), X.cuda(), nb, B, K)
    torch.cuda.synchronize()
    assert got.shape == (nb, 64, 64)
    torch.testing.assert_close(got.cpu(), want, rtol=2e-7, atol=1e-5)


@pytest.mark.parametrize("N,B", [(2, 64), (3, 48), (8, 64)])
def test_gram_table_dp_matches_float64_oracle(N, B):
    g = torch.Generator().manual_seed(N * 7 + B)
    nb, K = 4, 784
    Xall = torch.rand(N, nb * B, K, generator=g)
    for rank in (0, N - 1):
        want = gram_table_dp(Xall.view(N, nb, B, K), rank)
        got = _C().gram_table(Xall.cuda(), Xall[rank].cuda(), nb, B, K)
        torch.cuda.synchronize()
        assert got.shape == (nb, N, 64, 64)
        torch.testing.assert_close(got.cpu(), want, rtol=2e-7, atol=1e-5)


def test_gram_table_strided_rows_and_mnist_scale():
    """Rows with padding columns (ld > K), real-pixel magnitudes (dot products of
    a few hundred): one fp32 rounding of the fp64 sum, as the oracle."""
    g = torch.Generator().manual_seed(3)
    nb, B, K = 6, 64, 784
    Xp = torch.zeros(nb * B, 800)
    Xp[:, :K] = (torch.rand(nb * B, K, generator=g) > 0.6).float() * torch.rand(nb * B, K, generator=g)
    want = gram_table(Xp[:, :K].reshape(nb, B, K))
    got = _C().gram_table(Xp.cuda()[:, :K], Xp.cuda()[:, :K], nb, B, K)
    torch.cuda.synchronize()
    torch.testing.assert_close(got.cpu(), want, rtol=2e-7, atol=1e-5)

"""Fragment-order layout of the activation exchange (kernels/mlp_f32_xact.hip):
the host-side input swizzle must match the kernel's lane map exactly."""
import pytest
import torch

from hipdsml.parallel.xchg import swizzle_inputs


@pytest.mark.parametrize("batch", [64, 48, 16])
def test_swizzle_inputs_lane_map(batch):
    N, nb, K = 3, 2, 48
    X = torch.randn(N, nb * batch + 5, K)  # trailing rows beyond whole batches are dropped
    S = swizzle_inputs(X, batch)
    assert S.shape == (N, nb, K // 16, 4, 64, 4)
    for r in range(N):
        for b in range(nb):
            for t in range(K // 16):
                for w in range(4):
                    for lane in range(64):
                        i, q = lane & 15, lane >> 4
                        for j in range(4):
                            row = 4 * w + 16 * j + q  # wave w's k-step s = w + 4j, row 4s + q
                            want = X[r, b * batch + row, 16 * t + i] if row < batch else 0.0
                            assert S[r, b, t, w, lane, j] == want


def test_swizzle_rejects_unaligned():
    with pytest.raises(ValueError):
        swizzle_inputs(torch.zeros(1, 64, 40), 64)
    with pytest.raises(ValueError):
        swizzle_inputs(torch.zeros(1, 128, 32), 128)

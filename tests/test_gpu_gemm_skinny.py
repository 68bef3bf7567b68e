"""Skinny bf16 GEMMs (kernels/gemm_skinny.hip) against the fp32 torch product of
the same bf16 operands: NT (forward, B = W [N x K]) and NN (dgrad, B = W
[K x N] read through transposing LDS reads), split-K with the last-arriver
reduction, every fused epilogue output, K / N / M tails, one workspace
shared by launches of different shapes."""
import pytest
import torch

from hipdsml.ops.native import require_native

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _ref(A, B, nn):
    return A.float() @ (B.float() if nn else B.float().t())


def _ws(M, N, K, splits=0):
    C = require_native()
    wsw, ctw = C.gemm_skinny_ws(M, N, K, splits)
    return (torch.zeros(max(wsw, 1), device=DEV), torch.zeros(max(ctw, 1), dtype=torch.int32, device=DEV))


@pytest.mark.parametrize("nn", [False, True])
@pytest.mark.parametrize("M,N,K,splits", [
    (64, 4096, 4096, 0), (64, 4096, 784, 0), (64, 512, 4096, 1), (64, 512, 4096, 3),
    (48, 136, 200, 2), (128, 256, 1024, 0), (64, 64, 64, 1), (17, 72, 1000, 0)])
def test_skinny_matches_fp32(nn, M, N, K, splits):
    C = require_native()
    g = torch.Generator(device="cpu").manual_seed(M * 7 + N + K)
    A = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16)
    B = (torch.randn(K, N, generator=g) if nn else torch.randn(N, K, generator=g)).to(DEV, torch.bfloat16)
    S = C.gemm_skinny_splits(M, N, K, splits)
    ws, ctr = _ws(M, N, K, splits)
    want = _ref(A, B, nn)
    for _ in range(3):  # back-to-back launches on one workspace
        out = torch.full((M, N), float("nan"), device=DEV)
        got = C.gemm_skinny(A, B, M, N, K, nn=nn, of32=out, splits=splits, ws=ws, ctr=ctr)
        assert got == S
        torch.cuda.synchronize()
        err = (out - want).abs().max().item()
        assert err <= 2e-5 * K ** 0.5 * want.abs().max().item() + 1e-4, err
    assert int(ctr.abs().sum().item()) == 0  # tickets re-armed


@pytest.mark.parametrize("nn", [False, True])
def test_skinny_epilogue_bias_relu_mask_and_copies(nn):
    C = require_native()
    M, N, K = 64, 1024, 2048
    g = torch.Generator(device="cpu").manual_seed(5)
    A = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16)
    B = (torch.randn(K, N, generator=g) if nn else torch.randn(N, K, generator=g)).to(DEV, torch.bfloat16)
    bias = torch.randn(N, generator=g).to(DEV)
    mask = torch.randn(M, N, generator=g).to(DEV, torch.bfloat16)
    ws, ctr = _ws(M, N, K)
    o32 = torch.empty(M, N, device=DEV)
    obf = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    obfT = torch.empty(N, M, dtype=torch.bfloat16, device=DEV)
    C.gemm_skinny(A, B, M, N, K, nn=nn, alpha=0.5, bias=bias, relu=True, mask=mask, of32=o32, obf=obf,
                  obfT=obfT, ws=ws, ctr=ctr)
    torch.cuda.synchronize()
    want = torch.relu(0.5 * _ref(A, B, nn) + bias) * (mask.float() > 0)
    tol = 2e-5 * K ** 0.5 * want.abs().max().item() + 1e-4
    assert (o32 - want).abs().max().item() <= tol
    assert torch.equal(obf, o32.to(torch.bfloat16))
    assert torch.equal(obfT, obf.t())


def test_skinny_repeated_calls_are_bit_identical():
    """Split-K reduction in slice order: the same bits whichever slice lands last."""
    C = require_native()
    M, N, K = 64, 4096, 4096
    A = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    B = torch.randn(N, K, device=DEV).to(torch.bfloat16)
    ws, ctr = _ws(M, N, K)
    outs = []
    for _ in range(5):
        o = torch.empty(M, N, device=DEV)
        C.gemm_skinny(A, B, M, N, K, of32=o, ws=ws, ctr=ctr)
        outs.append(o)
    torch.cuda.synchronize()
    assert all(torch.equal(outs[0], o) for o in outs[1:])


def test_skinny_shared_workspace_across_shapes():
    """One ws / ctr pair serving launches of different tile counts and split
    counts, interleaved (as the wide engine shares them)."""
    C = require_native()
    g = torch.Generator(device="cpu").manual_seed(11)
    shapes = [(64, 4096, 4096, 0, False), (64, 512, 4096, 3, True), (64, 1024, 2048, 0, False),
              (64, 4096, 784, 0, True), (64, 512, 4096, 7, False)]
    wsw = max(C.gemm_skinny_ws(M, N, K, sp)[0] for (M, N, K, sp, _) in shapes)
    ctw = max(C.gemm_skinny_ws(M, N, K, sp)[1] for (M, N, K, sp, _) in shapes)
    ws = torch.zeros(wsw, device=DEV)
    ctr = torch.zeros(ctw, dtype=torch.int32, device=DEV)
    ops = []
    for (M, N, K, sp, nn) in shapes:
        A = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16)
        B = (torch.randn(K, N, generator=g) if nn else torch.randn(N, K, generator=g)).to(DEV, torch.bfloat16)
        ops.append((A, B, M, N, K, sp, nn, _ref(A, B, nn)))
    for rep in range(3):
        for (A, B, M, N, K, sp, nn, want) in ops[rep % 2:] + ops[:rep % 2]:
            out = torch.full((M, N), float("nan"), device=DEV)
            C.gemm_skinny(A, B, M, N, K, nn=nn, of32=out, splits=sp, ws=ws, ctr=ctr)
            torch.cuda.synchronize()
            err = (out - want).abs().max().item()
            assert err <= 2e-5 * K ** 0.5 * want.abs().max().item() + 1e-4, (M, N, K, sp, err)
    assert int(ctr.abs().sum().item()) == 0


@pytest.mark.parametrize("M,N,K", [(64, 4096, 4096), (64, 4096, 784), (64, 10, 4096), (48, 200, 136),
                                   (128, 64, 256)])
def test_wgrad_sgd_matches_fp32(M, N, K):
    """W -= lr * alpha * Z^T X from ROW-MAJOR activations (transposing LDS reads),
    bf16 copy refreshed, bias step from the column sums of Z."""
    C = require_native()
    g = torch.Generator(device="cpu").manual_seed(N + K + M)
    pn, pk = (N + 15) // 16 * 16, (K + 15) // 16 * 16
    Z = torch.zeros(M, pn, dtype=torch.bfloat16, device=DEV)
    X = torch.zeros(M, pk, dtype=torch.bfloat16, device=DEV)
    Z[:, :N] = torch.randn(M, N, generator=g).to(DEV, torch.bfloat16)
    X[:, :K] = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16)
    W = torch.randn(N, K, generator=g).to(DEV)
    b = torch.randn(N, generator=g).to(DEV)
    W0, b0 = W.clone(), b.clone()
    Wb = torch.zeros(N, pk, dtype=torch.bfloat16, device=DEV)
    lr, alpha = 0.01, 0.25
    C.wgrad_sgd(Z, X, M, N, K, alpha=alpha, lr=lr, W=W, Wb=Wb, bias=b)
    torch.cuda.synchronize()
    Gref = alpha * Z[:, :N].float().t() @ X[:, :K].float()
    want = W0 - lr * Gref
    assert (W - want).abs().max().item() < 1e-5 * max(1.0, M ** 0.5)
    assert torch.equal(Wb[:, :K], W.to(torch.bfloat16))
    bref = b0 - lr * alpha * Z[:, :N].float().sum(0)
    assert (b - bref).abs().max().item() < 1e-5 * max(1.0, M ** 0.5)
    # gradient-out form (multi-replica: all-reduced before the update)
    G = torch.full((N, K), float("nan"), device=DEV)
    db = torch.zeros(N, device=DEV)
    C.wgrad_sgd(Z, X, M, N, K, alpha=alpha, G=G, bgrad=db)
    torch.cuda.synchronize()
    assert (G - Gref).abs().max().item() < 1e-4
    assert (db - alpha * Z[:, :N].float().sum(0)).abs().max().item() < 1e-4


@pytest.mark.parametrize("tile,M", [(64, 64), (0, 64), (128, 64), (0, 512), (128, 48), (128, 200),
                                    (128, 8), (64, 512)])
def test_wgrad_sgd_multi_matches_per_layer_launches(tile, M):
    """Three layers' updates in one flattened launch == one launch per layer
    (64 x 64 tiles), bit for bit -- also with the 128 x 128 tiles (tile 128) of
    the big layers, whose 32-row batch blocks stream through a 4-slot LDS
    ring: the same MFMA order per element, the same bias-sum order.  M = 512 is the global batch
    of the activation-exchange sync at 8 replicas; 48 / 200 have a batch tail."""
    C = require_native()
    g = torch.Generator(device="cpu").manual_seed(77 + M)
    shapes = [(10, 4096), (4096, 4096), (4096, 784)]  # (N, K) of the wide MLP's layers, top down
    args_a, args_b = [], []
    for N, K in shapes:
        pn, pk = (N + 15) // 16 * 16, (K + 15) // 16 * 16
        Z = torch.zeros(M, pn, dtype=torch.bfloat16)
        X = torch.zeros(M, pk, dtype=torch.bfloat16)
        Z[:, :N] = torch.randn(M, N, generator=g).to(torch.bfloat16)
        X[:, :K] = torch.randn(M, K, generator=g).to(torch.bfloat16)
        W = torch.randn(N, K, generator=g)
        b = torch.randn(N, generator=g)
        for lst in (args_a, args_b):
            lst.append((Z.to(DEV), X.to(DEV), M, N, K, 1.0, 0.01, W.to(DEV),
                        torch.zeros(N, pk, dtype=torch.bfloat16, device=DEV), None, b.to(DEV), None))
    C.wgrad_sgd_multi(args_a, tile=tile)
    for (Z, X, M_, N, K, al, lr, W, Wb, G, b, bg) in args_b:
        C.wgrad_sgd(Z, X, M_, N, K, alpha=al, lr=lr, W=W, Wb=Wb, bias=b)
    torch.cuda.synchronize()
    for a, b in zip(args_a, args_b):
        assert torch.equal(a[7], b[7]) and torch.equal(a[8], b[8]) and torch.equal(a[10], b[10])


@pytest.mark.parametrize("M", [64, 512])
def test_wgrad_sgd_multi_big_tiles_gradient_form(M):
    """The 128 x 128 tiles in the gradient-out form (W = None: G and db written
    for an all-reduce) against fp32."""
    C = require_native()
    g = torch.Generator(device="cpu").manual_seed(5 + M)
    N, K = 512, 784
    Z = torch.randn(M, N, generator=g).to(DEV, torch.bfloat16)
    X = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16)
    G = torch.full((N, K), float("nan"), device=DEV)
    db = torch.zeros(N, device=DEV)
    C.wgrad_sgd_multi([(Z, X, M, N, K, 0.5, 0.0, None, None, G, None, db)], tile=128)
    torch.cuda.synchronize()
    Gref = 0.5 * Z.float().t() @ X.float()
    assert (G - Gref).abs().max().item() < 1e-4 * max(1.0, M ** 0.5)
    assert (db - 0.5 * Z.float().sum(0)).abs().max().item() < 1e-4 * max(1.0, M ** 0.5)


@pytest.mark.parametrize("M", [64, 256, 512])
def test_wgrad_rowblk_matches_square_tiles(M):
    """The row-block form of the split-master update (tile=256: Z^T resident in
    registers, X streamed through a one-tile LDS ring; what sync=xact runs from
    M = 256 on) against the 64 x 64 tiles: the same 32-row MFMA sequence per
    element, so the updated hi / lo words are bit-identical; the bias sums run
    in another order (tolerance).  Shapes with an n tail (200 rows: a partial
    128-row block), a k tail (784 = 12 x 64 + 16) and the 10-row classifier;
    more units than workgroups, so runs cross n blocks and layers."""
    C = require_native()
    g = torch.Generator(device="cpu").manual_seed(123 + M)
    # (4096, 512): 32 n blocks of 128 rows x 8 k tiles -- the XCD-split walk on 256 CUs
    shapes = [(10, 1024), (200, 784), (1024, 1024), (4096, 512)]
    runs = {}
    for tile in (64, 256):
        args = []
        for N, K in shapes:
            pn, pk = (N + 15) // 16 * 16, (K + 15) // 16 * 16
            g.manual_seed(7 * N + K + M)
            Z = torch.zeros(M, pn, dtype=torch.bfloat16)
            X = torch.zeros(M, pk, dtype=torch.bfloat16)
            Z[:, :N] = torch.randn(M, N, generator=g).to(torch.bfloat16)
            X[:, :K] = torch.randn(M, K, generator=g).to(torch.bfloat16)
            W = torch.randn(N, pk, generator=g)
            W[:, K:] = 0
            Wh = torch.zeros(N, pk, dtype=torch.bfloat16, device=DEV)
            Wl = torch.zeros(N, pk, dtype=torch.int16, device=DEV)
            C.hilo_split(W.to(DEV), Wh, Wl)
            b = torch.randn(N, generator=g).to(DEV)
            args.append((Z.to(DEV), X.to(DEV), M, N, K, 0.5, 0.01, None,
                         torch.zeros(N, pk, dtype=torch.bfloat16, device=DEV), None, b, None, Wh, Wl))
        C.wgrad_sgd_multi(args, tile=tile)
        torch.cuda.synchronize()
        runs[tile] = args
    for a64, a256 in zip(runs[64], runs[256]):
        assert torch.equal(a64[8], a256[8]), "updated hi words differ"
        assert torch.equal(a64[13], a256[13]), "updated lo words differ"
        assert (a64[10] - a256[10]).abs().max().item() < 1e-4 * max(1.0, M ** 0.5)
    # and against fp32: W - lr * alpha * Z^T X
    for (Z, X, M_, N, K, al, lr, _, Wb, _, b, _, Wh, Wl) in runs[256]:
        Wn = torch.zeros(N, Wb.shape[1], device=DEV)
        C.hilo_join(Wb, Wl, Wn)
        g.manual_seed(7 * N + K + M)
        Zr = torch.randn(M, N, generator=g).to(torch.bfloat16).float()
        Xr = torch.randn(M, K, generator=g).to(torch.bfloat16).float()
        W0 = torch.randn(N, (K + 15) // 16 * 16, generator=g)[:, :K]
        want = W0 - lr * al * (Zr.t() @ Xr)
        assert (Wn[:, :K].cpu() - want).abs().max().item() < 1e-4 * max(1.0, M ** 0.5)



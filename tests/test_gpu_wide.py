"""bf16 MFMA GEMM toolkit and the wide-MLP engine vs fp32 PyTorch references."""
import pytest
import torch

from hipdsml.data.mnist import synthetic_mnist
from hipdsml.engine.wide import WideMlpTrainer
from hipdsml.models.mlp import MlpLayout, MlpSpec, grads_ref, init_params
from hipdsml.ops.native import require_native

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


@pytest.mark.parametrize("M,N,K,splits", [(64, 4096, 4096, 8), (50, 70, 72, 1), (64, 784, 64, 1),
                                          (4096, 128, 64, 1), (64, 10, 4096, 16), (33, 130, 520, 3)])
def test_gemm_bf16_nt(M, N, K, splits):
    C = require_native()
    g = torch.Generator().manual_seed(M + N + K)
    A = torch.randn(M, K, generator=g).to(torch.bfloat16)
    B = torch.randn(N, K, generator=g).to(torch.bfloat16)
    bias = torch.randn(N, generator=g)
    want = A.float() @ B.float().t() + bias
    Ad, Bd = A.to(DEV), B.to(DEV)
    S = C.gemm_num_splits(K, splits)
    Cp = torch.empty(S * M * N, device=DEV)
    assert C.gemm_bf16_nt(Ad, Bd, Cp, M, N, K, splits) == S
    out = torch.empty(M, N, device=DEV)
    outb = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    outT = torch.empty(N, M, dtype=torch.bfloat16, device=DEV)
    C.gemm_epilogue(Cp, S, M, N, bias=bias.to(DEV), of32=out, obf=outb, obfT=outT)
    torch.cuda.synchronize()
    tol = 1e-3 * K ** 0.5
    assert (out.cpu() - want).abs().max().item() < tol
    assert torch.equal(outT.cpu().t(), outb.cpu())
    assert torch.equal(outb.cpu(), out.cpu().to(torch.bfloat16))
    # relu + mask epilogue
    mask = (torch.randn(M, N, generator=g) > 0).to(torch.bfloat16)
    C.gemm_epilogue(Cp, S, M, N, relu=True, mask=mask.to(DEV), of32=out)
    torch.cuda.synchronize()
    ref = torch.relu(A.float() @ B.float().t()) * (mask.float() > 0)
    assert (out.cpu() - ref).abs().max().item() < tol


def test_wide_step_matches_fp32_reference():
    spec = MlpSpec((784, 256, 128, 10))
    ds = synthetic_mnist(64 * 2, seed=3)
    tr = WideMlpTrainer(spec, ds, batch=64, lr=0.05, seed=1)
    lay = MlpLayout(spec, 64, 1)
    P0 = init_params(lay, 1, "kaiming")
    tr.train_steps(1)
    tr.synchronize()
    g_ref, loss_sum, corr = grads_ref(lay, P0, ds.X[:64], ds.y[:64])
    g = (P0 - tr.P.cpu()) / 0.05  # single replica: SGD is fused, recover the applied gradient
    cos = torch.nn.functional.cosine_similarity(g, g_ref, dim=0).item()
    assert cos > 0.999, cos
    rel = (g - g_ref).norm().item() / g_ref.norm().item()
    assert rel < 0.05, rel  # bf16 activations / dZ: ~0.4 % per element, compounded over layers
    st = tr.read_stats()
    assert st.count == 64 and abs(st.loss_sum - float(loss_sum)) / float(loss_sum) < 0.02
    # the bf16 GEMM copy IS the high half of the split fp32 master: the
    # master's bits rounded half away from zero (RNE but at exact ties), and
    # high half + int16 remainder rebuild the master exactly
    W0, _ = tr.views[0]
    bits = W0.cpu().contiguous().view(torch.int32).to(torch.int64) & 0xFFFFFFFF
    hi = ((bits + 0x8000) >> 16) & 0xFFFF
    got = tr.wb(0)[:256, :784].cpu().contiguous().view(torch.int16).to(torch.int64) & 0xFFFF
    assert torch.equal(got, hi)
    lo = tr.Wlo[0][:256, :784].cpu().to(torch.int64)
    assert torch.equal(((hi << 16) + lo) & 0xFFFFFFFF, bits)
    rne = W0.cpu().to(torch.bfloat16).view(torch.int16).to(torch.int64) & 0xFFFF
    ties = (bits & 0xFFFF) == 0x8000
    assert torch.equal(got[~ties], rne[~ties])


@pytest.mark.parametrize("graph", [False, True])
def test_wide_training_converges(graph):
    spec = MlpSpec((784, 1024, 1024, 10))
    ds = synthetic_mnist(64 * 40, seed=4)
    tr = WideMlpTrainer(spec, ds, batch=64, lr=0.05, seed=2, graph=graph)
    tr.train_steps(40)
    first = tr.read_stats()
    tr.train_steps(120)
    last = tr.read_stats()
    assert last.avg_loss < first.avg_loss
    assert last.accuracy > 90.0


@pytest.mark.parametrize("M,N,K", [(64, 4096, 4096), (64, 10, 4096), (64, 4096, 16), (50, 70, 520),
                                   (64, 4096, 784), (130, 48, 96)])
def test_gemm_rows64_epilogues(M, N, K):
    """Batch-row kernel (full K per block, 4-way in-block K split) vs fp32."""
    C = require_native()
    g = torch.Generator().manual_seed(M + 7 * N + K)
    A = torch.randn(M, K, generator=g).to(torch.bfloat16)
    B = torch.randn(N, K, generator=g).to(torch.bfloat16)
    bias = torch.randn(N, generator=g)
    mask = (torch.randn(M, N, generator=g) > 0).to(torch.bfloat16)
    ref = A.float() @ B.float().t()
    tol = 1e-3 * K ** 0.5
    Ad, Bd = A.to(DEV), B.to(DEV)
    o32 = torch.empty(M, N, device=DEV)
    ob = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    Mt = (M + 15) // 16 * 16
    obT = torch.zeros(N, Mt, dtype=torch.bfloat16, device=DEV)
    C.gemm_bf16_nt_fused(Ad, Bd, M, N, K, bias=bias.to(DEV), relu=True, of32=o32, obf=ob,
                         obfT=obT, splits=0)
    torch.cuda.synchronize()
    want = torch.relu(ref + bias)
    assert (o32.cpu() - want).abs().max().item() < tol
    assert torch.equal(ob.cpu(), o32.cpu().to(torch.bfloat16))
    assert torch.equal(obT.cpu()[:, :M].t(), ob.cpu())
    C.gemm_bf16_nt_fused(Ad, Bd, M, N, K, mask=mask.to(DEV), of32=o32, splits=0)
    torch.cuda.synchronize()
    assert (o32.cpu() - ref * (mask.float() > 0)).abs().max().item() < tol


@pytest.mark.parametrize("C_,K", [(10, 4096), (16, 784), (3, 64)])
def test_head_softmax_xent(C_, K):
    C = require_native()
    B = 64
    g = torch.Generator().manual_seed(C_ * K)
    H = torch.randn(B, K, generator=g).to(torch.bfloat16)
    W = (0.05 * torch.randn(C_, K, generator=g)).to(torch.bfloat16)
    b = torch.randn(C_, generator=g)
    y = torch.randint(0, C_, (B,), generator=g, dtype=torch.int32)
    logits = torch.empty(B, C_, device=DEV)
    Cp = (C_ + 15) // 16 * 16
    dz = torch.zeros(B, Cp, dtype=torch.bfloat16, device=DEV)
    dzT = torch.zeros(Cp, B, dtype=torch.bfloat16, device=DEV)
    stats = torch.zeros(4, device=DEV)
    C.head_softmax_xent(H.to(DEV), W.to(DEV), b.to(DEV), B, K, C_, y.to(DEV), 1.0 / B, logits, dz,
                        dzT, stats)
    torch.cuda.synchronize()
    z = H.float() @ W.float().t() + b
    assert (logits.cpu() - z).abs().max().item() < 1e-3
    p = torch.softmax(z, 1)
    onehot = torch.nn.functional.one_hot(y.long(), C_).float()
    want = (p - onehot) / B
    assert (dz.cpu()[:, :C_].float() - want).abs().max().item() < 1e-3
    assert torch.equal(dzT.cpu()[:C_].t(), dz.cpu()[:, :C_])
    assert stats[2].item() == B
    loss = -torch.log(p.gather(1, y.long().view(-1, 1)) + 1e-10).sum().item()
    assert abs(stats[0].item() - loss) / loss < 1e-3
    # per-row accumulators (no atomics): the rows' sums equal the atomic totals
    rows = torch.zeros(B * 4, device=DEV)
    C.head_softmax_xent(H.to(DEV), W.to(DEV), b.to(DEV), B, K, C_, y.to(DEV), 1.0 / B, logits, dz,
                        dzT, rows, row_stats=True)
    torch.cuda.synchronize()
    tot = rows.view(-1, 4).sum(0)
    assert tot[2].item() == B and torch.all(rows.view(-1, 4)[:, 2] == 1)
    assert abs(tot[0].item() - loss) / loss < 1e-3 and tot[1].item() == stats[1].item()
    # fused next activation gradient: dZ_prev = (bf16(dZ) . W) * (H > 0)
    Kp = (K + 15) // 16 * 16
    dzp = torch.zeros(B, Kp, dtype=torch.bfloat16, device=DEV)
    dzpT = torch.zeros(Kp, B, dtype=torch.bfloat16, device=DEV)
    C.head_softmax_xent(H.to(DEV), W.to(DEV), b.to(DEV), B, K, C_, y.to(DEV), 1.0 / B, logits, dz,
                        dzT, stats, dzp=dzp, dzpT=dzpT)
    torch.cuda.synchronize()
    dzb = dz.cpu()[:, :C_].float()
    want = (dzb @ W.float()) * (H.float() > 0)
    got = dzp.cpu()[:, :K].float()
    assert (got - want).abs().max().item() < 1e-2 * max(1.0, want.abs().max().item())
    assert torch.equal(dzpT.cpu()[:K].t(), dzp.cpu()[:, :K])


@pytest.mark.parametrize("gemm", ["skinny", "rows64"])
def test_wide_gemm_variants_train_identically_close(gemm):
    spec = MlpSpec((784, 512, 256, 10))
    ds = synthetic_mnist(64 * 4, seed=8)
    t = WideMlpTrainer(spec, ds, batch=64, lr=0.05, seed=4, graph=False, gemm=gemm)
    t.train_steps(8)
    st = t.read_stats()
    assert st.count == 8 * 64 and st.avg_loss < 2.5


def test_wide_native_evaluate_matches_fp32_forward():
    """evaluate() runs the step's bf16 kernels (incl. a short last batch) and
    agrees with the fp32 torch forward of the master weights."""
    from hipdsml.models.mlp import forward_ref

    spec = MlpSpec((784, 512, 256, 10))
    ds = synthetic_mnist(64 * 20, seed=9)
    t = WideMlpTrainer(spec, ds, batch=64, lr=0.05, seed=6, graph=False)
    t.train_steps(40)
    ev = synthetic_mnist(64 * 5 + 24, seed=10)
    got = t.evaluate(ev)
    assert got["n"] == len(ev)
    logits, _ = forward_ref(t.layout, t.P, ev.X.to(DEV))
    y = ev.y.to(DEV).long()
    acc = 100.0 * (logits.argmax(1) == y).float().mean().item()
    loss = torch.nn.functional.cross_entropy(logits, y).item()
    assert abs(got["accuracy"] - acc) <= 2.0, (got, acc)
    assert abs(got["loss"] - loss) <= 0.02 * max(1.0, loss), (got, loss)


def test_wide_graph_matches_eager():
    spec = MlpSpec((784, 256, 128, 10))
    ds = synthetic_mnist(64 * 4, seed=5)
    a = WideMlpTrainer(spec, ds, batch=64, lr=0.05, seed=3, graph=False)
    b = WideMlpTrainer(spec, ds, batch=64, lr=0.05, seed=3, graph=True)
    a.train_steps(10)
    b.train_steps(10)
    a.synchronize(); b.synchronize()
    assert torch.equal(a.P.cpu(), b.P.cpu())


@pytest.mark.parametrize("M,N,K,splits", [(64, 4096, 4096, 8), (64, 10, 4096, 32), (50, 70, 520, 3),
                                          (64, 784, 64, 1), (33, 130, 1024, 5)])
def test_gemm_splitk_fused_epilogue_matches_two_kernel_path(M, N, K, splits):
    """In-kernel split-K reduction (last split per tile) == slabs + gemm_epilogue,
    bit for bit, and the tile counters are left re-armed."""
    C = require_native()
    g = torch.Generator().manual_seed(M * N + K)
    A = torch.randn(M, K, generator=g).to(torch.bfloat16).to(DEV)
    B = torch.randn(N, K, generator=g).to(torch.bfloat16).to(DEV)
    bias = torch.randn(N, generator=g).to(DEV)
    mask = (torch.randn(M, N, generator=g) > 0).to(torch.bfloat16).to(DEV)
    S = C.gemm_num_splits(K, splits)
    tiles = ((M + 63) // 64) * ((N + 63) // 64)
    Cp = torch.zeros(max(S * M * N, S * tiles * 4096), device=DEV)
    ctr = torch.zeros(tiles, dtype=torch.int32, device=DEV)
    tr = M % 4 == 0  # transposed bf16 output needs 8 B runs along M
    for relu, use_mask in ((True, False), (False, True)):
        want32 = torch.empty(M, N, device=DEV)
        wantT = torch.zeros(N, M, dtype=torch.bfloat16, device=DEV) if tr else None
        C.gemm_bf16_nt(A, B, Cp, M, N, K, splits)
        C.gemm_epilogue(Cp, S, M, N, bias=bias, relu=relu, mask=mask if use_mask else None,
                        of32=want32, obfT=wantT)
        got32 = torch.empty(M, N, device=DEV)
        gotT = torch.zeros(N, M, dtype=torch.bfloat16, device=DEV) if tr else None
        assert C.gemm_bf16_nt_fused(A, B, M, N, K, bias=bias, relu=relu,
                                    mask=mask if use_mask else None, of32=got32, obfT=gotT,
                                    splits=splits, ws=Cp, ctr=ctr) == S
        torch.cuda.synchronize()
        assert torch.equal(got32.cpu(), want32.cpu())
        if tr:
            assert torch.equal(gotT.cpu(), wantT.cpu())
        assert int(ctr.abs().sum().item()) == 0


@pytest.mark.parametrize("M,N", [(4096, 784), (256, 512), (10, 4096), (40, 36)])
def test_dw_gemm_fused_sgd_and_bias(M, N):
    """dW GEMM with fused SGD (LDS-vectorised path when aligned), bf16 W / W^T
    refresh and the bias step from the row sums of dZ^T."""
    C = require_native()
    K = 64
    g = torch.Generator().manual_seed(M + N)
    dZT = torch.randn(M, K, generator=g).to(torch.bfloat16)
    HT = torch.randn(N, K, generator=g).to(torch.bfloat16)
    W = torch.randn(M, N, generator=g)
    b = torch.randn(M, generator=g)
    lr = 0.01
    Wd, bd = W.to(DEV), b.to(DEV)
    Wb = torch.zeros(M, N, dtype=torch.bfloat16, device=DEV)
    WbT = torch.zeros(N, (M + 15) // 16 * 16, dtype=torch.bfloat16, device=DEV)  # padded like the engine
    C.gemm_bf16_nt_fused(dZT.to(DEV), HT.to(DEV), M, N, K, sgdW=Wd, lr=lr, obf=Wb, obfT=WbT, bsgd=bd)
    torch.cuda.synchronize()
    gW = dZT.float() @ HT.float().t()
    wantW = W - lr * gW
    assert (Wd.cpu() - wantW).abs().max().item() < 1e-5
    assert torch.equal(Wb.cpu(), Wd.cpu().to(torch.bfloat16))
    assert torch.equal(WbT.cpu()[:, :M].t(), Wb.cpu())
    wantb = b - lr * dZT.float().sum(1)
    assert (bd.cpu() - wantb).abs().max().item() < 1e-5
    gb = torch.zeros(M, device=DEV)
    G = torch.zeros(M, N, device=DEV)
    C.gemm_bf16_nt_fused(dZT.to(DEV), HT.to(DEV), M, N, K, of32=G, bgrad=gb)
    torch.cuda.synchronize()
    assert (G.cpu() - gW).abs().max().item() < 1e-3
    assert (gb.cpu() - dZT.float().sum(1)).abs().max().item() < 1e-4


@pytest.mark.parametrize("M,K", [(64, 784), (40, 520), (64, 1024)])
def test_gemm_rows64_kblocked_a_is_bit_exact(M, K):
    """rows64 reading A from a k-blocked [K/32][rows][32] copy: same products
    in the same order as the row-major A, so bit-identical outputs."""
    C = require_native()
    g = torch.Generator().manual_seed(M * K)
    rows = 3 * M
    A = torch.randn(rows, K, generator=g).to(torch.bfloat16).to(DEV)
    B = (torch.randn(4096, K, generator=g) / K ** 0.5).to(torch.bfloat16).to(DEV)
    bias = torch.randn(4096, generator=g).to(DEV)
    nb = (K + 31) // 32
    Ap = torch.zeros(rows, nb * 32, dtype=torch.bfloat16, device=DEV)
    Ap[:, :K] = A
    Ablk = Ap.view(rows, nb, 32).transpose(0, 1).contiguous()
    r0 = M  # a batch offset inside the shard
    o1 = torch.zeros(M, 4096, dtype=torch.bfloat16, device=DEV)
    o2 = torch.zeros_like(o1)
    C.gemm_bf16_nt_fused(A[r0:r0 + M], B, M, 4096, K, bias=bias, relu=True, obf=o1, splits=0)
    C.gemm_bf16_nt_fused(Ablk[:, r0:r0 + M], B, M, 4096, K, bias=bias, relu=True, obf=o2, splits=0)
    torch.cuda.synchronize()
    assert torch.equal(o1, o2)


def test_wide_kblocked_input_engine_is_bit_identical():
    spec = MlpSpec((784, 512, 256, 10))
    ds = synthetic_mnist(64 * 3, seed=19)
    a = WideMlpTrainer(spec, ds, batch=64, lr=0.05, seed=3, graph=True, xblk=False)
    b = WideMlpTrainer(spec, ds, batch=64, lr=0.05, seed=3, graph=True, xblk=True)
    assert b.Xblk is not None
    a.train_steps(7)
    b.train_steps(7)
    a.synchronize(); b.synchronize()
    assert torch.equal(a.P.cpu(), b.P.cpu())


@pytest.mark.parametrize("M,N", [(64, 4096), (50, 4096), (64, 2048)])
def test_head_combines_raw_skinny_slices_bit_identically(M, N):
    """VERDICT r5 Next #2: the last hidden layer's split-K GEMM leaves its raw
    slices (no ticket, no combine, no epilogue) and the head sums them in slice
    order as it loads H, applies bias + ReLU, rounds to bf16 and writes H back.
    Same bits as the GEMM's own combine + epilogue followed by the head."""
    C = require_native()
    g = torch.Generator().manual_seed(M + N)
    K = N
    A = torch.randn(M, K, generator=g).to(torch.bfloat16).to(DEV)
    B = (torch.randn(N, K, generator=g) / K ** 0.5).to(torch.bfloat16).to(DEV)
    bias = (0.1 * torch.randn(N, generator=g)).to(DEV)
    Wh = (0.05 * torch.randn(10, N, generator=g)).to(torch.bfloat16).to(DEV)
    bh = torch.randn(10, generator=g).to(DEV)
    y = torch.randint(0, 10, (M,), generator=g, dtype=torch.int32).to(DEV)
    S = C.gemm_skinny_splits(M, N, K, 0)
    assert S in (2, 4, 8)
    ws_words, ctr_words = C.gemm_skinny_ws(M, N, K, 0)
    ws = torch.zeros(max(ws_words, S * (N // 64) * 4096), device=DEV)
    ctr = torch.zeros(max(ctr_words, 1), dtype=torch.int32, device=DEV)
    outs = []
    for raw in (False, True):
        H = torch.zeros(64, N, dtype=torch.bfloat16, device=DEV)
        dz = torch.zeros(64, 16, dtype=torch.bfloat16, device=DEV)
        dzp = torch.zeros(64, N, dtype=torch.bfloat16, device=DEV)
        st = torch.zeros(64 * 4, device=DEV)
        lg = torch.zeros(64, 10, device=DEV)
        if raw:
            C.gemm_skinny(A, B, M, N, K, ws=ws, raw=True)
            C.head_softmax_xent(H, Wh, bh, M, N, 10, y, 1.0 / M, lg, dz, None, st, dzp=dzp, row_stats=True,
                                hs=ws, hs_splits=S, hs_bias=bias, hs_relu=True)
        else:
            C.gemm_skinny(A, B, M, N, K, bias=bias, relu=True, obf=H, ws=ws, ctr=ctr)
            C.head_softmax_xent(H, Wh, bh, M, N, 10, y, 1.0 / M, lg, dz, None, st, dzp=dzp, row_stats=True)
        torch.cuda.synchronize()
        outs.append((H[:M].cpu(), dz[:M].cpu(), dzp[:M].cpu(), st.cpu(), lg[:M].cpu()))
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    ref = torch.relu(A.float().cpu() @ B.float().cpu().t() + bias.cpu())
    assert (outs[1][0].float() - ref).abs().max().item() < 2e-2 * max(1.0, ref.abs().max().item())


@pytest.mark.parametrize("dims", [(784, 4096, 4096, 10), (784, 2048, 2048, 10)])
def test_wide_head_slab_engine_is_bit_identical(dims, monkeypatch):
    """The consumer-combined split-K form (the head sums the last hidden
    GEMM's slices) against the in-GEMM combine: the same parameters,
    statistics and evaluation, bit for bit."""
    spec = MlpSpec(dims)
    ds = synthetic_mnist(64 * 3, seed=23)
    runs = []
    for head in (0, 1):
        monkeypatch.setenv("HIPDSML_WIDE_HEAD_SLABS", str(head))
        t = WideMlpTrainer(spec, ds, batch=64, lr=0.05, seed=3, graph=True)
        assert (t._slab_plan(len(dims) - 3) in (4, 8)) == bool(head)
        t.train_steps(7)
        st = t.read_stats()
        runs.append((t.P.cpu(), st.loss_sum, st.correct, t.evaluate(ds)))
    for r in runs[1:]:
        assert torch.equal(r[0], runs[0][0])
        assert r[1:] == runs[0][1:]


@pytest.mark.gpu
@pytest.mark.parametrize("dims", [(784, 4096, 4096, 10), (784, 2048, 1024, 10), (784, 4096, 2048, 2048, 10)])
@pytest.mark.parametrize("graph", [False, True])
def test_wide_fused_input_layer_is_bit_identical(dims, graph, monkeypatch):
    """kernels/wide_input.hip (dZ_1 from the raw dgrad slices, the W_0 / b_0
    step and the NEXT step's H_1 in one launch) against the separate dgrad
    combine + update tiles + input-layer forward: the same parameters,
    statistics and evaluation, bit for bit -- across an epoch wrap (4 batches,
    9 steps), an evaluation in the middle (the carried H_1 is invalidated and
    recomputed) and, with graph=True, epoch-graph replays."""
    spec = MlpSpec(dims)
    ds = synthetic_mnist(64 * 4, seed=29)
    runs = []
    # separate kernels; the input-layer launch of its own; its strips inside
    # the update launch of the layers above (kernels/wgrad_sgd.hip wgrad_multi_in_k)
    for fused, beside in ((0, 0), (1, 0), (1, 1)):
        monkeypatch.setenv("HIPDSML_WIDE_FUSED_INPUT", str(fused))
        monkeypatch.setenv("HIPDSML_WIDE_INPUT_BESIDE", str(beside))
        t = WideMlpTrainer(spec, ds, batch=64, lr=0.05, seed=5, graph=graph)
        assert t.fused_input == bool(fused)
        t.train_steps(5)
        ev = t.evaluate(ds)
        t.train_steps(9)
        st = t.read_stats()
        runs.append((t.P.cpu(), st.loss_sum, st.correct, ev, t.evaluate(ds)))
    for r in runs[1:]:
        assert torch.equal(r[0], runs[0][0])
        assert r[1:] == runs[0][1:]

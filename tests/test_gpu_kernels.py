"""Numerics of the hand-written HIP kernels vs the plain PyTorch fp32 reference.

Every comparison runs the native path (hipdsml._C must be loaded — a missing
extension fails, it never falls back).
"""
import pytest
import torch

from hipdsml.data.mnist import synthetic_mnist
from hipdsml.engine.trainer import MlpTrainer
from hipdsml.models.mlp import MlpLayout, MlpSpec, forward_ref, grads_ref, init_params
from hipdsml.ops import functional as F
from hipdsml.ops.native import require_native
from hipdsml.parallel.dist import DistContext

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


def _ctx():
    return DistContext(device=DEV)


def _ref_steps(layout, P, X, y, batch, nsteps, lr):
    P = P.clone()
    nb = X.shape[0] // batch
    loss_tot = 0.0
    correct_tot = 0
    for s in range(nsteps):
        b = s % nb
        g, loss, corr = grads_ref(layout, P, X[b * batch:(b + 1) * batch], y[b * batch:(b + 1) * batch])
        P -= lr * g
        loss_tot += float(loss)
        correct_tot += int(corr)
    return P, loss_tot, correct_tot


def test_native_loaded():
    C = require_native()
    assert C.device_count() >= 1
    assert C.__file__.endswith("_C.so")


@pytest.mark.parametrize("dims,batch", [
    ((784, 128, 64, 10), 64),
    ((784, 128, 10), 64),
    ((784, 256, 128, 64, 10), 64),
    ((784, 128, 64, 10), 50),     # partial row tiles
    ((784, 128, 64, 10), 128),
    ((64, 32, 10), 32),
    ((784, 256, 128, 10), 64),   # specialised row chain <256,128,10>
    ((784, 128, 128, 10), 48),   # specialised row chain <128,128,10>, partial tile
    ((784, 96, 48, 10), 64),     # generic row chain, 3 layers
])
def test_fused_step_matches_reference(dims, batch):
    spec = MlpSpec(dims)
    ds = synthetic_mnist(batch * 3, seed=1, dim=dims[0])
    tr = MlpTrainer(spec, ds, batch=batch, lr=0.05, ctx=_ctx(), seed=3)
    layout = MlpLayout(spec, batch, 3)
    P0 = init_params(layout, 3)
    tr.train_steps(5)
    tr.synchronize()
    want, loss, corr = _ref_steps(layout, P0, ds.X, ds.y, batch, 5, 0.05)
    got = tr.P.cpu()
    err = (got - want).abs().max().item()
    assert err < 2e-5, err
    st = tr.read_stats()
    assert st.count == 5 * batch
    assert abs(st.loss_sum - loss) < 1e-3 * max(1.0, loss)
    assert st.correct == corr


def test_fwd_bwd_gradients_match_reference():
    C = require_native()
    spec = MlpSpec((784, 128, 64, 10))
    ds = synthetic_mnist(128, seed=2)
    layout = MlpLayout(spec, 64, 2)
    P0 = init_params(layout, 5)
    tr = MlpTrainer(spec, ds, batch=64, lr=0.0, ctx=_ctx(), seed=5)
    tr.runner.fwd_bwd()
    tr.synchronize()
    g, _, _ = grads_ref(layout, P0, ds.X[:64], ds.y[:64])
    got = tr.G.cpu()
    for l, ((gw, gb), (ww, wb)) in enumerate(zip(layout.views(got), layout.views(g))):
        assert torch.allclose(gw, ww, atol=2e-6, rtol=1e-4), (l, (gw - ww).abs().max())
        assert torch.allclose(gb, wb, atol=2e-6, rtol=1e-4), (l, (gb - wb).abs().max())
    assert C is not None


def test_graph_capture_matches_eager():
    spec = MlpSpec((784, 128, 64, 10))
    ds = synthetic_mnist(64 * 4, seed=4)
    a = MlpTrainer(spec, ds, batch=64, lr=0.01, ctx=_ctx(), seed=9)
    b = MlpTrainer(spec, ds, batch=64, lr=0.01, ctx=_ctx(), seed=9, graph_steps=3)
    a.train_steps(7)
    b.train_steps(7)
    a.synchronize(); b.synchronize()
    assert torch.equal(a.P.cpu(), b.P.cpu())
    assert int(b.ctr[0].item()) == 7


def test_momentum_path():
    spec = MlpSpec((784, 128, 64, 10))
    ds = synthetic_mnist(128, seed=6)
    tr = MlpTrainer(spec, ds, batch=64, lr=0.01, ctx=_ctx(), seed=1, momentum=0.9, weight_decay=1e-4)
    ref = MlpTrainer(spec, ds, batch=64, lr=0.01, ctx=DistContext(), seed=1, momentum=0.9,
                     weight_decay=1e-4)
    tr.train_steps(4)
    ref.train_steps(4)
    tr.synchronize()
    assert (tr.P.cpu() - ref.P).abs().max().item() < 2e-5


def test_eval_matches_reference():
    spec = MlpSpec((784, 128, 64, 10))
    ds = synthetic_mnist(1000, seed=7)
    tr = MlpTrainer(spec, ds, batch=64, lr=0.01, ctx=_ctx(), seed=2)
    ev = tr.evaluate(ds)
    logits, _ = forward_ref(tr.layout, tr.P.cpu(), ds.X)
    acc = 100.0 * (logits.argmax(1) == ds.y.long()).float().mean().item()
    assert abs(ev["accuracy"] - acc) < 1e-6
    assert ev["n"] == 1000


def test_training_converges_on_gpu():
    spec = MlpSpec((784, 128, 64, 10))
    ds = synthetic_mnist(64 * 50, seed=8)
    tr = MlpTrainer(spec, ds, batch=64, lr=0.05, ctx=_ctx(), seed=0, graph_steps=10)
    tr.train_steps(50)
    first = tr.read_stats()
    tr.train_steps(200)
    last = tr.read_stats()
    assert last.avg_loss < first.avg_loss
    assert last.accuracy > 90.0


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16, torch.uint8, torch.int32])
@pytest.mark.parametrize("op", ["sum", "prod", "min", "max"])
def test_reduce_kernels(dtype, op):
    n = 4099  # vector body + scalar tail
    g = torch.Generator().manual_seed(0)
    if dtype == torch.uint8:
        a = torch.randint(0, 256, (n,), generator=g, dtype=torch.uint8)
        b = torch.randint(0, 256, (n,), generator=g, dtype=torch.uint8)
    elif dtype == torch.int32:
        a = torch.randint(-1000, 1000, (n,), generator=g, dtype=torch.int32)
        b = torch.randint(-1000, 1000, (n,), generator=g, dtype=torch.int32)
    else:
        a = torch.randn(n, generator=g).to(dtype)
        b = torch.randn(n, generator=g).to(dtype)
    want = F.reduce_ref(a, b, op)
    da, db = a.to(DEV), b.to(DEV)
    out = torch.empty_like(da)
    F.reduce_into(out, da, db, op)
    torch.cuda.synchronize()
    if dtype in (torch.bfloat16, torch.float16):
        assert torch.allclose(out.cpu().float(), want.float(), rtol=1e-2, atol=1e-2)
    else:
        assert torch.equal(out.cpu(), want)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.uint8, torch.int32])
@pytest.mark.parametrize("op", ["sum", "max"])
def test_reduce_multi_matches_per_segment_reduce(dtype, op):
    """The ring step's merged reduce: up to 8 (dst, src) segments of mixed
    sizes and alignments in ONE launch == the single-segment kernel on each."""
    C = require_native()
    opc = {"sum": 0, "prod": 1, "min": 2, "max": 3}[op]
    g = torch.Generator().manual_seed(1)
    sizes, offs = (4099, 17, 65536, 1, 3000, 8, 257, 12345), (0, 1, 4, 3, 0, 2, 5, 7)
    base_d, base_s, dsts, srcs = [], [], [], []
    for n, o in zip(sizes, offs):
        if dtype in (torch.uint8, torch.int32):
            a = torch.randint(0, 100, (n + o,), generator=g).to(dtype)
            b = torch.randint(0, 100, (n + o,), generator=g).to(dtype)
        else:
            a, b = torch.randn(n + o, generator=g).to(dtype), torch.randn(n + o, generator=g).to(dtype)
        base_d.append(a.to(DEV))
        base_s.append(b.to(DEV))
        dsts.append(base_d[-1][o:])  # odd offsets: the element path
        srcs.append(base_s[-1][o:])
    want = [d.clone() for d in dsts]
    for w, s in zip(want, srcs):
        C.reduce_into(w, w, s, opc)
    C.reduce_multi_(dsts, srcs, opc)
    torch.cuda.synchronize()
    for d, w in zip(dsts, want):
        assert torch.equal(d, w)


def test_sgd_and_conversion_kernels():
    P = torch.randn(1003, device=DEV)
    G = torch.randn(1003, device=DEV)
    want = P.cpu() - 0.1 * G.cpu()
    F.sgd_update_(P, G, 0.1)
    torch.cuda.synchronize()
    assert torch.allclose(P.cpu(), want, atol=1e-6)
    u = torch.randint(0, 256, (5000,), dtype=torch.uint8)
    f = F.u8_to_f32(u.to(DEV))
    assert torch.allclose(f.cpu(), u.float() / 255.0)
    C = require_native()
    x = torch.randn(777, device=DEV)
    bf = torch.empty(777, dtype=torch.bfloat16, device=DEV)
    C.f32_to_bf16(bf, x)
    assert torch.equal(bf.cpu(), x.cpu().to(torch.bfloat16))
    back = torch.empty(777, device=DEV)
    C.bf16_to_f32(back, bf)
    assert torch.equal(back.cpu(), bf.cpu().float())


def test_rccl_single_rank_comm():
    C = require_native()
    uid = C.rccl_unique_id()
    assert len(uid) == 128
    comm = C.RcclComm(uid, 0, 1, 0, True)
    t = torch.arange(1024, dtype=torch.float32, device=DEV)
    comm.allreduce_(t, 0)
    comm.ring_allreduce_(t, 0, 4096)
    hb = torch.arange(512, device=DEV).to(torch.bfloat16)
    comm.allgather_(hb)  # in-place all-gather (the wide engine's activation exchange)
    torch.cuda.synchronize()
    assert torch.equal(t.cpu(), torch.arange(1024, dtype=torch.float32))
    assert torch.equal(hb.cpu(), torch.arange(512).to(torch.bfloat16))
    with pytest.raises(Exception, match="nranks equal parts|contiguous"):
        comm.allgather_(hb[::2])
    assert comm.async_error() == ""
    comm.abort()
    assert comm.aborted


@pytest.mark.parametrize("blocking", [True, False])
def test_rccl_collectives_captured_in_graph(blocking):
    """RCCL calls recorded into a hipGraph (how multi-GPU steps are replayed)
    give the same bytes as the eager calls; non-blocking comms too."""
    C = require_native()
    comm = C.RcclComm(C.rccl_unique_id(), 0, 1, 0, blocking)
    x = torch.randn(4096, device=DEV)
    eager = x.clone()
    comm.allreduce_(eager, 0)
    torch.cuda.synchronize()
    buf = x.clone()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream(DEV)
    s.wait_stream(torch.cuda.current_stream())
    hb = x[:1024].to(torch.bfloat16)
    comm.allgather_(hb)  # eager first: RCCL connects outside the capture
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=s):
        comm.allreduce_(buf, 0)
        buf.mul_(2.0)
        comm.allreduce_(buf, 0)
        comm.allgather_(hb)
    for _ in range(3):
        buf.copy_(x)
        g.replay()
    torch.cuda.synchronize()
    assert torch.equal(buf, 2.0 * eager)
    assert torch.equal(hb, x[:1024].to(torch.bfloat16))
    assert comm.async_error() == ""


def test_rccl_abort_with_collective_enqueued():
    """ncclCommAbort while a collective is still queued behind other work:
    nothing hangs, the comm reports aborted and refuses further calls."""
    C = require_native()
    comm = C.RcclComm(C.rccl_unique_id(), 0, 1, 0, False)
    t = torch.ones(1 << 20, device=DEV)
    torch.cuda._sleep(20_000_000)  # GPU busy ahead of the collective
    comm.allreduce_(t, 0)
    comm.abort()
    torch.cuda.synchronize()
    assert comm.aborted and comm.async_error() == "aborted"
    with pytest.raises(RuntimeError, match="aborted"):
        comm.allreduce_(t, 0)


def test_trainer_graph_sizes_cover_any_step_count():
    """train_steps(n) replays a G-step and an r-step graph for n = q*G + r
    (no eager fallback), bit-identical to eager launches."""
    spec = MlpSpec((784, 128, 64, 10))
    ds = synthetic_mnist(64 * 8, seed=4)
    a = MlpTrainer(spec, ds, batch=64, lr=0.01, ctx=_ctx(), seed=9, persist=False)
    b = MlpTrainer(spec, ds, batch=64, lr=0.01, ctx=_ctx(), seed=9, graph_steps=5, persist=False)
    for n in (3, 12, 7):
        a.train_steps(n)
        b.train_steps(n)
    a.synchronize()
    b.synchronize()
    assert b.runner.captured(5) and b.runner.captured(3) and b.runner.captured(2)
    assert torch.equal(a.P, b.P)


def test_device_runtime_roundtrip():
    C = require_native()
    arena = C.DeviceArena(0, 1 << 20)
    assert arena.min_addr == 0x1000 and arena.max_addr == 0x1000 + (1 << 20)
    ce = C.CopyEngine(0, 1 << 16)  # small staging: forces multi-chunk pipelining
    payload = bytes(range(256)) * 1000
    ce.h2d(arena, 0x2000, payload)
    assert ce.d2h(arena, 0x2000, len(payload)) == payload
    with pytest.raises(IndexError):
        ce.h2d(arena, 0x1000 + (1 << 20) - 4, b"12345678")
    st = C.StreamTable(arena, ce)
    sid = st.begin_send(0x2000, 10, 1)
    assert sid >= 1
    st.begin_receive(sid, 0x8000, 10, 0)
    assert st.push_chunk(sid, b"chunk")
    assert st.push_chunk(sid, b"chunk")
    assert st.finish(sid)
    assert st.status(sid) == 1
    assert ce.d2h(arena, 0x8000, 10) == b"chunkchunk"
    assert st.status(999) == 2
    # on-device reduction between arena addresses (f32 sum)
    a = torch.arange(64, dtype=torch.float32).numpy().tobytes()
    ce.h2d(arena, 0x10000, a)
    ce.h2d(arena, 0x20000, a)
    arena.reduce(0x10000, 0x20000, len(a), 0, 0)
    out = torch.frombuffer(bytearray(ce.d2h(arena, 0x10000, len(a))), dtype=torch.float32)
    assert torch.equal(out, 2 * torch.arange(64, dtype=torch.float32))

"""Persistent fused step (kernels/mlp_persist.hip): S SGD steps per launch,
weights resident on chip, flag / tagged-granule hand-offs between 56
layer-1 blocks, 4 row chains and 4 upper-layer gradient blocks.  Covers the
BASELINE model 784-128-64-10 and the reference client's own 784-128-10
(client.go:22-33), at batch 64 and below.  Checked against the fp32 torch
reference (models/mlp.py grads_ref) and the three-launch path."""
import pytest
import torch

from hipdsml.data.mnist import synthetic_mnist
from hipdsml.engine.trainer import MlpTrainer
from hipdsml.models.mlp import MlpLayout, MlpSpec, grads_ref, init_params
from hipdsml.parallel.dist import DistContext

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
SPEC = MlpSpec((784, 128, 64, 10))
REF_SPEC = MlpSpec((784, 128, 10))  # the model client.go codes


def _tr(ds, persist, lr=0.05, seed=3, spec=SPEC, batch=64):
    return MlpTrainer(spec, ds, batch=batch, lr=lr, ctx=DistContext(device=DEV), seed=seed,
                      persist=persist)


def _ref(ds, steps, lr=0.05, seed=3, spec=SPEC, batch=64):
    nb = len(ds) // batch
    lay = MlpLayout(spec, batch, nb)
    P = init_params(lay, seed, "reference")
    loss = 0.0
    for s in range(steps):
        b = s % nb
        g, ls, _ = grads_ref(lay, P, ds.X[b * batch:(b + 1) * batch], ds.y[b * batch:(b + 1) * batch])
        loss += float(ls)
        P = P - lr * g
    return P, loss


@pytest.mark.parametrize("spec", [SPEC, REF_SPEC], ids=str)
def test_persistent_step_is_active_for_both_models(spec):
    t = _tr(synthetic_mnist(64 * 4, seed=1), None, spec=spec)
    assert t.persistent and t.runner.persist_active()
    assert not _tr(synthetic_mnist(64 * 4, seed=1), False, spec=spec).persistent
    # outside the family: the three-launch path
    assert not _tr(synthetic_mnist(64 * 4, seed=1), None, spec=MlpSpec((784, 96, 10))).persistent


@pytest.mark.parametrize("spec,batch,steps", [(SPEC, 64, 1), (SPEC, 64, 2), (SPEC, 64, 9),
                                              (REF_SPEC, 64, 1), (REF_SPEC, 64, 9),
                                              (SPEC, 32, 7), (REF_SPEC, 48, 7), (SPEC, 1, 3)],
                         ids=lambda v: str(v))
def test_persistent_matches_fp32_reference(spec, batch, steps):
    ds = synthetic_mnist(batch * 4, seed=11)
    t = _tr(ds, True, spec=spec, batch=batch)
    assert t.persistent
    t.train_steps(steps)
    t.synchronize()
    want, loss = _ref(ds, steps, spec=spec, batch=batch)
    err = (t.P.cpu() - want).abs().max().item()
    assert err < 2e-5, err
    st = t.read_stats()
    assert st.count == batch * steps
    assert abs(st.loss_sum - loss) < 1e-3 * max(1.0, loss)
    assert int(t.ctr[0].item()) == steps and int(t.ctr[1].item()) == steps


@pytest.mark.parametrize("spec", [SPEC, REF_SPEC], ids=str)
def test_persistent_launch_split_is_bit_exact_and_matches_three_launch_path(spec):
    ds = synthetic_mnist(64 * 5, seed=12)
    a, b, c = _tr(ds, True, spec=spec), _tr(ds, True, spec=spec), _tr(ds, False, spec=spec)
    a.train_steps(23)
    for n in (7, 1, 15):  # epoch wrap-around inside and across launches
        b.train_steps(n)
    c.train_steps(23)
    for t in (a, b, c):
        t.synchronize()
    assert torch.equal(a.P, b.P)
    assert (a.P - c.P).abs().max().item() < 5e-5


def test_persistent_resume_rewinds_tags(tmp_path):
    ds = synthetic_mnist(64 * 4, seed=13)
    a = _tr(ds, True)
    a.train_steps(6)
    sd = a.state_dict()
    a.train_steps(5)
    a.synchronize()
    b = _tr(ds, True)
    b.train_steps(9)  # ahead of the checkpoint: its buffers hold later tags
    b.load_state_dict(sd)
    b.train_steps(5)
    b.synchronize()
    assert torch.equal(a.P, b.P)


def test_persistent_resume_into_other_batching_drops_the_carry():
    """A checkpoint's carried pipeline state (next step's Z1 partials) belongs to
    its batch size and data: resuming into a trainer with another batch size
    must recompute the first step instead of feeding the stale Z1."""
    ds = synthetic_mnist(64 * 4, seed=17)
    a = _tr(ds, True, batch=64)
    a.train_steps(5)
    sd = a.state_dict()
    assert "persist_carry" in sd and sd["persist_meta"]["batch"] == 64
    b = _tr(ds, True, batch=32)
    sd = dict(sd, steps_done=0)  # same params, step 0 of the 32-row batching
    b.load_state_dict(sd)
    assert not b.runner.persist_carry()
    b.train_steps(3)
    b.synchronize()
    # reference: plain SGD on 32-row batches from the checkpoint's params
    lay = MlpLayout(SPEC, 32, len(ds) // 32)
    P = sd["params"].clone()
    for s in range(3):
        g, _, _ = grads_ref(lay, P, ds.X[s * 32:(s + 1) * 32], ds.y[s * 32:(s + 1) * 32])
        P = P - 0.05 * g
    assert (b.P.cpu() - P).abs().max().item() < 2e-5


def test_persistent_long_run_converges():
    ds = synthetic_mnist(64 * 50, seed=14)
    t = _tr(ds, True, lr=0.05)
    t.train_steps(50)
    first = t.read_stats()
    t.train_steps(500)
    last = t.read_stats()
    assert last.avg_loss < first.avg_loss
    assert torch.isfinite(t.P).all()


def test_persistent_handoff_timeout_is_reported_and_recoverable():
    """A hand-off wait past its bound ends the launch on every block (err word)
    and the host sees it through the host-mapped mirror, without a copy."""
    ds = synthetic_mnist(64 * 4, seed=15)
    t = _tr(ds, True)
    t.runner.set_persist(t.pk_buf, t.pk_err, 1e-4)  # 10 ticks: the first wait gives up
    t.train_steps(5)
    with pytest.raises(RuntimeError, match="hand-off timed out"):
        t.synchronize()
    assert t.runner.persist_failed() and int(t.pk_err.item()) != 0
    # rearm with a sane bound: the job can restart from a checkpoint
    t.runner.set_persist(t.pk_buf, t.pk_err, 2000.0)
    t._rewound()
    t.ctr.zero_()
    torch.cuda.synchronize()  # the runner's stream does not wait on torch's
    t.train_steps(3)
    t.synchronize()
    assert not t.runner.persist_failed()


@pytest.mark.parametrize("spec", [SPEC, REF_SPEC], ids=str)
def test_persistent_uneven_load_is_bit_exact(spec):
    """Uneven load: with jitter injection every block sleeps a pseudo-random
    0-8 us before its hand-off waits and publications, so producers and
    consumers (and the chains among themselves) drift apart; the parity /
    tag protocol must still give the same bits, across a launch split too."""
    from hipdsml.ops.native import require_native

    C = require_native()
    ds = synthetic_mnist(64 * 5, seed=16)
    a, b = _tr(ds, True, spec=spec), _tr(ds, True, spec=spec)
    a.train_steps(23)
    a.synchronize()
    C.mlp_persist_set_jitter(300)
    try:
        for n in (9, 14):
            b.train_steps(n)
        b.synchronize()
    finally:
        C.mlp_persist_set_jitter(0)
    assert torch.equal(a.P, b.P)


@pytest.mark.parametrize("algo,n,helpers,l1push", [(4, 2, -1, -1), (4, 3, -1, -1), (4, 4, -1, -1), (4, 8, -1, -1),
                                                   (4, 8, 1, -1), (4, 6, -1, -1), (4, 2, 1, -1), (4, 4, 0, -1),
                                                   (4, 8, -1, 1), (4, 8, -1, 0), (4, 3, -1, 1), (2, 4, -1, -1),
                                                   (2, 8, -1, -1), (0, 4, -1, -1)],
                         ids=lambda v: str(v))
def test_data_parallel_forms_mirrored_replicas(algo, n, helpers, l1push):
    """One GPU runs the n-replica persistent step (pk = 0, pkg = 2, pkx = 4)
    against n - 1 exact copies of itself: in the kernel's mirror test mode every
    push to peer d lands in this replica's OWN receive buffer, in d's source
    slot, with its tags and flags.  Every replica then holds the same shard, so
    the global-batch gradient is n x its own at lr / n: the parameters must
    match single-replica SGD.  This is the only way one GPU runs pkx at n >= 4,
    where the dW1 sum is split with the helper blocks (the Gram grid of more
    than 2 real replicas cannot share one GPU)."""
    from hipdsml.ops.native import require_native
    from hipdsml.parallel.xchg import make_local_group, swizzle_inputs

    C = require_native()
    ds = synthetic_mnist(64 * 4, seed=21)
    t = _tr(ds, True)
    half, ntiles = C.MlpRunner.persist_xchg_size(n, algo)
    xs = make_local_group(None, [0] * n, 5000.0, half_floats=half, ntiles=ntiles)
    t.runner.set_world_size(n)
    nb = t.nbatches
    Xs = t.X[: nb * 64, :784].reshape(1, nb, 64, 784).expand(n, nb, 64, 784).contiguous()
    if algo >= 2:
        t.runner.set_persist_gram(C.gram_table(Xs.reshape(n, nb * 64, 784), t.X, nb, 64, 784))
    if algo == 4:
        xall = swizzle_inputs(Xs.reshape(n, nb * 64, 784), 64)
        t.runner.set_persist_xall(xall, xall[0].numel())
    C.mlp_persist_set_probe(2)
    C.mlp_persist_set_pkx_helpers(helpers)  # pkx: the dW1 split over 0 / 1 / 3 helper blocks
    C.mlp_persist_set_pkx_l1push(l1push)
    try:
        t.runner.set_persist(t.pk_buf, t.pk_err, 5000.0, xs[0], algo)
        for k in (5, 1, 9):  # launch splits: carried state, parity and slot reuse
            t.train_steps(k)
        t.synchronize()
    finally:
        C.mlp_persist_set_probe(0)
        C.mlp_persist_set_pkx_helpers(-1)
        C.mlp_persist_set_pkx_l1push(-1)
    want, _ = _ref(ds, 15)
    err = (t.P.cpu() - want).abs().max().item()
    assert err < 2e-5, err


def _replay_group(algo, n, shards):
    """n persistent-step instances on one GPU, instance r holding shard r, wired
    into one local exchange group as ranks 0..n-1 (data-parallel persistent
    step `algo`), with the all-gathered inputs / cross-replica Gram tables the
    real job builds from the distinct shards."""
    from hipdsml.ops.native import require_native
    from hipdsml.parallel.xchg import make_local_group, swizzle_inputs

    C = require_native()
    trs = [MlpTrainer(SPEC, ds, batch=64, lr=0.05, ctx=DistContext(device=DEV), seed=3, persist=True,
                      persist_place_trials=1) for ds in shards]
    nb = trs[0].nbatches
    plain = torch.stack([t.X[: nb * 64, :784] for t in trs]).contiguous()  # [n][rows][784], rank order
    half, ntiles = C.MlpRunner.persist_xchg_size(n, algo)
    xs = make_local_group(None, [0] * n, 5000.0, half_floats=half, ntiles=ntiles)
    xall = swizzle_inputs(plain, 64) if algo == 4 else None
    for r, t in enumerate(trs):
        t.runner.set_world_size(n)
        if algo >= 2:
            t.runner.set_persist_gram(C.gram_table(plain, t.X, nb, 64, 784))
        if xall is not None:
            t.runner.set_persist_xall(xall, xall[0].numel())
        t.runner.set_persist(t.pk_buf, t.pk_err, 5000.0, xs[r], algo)
    return C, trs, xs


def _replay_steps(C, trs, xs, r, algo, steps):
    """Replay: replica r runs the n-rank persistent step one launch per step
    (its pipeline state carried from launch to launch), and before each of its
    launches every peer r' != r runs that step once as a CAPTURE: a fresh
    (uncarried) one-step launch of the same kernel on r's current weights and
    step counter -- the weights every replica holds at that step, since
    replicas stay identical -- with its own shard.  The capture's pushes land
    in r's receive buffer exactly as a real peer's would (its dZ1 rows, its
    gradient-tile / layer-1 slots, tags and flags), computed from distinct data
    by the real kernel; its own sums run in the probe test mode (peers taken
    as arrived: its state is thrown away).  Then r's launch finds every peer's
    data of the step in place and must produce n-replica SGD."""
    t = trs[r]
    for _ in range(steps):
        torch.cuda.synchronize()
        C.mlp_persist_set_probe(1)
        try:
            for rp, tp in enumerate(trs):
                if rp == r:
                    continue
                tp.P.copy_(t.P)
                tp.ctr.copy_(t.ctr)
                tp.runner.set_persist_carry(False)
                xs[rp].fill_flags(1 << 62)  # its own flags preset (the probe's rule): it never waits
                tp.train_steps(1)
                tp.synchronize()
        finally:
            C.mlp_persist_set_probe(0)
        torch.cuda.synchronize()
        t.train_steps(1)
        t.synchronize()


@pytest.mark.parametrize("algo,n,r,l1push", [(4, 4, 0, -1), (4, 4, 1, -1), (4, 4, 3, -1), (4, 8, 0, -1),
                                             (4, 8, 1, -1), (4, 8, 7, -1), (4, 8, 3, 1), (4, 4, 2, 1), (4, 2, 1, 1),
                                             (4, 8, 5, 0), (2, 4, 1, -1), (2, 8, 7, -1), (0, 4, 2, -1)],
                         ids=lambda v: str(v))
def test_pkx_replay_distinct_peers(algo, n, r, l1push):
    """VERDICT r5 Next #1: the N >= 4 data-parallel persistent code (pkx's
    helper split and pusher blocks switch on from 4 replicas) on DISTINCT
    replica data, which mirror mode (every peer an exact copy) cannot check: a
    rank-offset or slot-permutation bug there passes mirror mode but not this.
    Replica r's parameters after 7 steps (3-slot dZ1 rotation, both parities,
    an epoch wrap) must match fp32 torch SGD on the global batch of n shards."""
    shards = [synthetic_mnist(64 * 4, seed=300 + k) for k in range(n)]
    C, trs, xs = _replay_group(algo, n, shards)
    steps = 7
    C.mlp_persist_set_pkx_l1push(l1push)  # pkx: dZ1 rows pushed by the chains (0) / layer-1 owners (1)
    try:
        _replay_steps(C, trs, xs, r, algo, steps)
    finally:
        C.mlp_persist_set_pkx_l1push(-1)
    lay = MlpLayout(SPEC, 64, 4)
    P = init_params(lay, 3, "reference")
    for s in range(steps):
        b = s % 4
        g = sum(grads_ref(lay, P, ds.X[b * 64:(b + 1) * 64], ds.y[b * 64:(b + 1) * 64])[0] for ds in shards)
        P = P - 0.05 * g / n
    err = (trs[r].P.cpu() - P).abs().max().item()
    assert err < 2e-5, err
    # and the replay is not vacuous: the shards differ, so single-shard SGD is far off
    P1 = init_params(lay, 3, "reference")
    for s in range(steps):
        b = s % 4
        P1 = P1 - 0.05 * grads_ref(lay, P1, shards[r].X[b * 64:(b + 1) * 64], shards[r].y[b * 64:(b + 1) * 64])[0]
    assert (trs[r].P.cpu() - P1).abs().max().item() > 100 * err

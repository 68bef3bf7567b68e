"""xGMI peer exchange (gradient all-reduce fused into the weight-gradient
kernel) on ONE MI355X: N replicas share the GPU, either inside one process
(pointers exchanged directly) or as separate processes (IPC handles) — the
same kernel and flag protocol that runs across GPUs of a node."""
import os
import tempfile

import pytest
import torch
import torch.multiprocessing as mp

from hipdsml.data.mnist import synthetic_mnist
from hipdsml.engine.trainer import MlpTrainer
from hipdsml.models.mlp import MlpLayout, MlpSpec, grads_ref, init_params
from hipdsml.parallel.dist import DistContext
from hipdsml.parallel.xchg import (make_local_act_group, make_local_group, replica_streams,
                                   swizzle_inputs)
from spawn_util import spawn_group

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
DIMS = (784, 128, 64, 10)


def _fresh(fn, *args):
    """Run `fn(*args)` in a freshly spawned process.

    Round 1 saw in-process replica groups read stale data intermittently in
    the long pytest process (never in a fresh one) and moved them here.  The
    suspected cause -- memory the caching allocator recycled from work on
    another queue, read by a replica queue without a stream-ordered hand-off
    -- is now excluded by construction: every replica input is produced before
    the PeerExchange constructor's device synchronize, every exchange payload
    and flag lives in uncached memory written and read at system scope
    (kernels/common.h), and test_local_group_in_the_long_process runs one
    3-replica group in the long process (green in the round-3 full suite,
    profiles/r3_gpu_suite.txt).  The other cases stay isolated so a fault in
    one cannot poison the rest of the suite.  Exceptions in the child fail the
    test with the child's traceback."""
    mp.start_processes(_fresh_entry, args=(fn, args), nprocs=1, start_method="spawn", join=True)


def _fresh_entry(_rank, fn, args):
    # replica streams are BLOCKING (CU-mask streams take no flags): runners join
    # torch's current stream, which must therefore not be the legacy null stream
    # (an event recorded there waits for every blocking stream, spinning peers too)
    with torch.cuda.stream(torch.cuda.Stream(DEV)):
        fn(*args)


def _reference(world, steps, lr, nb, seed=7):
    lay = MlpLayout(MlpSpec(DIMS), 64, nb)
    P = init_params(lay, seed, "reference")
    shards = [synthetic_mnist(64 * nb, seed=300 + r) for r in range(world)]
    for s in range(steps):
        b = s % nb
        g = None
        for sh in shards:
            gi = grads_ref(lay, P, sh.X[b * 64:(b + 1) * 64], sh.y[b * 64:(b + 1) * 64])[0]
            g = gi if g is None else g + gi
        P = P - lr * g / world
    return P


def _local_group(world, nb, graph_steps, timeout_ms=5000.0):
    # replicas spin on each other: their streams must sit on distinct HW queues
    ss = replica_streams(DEV, world)
    trs = [MlpTrainer(MlpSpec(DIMS), synthetic_mnist(64 * nb, seed=300 + r), batch=64, lr=0.05,
                      seed=7, ctx=DistContext(device=DEV), graph_steps=graph_steps, stream=ss[r])
           for r in range(world)]
    xs = make_local_group(trs[0].layout, [0] * world, timeout_ms)
    for t, x in zip(trs, xs):
        t.runner.set_exchange(x)
        t.xchg = x
    return trs, xs


def _case_local_group(world, graph_steps):
    nb, steps = 4, 10
    trs, xs = _local_group(world, nb, graph_steps)
    for chunk in (5, 5):
        for t in trs:
            t.train_steps(chunk)
        for t in trs:
            t.synchronize()  # raises if a peer timed out
    Ps = [t.P.cpu() for t in trs]
    for P in Ps[1:]:
        assert torch.equal(P, Ps[0])  # replicas bit-identical (rank-order sums)
    want = _reference(world, steps, 0.05, nb)
    err = (Ps[0] - want).abs().max().item()
    assert err < 2e-5, err
    assert xs[0].memory_kind in ("uncached", "finegrained", "coarse")


@pytest.mark.parametrize("world,graph_steps", [(2, 0), (3, 0), (2, 5)])
def test_local_group_matches_reference(world, graph_steps):
    _fresh(_case_local_group, world, graph_steps)


def test_local_group_in_the_long_process():
    """The same 3-replica group run IN this long-lived pytest process (after
    the tests above have churned the caching allocator), inside a non-null
    torch stream as _fresh_entry sets up: the replicas' inputs are produced
    on torch's stream and consumed on the replica queues only behind the
    PeerExchange constructor's device synchronize, and every runner call
    joins back into torch's stream before the parameters are read."""
    with torch.cuda.stream(torch.cuda.Stream(DEV)):
        _case_local_group(3, 0)


def _case_missing_peer():
    trs, xs = _local_group(2, 2, 0, timeout_ms=200.0)
    trs[0].train_steps(1)  # rank 1 never runs
    with pytest.raises(RuntimeError, match="timed out"):
        trs[0].synchronize()
    xs[0].reset()
    torch.cuda.synchronize()
    assert xs[0].error() == 0


def test_missing_peer_times_out_instead_of_hanging():
    _fresh(_case_missing_peer)


def _local_act_group(world, nb, graph_steps, timeout_ms=5000.0, waves=0):
    """Activation exchange between `world` replicas of one process."""
    ss = replica_streams(DEV, world)
    trs = [MlpTrainer(MlpSpec(DIMS), synthetic_mnist(64 * nb, seed=300 + r), batch=64, lr=0.05,
                      seed=7, ctx=DistContext(device=DEV), graph_steps=graph_steps, stream=ss[r])
           for r in range(world)]
    rows = nb * 64
    Xall = swizzle_inputs(torch.stack([t.X[:rows] for t in trs]), 64)
    xs = make_local_act_group(trs[0].layout, [0] * world, timeout_ms)
    for t, x in zip(trs, xs):
        t.runner.set_act_exchange(x, Xall, Xall[0].numel(), waves)
        t.xchg = x
        assert t.runner.exchange_mode() == 2
    return trs, xs


# in-process groups stay at <= 3 replicas: with 4 HIP hardware queues per
# process, a 4th replica stream could queue behind a spinning peer
# 8-wave tile blocks (the form used from 4 ranks on): two replicas are the most
# whose spinning launches (2 x 243 blocks of 512 threads) fit one GPU together
def _case_local_act_group(world, graph_steps, waves):
    nb, steps = 4, 10
    trs, xs = _local_act_group(world, nb, graph_steps, waves=waves)
    for chunk in (5, 5):
        for t in trs:
            t.train_steps(chunk)
        for t in trs:
            t.synchronize()  # raises if a peer timed out
    Ps = [t.P.cpu() for t in trs]
    for P in Ps[1:]:
        assert torch.equal(P, Ps[0])  # every replica computes the same global-batch sums
    want = _reference(world, steps, 0.05, nb)
    err = (Ps[0] - want).abs().max().item()
    assert err < 2e-5, err


@pytest.mark.parametrize("world,graph_steps,waves", [(2, 0, 0), (3, 0, 0), (3, 5, 0), (2, 5, 0),
                                                    (2, 0, 8), (2, 5, 8)])
def test_local_act_group_matches_reference(world, graph_steps, waves):
    _fresh(_case_local_act_group, world, graph_steps, waves)


def _case_act_missing_peer():
    trs, xs = _local_act_group(2, 2, 0, timeout_ms=200.0)
    P0 = trs[0].P.clone()
    trs[0].train_steps(1)  # rank 1 never pushes
    with pytest.raises(RuntimeError, match="timed out"):
        trs[0].synchronize()
    # a timed-out tile leaves its weights alone
    assert torch.equal(trs[0].P, P0)
    xs[0].reset()
    torch.cuda.synchronize()
    assert xs[0].error() == 0


def test_act_exchange_missing_peer_times_out():
    _fresh(_case_act_missing_peer)



def _ipc_worker(rank, world, port, outdir, graph_steps, sync="xgmi", xact_waves=0):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK="0",
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    ctx = DistContext.from_env(device="cuda", backend="gloo")
    tr = MlpTrainer(MlpSpec(DIMS), synthetic_mnist(64 * 4, seed=300 + rank), batch=64, lr=0.05,
                    ctx=ctx, seed=7, sync=sync, graph_steps=graph_steps, xchg_timeout_ms=5000.0,
                    xact_waves=xact_waves, auto_fallback="torch")
    if sync == "auto":  # every candidate self-tested and timed; any may win on a shared GPU
        # (3 replicas on one GPU: the Gram form reports itself unavailable)
        cands = ({"pkx", "pkg", "pk", "xact", "xgmi", "torch"} if world == 2
                 else {"pk", "pk2", "xact", "xgmi", "torch"})
        assert tr.sync_active in cands, tr.sync_active
        assert set(tr.sync_times) == cands, tr.sync_times
    else:
        assert tr.sync_active == sync
    if sync in ("pk", "pk2", "pkg", "pkg2", "pkx"):  # launches split anywhere: counter and tags carry over
        assert tr.persistent
        tr.train_steps(2)
        tr.train_steps(4)
    else:
        tr.train_steps(6)
    tr.synchronize()
    torch.save({"P": tr.P.cpu()}, os.path.join(outdir, f"r{rank}.pt"))
    ctx.destroy()


@pytest.mark.parametrize("world,graph_steps,sync", [(2, 0, "xgmi"), (2, 3, "xgmi"), (2, 0, "xact"),
                                                    (2, 3, "xact"), (3, 3, "xact"), (3, 3, "xgmi"),
                                                    (2, 0, "pk"), (3, 0, "pk"), (2, 0, "pk2"),
                                                    (3, 0, "pk2"), (2, 0, "pkg"), (2, 0, "pkg2"),
                                                    (2, 0, "pkx"), (2, 3, "auto"), (3, 3, "auto")])
def test_two_processes_ipc(world, graph_steps, sync):
    """N processes sharing the GPU through IPC handles.  Sharing one GPU, every
    process's spinning weight-gradient launch must be resident at once: the
    activation exchange runs 4-wave tile blocks (3 x 243 of 1,024 block slots;
    the 8-wave form is covered in-process above), and groups stay at <= 3
    processes — with 4 or more, the hardware scheduler can leave a process's
    queue unmapped while its peers spin (seen as a timed-out self-test).  On a
    node each GPU runs one process and one launch.  sync='pk' runs the
    persistent step in every process (64 workgroups each, all resident) with
    the weight gradients summed over the replicas inside the launch; 'pk2'
    sums them two-shot (reduce-scatter + all-gather per wave slot).  'pkg' /
    'pkg2' run the persistent step in Gram form across the replicas: every
    chain's dZ1 rows pushed to every peer for the layer-1 correction (cross-
    replica Gram blocks), the gradient slots summed one- / two-shot.  'pkx'
    is the Gram form with an exchange-free layer 1: every replica forms the
    global-batch dW1 from the peers' dZ1 rows and the all-gathered shards."""
    with tempfile.TemporaryDirectory() as d:
        spawn_group(_ipc_worker, world, lambda port: (world, port, d, graph_steps, sync,
                                              4 if sync in ("xact", "auto") else 0))
        Ps = [torch.load(os.path.join(d, f"r{r}.pt"), weights_only=True)["P"] for r in range(world)]
    for P in Ps[1:]:
        assert torch.equal(Ps[0], P)
    err = (Ps[0] - _reference(world, 6, 0.05, 4)).abs().max().item()
    assert err < 2e-5, err


def _long_worker(rank, world, port, outdir, sync, launches):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK="0",
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    ctx = DistContext.from_env(device="cuda", backend="gloo")
    tr = MlpTrainer(MlpSpec(DIMS), synthetic_mnist(64 * 4, seed=300 + rank), batch=64, lr=0.05,
                    ctx=ctx, seed=7, sync=sync, xchg_timeout_ms=5000.0, auto_fallback="torch")
    assert tr.sync_active == sync and tr.persistent
    for n in launches:
        tr.train_steps(n)
    tr.synchronize()
    torch.save({"P": tr.P.cpu()}, os.path.join(outdir, f"r{rank}.pt"))
    ctx.destroy()


@pytest.mark.parametrize("sync", ["pkx", "pkg"])
def test_gram_forms_many_steps_ipc(sync):
    """37 steps in three launches (13, 1, 23): every parity half and every one
    of pkx's three rotating dZ1 slots is reused many times over, across launch
    splits and epoch wrap-arounds (4 batches), so a slot region that overlaps
    another or a tag that can match stale rows would show here."""
    launches = (13, 1, 23)
    with tempfile.TemporaryDirectory() as d:
        spawn_group(_long_worker, 2, lambda port: (2, port, d, sync, launches))
        Ps = [torch.load(os.path.join(d, f"r{r}.pt"), weights_only=True)["P"] for r in range(2)]
    assert torch.equal(Ps[0], Ps[1])
    err = (Ps[0] - _reference(2, sum(launches), 0.05, 4)).abs().max().item()
    assert err < 1e-4, err


def _ar_worker(rank, world, port, outdir, algo="oneshot"):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK="0",
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from hipdsml.parallel.xchg import XgmiAllReduce

    ctx = DistContext.from_env(device="cuda", backend="gloo")
    ar = XgmiAllReduce(ctx, 1 << 18, algo=algo)
    res = []
    for it in range(4):
        t = torch.full((1 << 18,), float(rank + 1 + it), device=ctx.device)
        ar(t)
        res.append(t[:8].cpu())
    torch.cuda.synchronize()
    ar.check()
    torch.save({"res": torch.stack(res)}, os.path.join(outdir, f"r{rank}.pt"))
    ctx.destroy()


@pytest.mark.parametrize("algo", ["oneshot", "twoshot"])
def test_standalone_allreduce_ipc(algo):
    world = 2
    with tempfile.TemporaryDirectory() as d:
        spawn_group(_ar_worker, world, lambda port: (world, port, d, algo))
        for r in range(world):
            res = torch.load(os.path.join(d, f"r{r}.pt"), weights_only=True)["res"]
            for it in range(4):
                assert torch.all(res[it] == float(1 + it + 2 + it))


SIZES = (262144, 1000, 4, 1 << 20, 12)


def _ar_values_worker(rank, world, port, outdir, algo):
    """Every element of random inputs, sizes from 4 floats to 4 MiB, parity
    alternating, in-place on the last call; one process per replica (the
    production shape: one process per GPU, here all on cuda:0)."""
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK="0",
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from hipdsml.parallel.xchg import XgmiAllReduce

    ctx = DistContext.from_env(device="cuda", backend="gloo")
    ar = XgmiAllReduce(ctx, max(SIZES), algo=algo, timeout_ms=5000.0)
    out = {}
    for n in SIZES:
        g = torch.Generator().manual_seed(n)
        for it in range(3):
            host = [torch.randn(n, generator=g) for _ in range(world)]
            x = host[rank].to(ctx.device)
            ar(x)
            out[f"{n}/{it}"] = x.cpu()
    torch.cuda.synchronize()
    ar.check()
    torch.save(out, os.path.join(outdir, f"r{rank}.pt"))
    ctx.destroy()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("algo", ["oneshot", "twoshot"])
def test_standalone_allreduce_values_ipc(world, algo):
    with tempfile.TemporaryDirectory() as d:
        spawn_group(_ar_values_worker, world, lambda port: (world, port, d, algo))
        res = [torch.load(os.path.join(d, f"r{r}.pt"), weights_only=True) for r in range(world)]
    for n in SIZES:
        g = torch.Generator().manual_seed(n)
        for it in range(3):
            host = [torch.randn(n, generator=g) for _ in range(world)]
            want = host[0].clone()
            for h in host[1:]:
                want = want + h  # the kernel's rank-ordered sum
            for r in range(world):
                got = res[r][f"{n}/{it}"]
                bad = (got != want).nonzero().flatten()
                assert bad.numel() == 0, (n, it, r, bad.numel(), bad[:4].tolist())

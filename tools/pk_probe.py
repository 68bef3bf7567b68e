#!/usr/bin/env python3
"""Compute-plus-push cost of the persistent data-parallel step (sync='pk') on
ONE GPU, per replica count N, with no peer to wait for: one replica runs the
N-rank persistent launch while the other N-1 ranks' receive buffers live on
the same device and every flag it would wait on is preset.  Each step then
holds the kernel's own work plus its pushes (into local uncached HBM instead
of over xGMI) but no link transfer and no peer skew -- the lone-replica probe
of profiles/r1_sync_probe_lone_replica.json, for every persistent form:
algo 0 pk, 1 pk2, 2 pkg, 3 pkg2, 4 pkx.  The Gram forms poll the peers' dZ1
rows by their tags, which no preset can match: the probe switch of the kernel
(mlp_persist_set_probe, testing only) takes them as arrived; pkx reads N
copies of this replica's swizzled shard as the all-gathered inputs.

Prints one JSON line per N, with the exchange bytes each replica sends per
step (to all peers) from the kernel's slot layout.

--mirror runs the kernel's MIRROR test mode instead: every push to a peer
lands in this replica's own receive buffer in that peer's slot, with real tags
and flags, so the replica waits for its own pushes exactly as for a peer's.
With --hop-us T1,T2,... (measurement build: python -m hipdsml._build
--measure) every such hop becomes usable only T us after its publication
(kernels/mlp_persist.hip g_pk_hop): the step time at each T prices what the
xGMI latency a one-GPU run lacks costs each form (one line per N and T)."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def pk_bytes_out(n: int, algo: int = 0) -> int:
    """Bytes one replica pushes per step at n ranks (kernels/mlp_persist.hip).
    Direct form (pk / pk2): each of the 224 layer-1 waves sums an
    8-float-per-lane slot (2 KiB), the 16 gradient-block waves 16 / 8 / 4
    floats per lane (3 layers: wave 0 four float4, waves 1-3 two).  Gram forms
    (pkg / pkg2 / pkx): the 224 layer-1 slots (not in pkx), the 16 gradient
    tiles' slots (3 layers: 2 dW2 waves of 4 floats a lane each, the 4 W3
    owners a dW3 wave carrying the bias partials in its padding rows: 36
    slots of 1 KiB of values) and this replica's
    dZ1 rows as 8-B granules (64 x 128 x 8 = 64 KiB) to every peer.  One-shot:
    every slot to every peer; two-shot: (n-1)/n of each slot to its owners,
    then the owners' (n-1)/n share to every peer."""
    if algo <= 1:
        slot_bytes = 224 * 64 * 8 * 4 + 4 * (64 * 16 * 4 + 3 * 64 * 8 * 4)
    else:
        slot_bytes = (224 * 64 * 8 * 4 if algo < 4 else 0) + (36 if algo != 3 else 40) * 1024
    out = (n - 1) * slot_bytes if algo in (0, 2, 4) else 2 * (n - 1) * slot_bytes // n
    if algo >= 2:
        out += (n - 1) * 64 * 128 * 8
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--launch", type=int, default=0, help="steps per launch (0: all in one)")
    ap.add_argument("--stamps", default="", help="also write the phase stamps of each N (JSON lines)")
    ap.add_argument("--helpers", type=int, default=-1,
                    help="pkx dW1 helper blocks per layer-1 block (-1: the default by N)")
    ap.add_argument("--place", type=int, default=1,
                    help="hand-off buffers tried per N (fresh allocations; every one timed, "
                         "us_per_step = the fastest, place_us = all)")
    ap.add_argument("--algo", type=int, default=0,
                    help="0 pk, 1 pk2, 2 pkg, 3 pkg2, 4 pkx (exchange-free layer 1)")
    ap.add_argument("--l1push", type=int, default=-1,
                    help="pkx dZ1 row pushes: 1 from the layer-1 owner blocks, 0 from the chains, -1 default")
    ap.add_argument("--push-stamps", default="",
                    help="measurement build: also write the pusher-0 / tile-0 gather timeline (JSON lines)")
    ap.add_argument("--mirror", action="store_true",
                    help="mirror test mode (pushes loop back with real tags / flags) instead of the probe")
    ap.add_argument("--hop-us", default="",
                    help="mirror mode, measurement build: extra one-way hop latencies to sweep (us)")
    a = ap.parse_args()
    hops = [float(x) for x in a.hop_us.split(",")] if a.hop_us else [0.0]
    if a.hop_us and not a.mirror:
        ap.error("--hop-us needs --mirror")
    import torch

    from hipdsml.data.mnist import synthetic_mnist
    from hipdsml.engine.trainer import MlpTrainer
    from hipdsml.models.mlp import MlpSpec
    from hipdsml.ops.native import require_native
    from hipdsml.parallel.dist import DistContext
    from hipdsml.parallel.xchg import make_local_group

    C = require_native()
    C.mlp_persist_set_pkx_helpers(a.helpers)
    C.mlp_persist_set_pkx_l1push(a.l1push)
    dev = torch.device("cuda", 0)
    for n in [int(x) for x in a.ranks.split(",")]:
        tr = MlpTrainer(MlpSpec((784, 128, 64, 10)), synthetic_mnist(64 * 100, seed=0),
                        batch=64, lr=0.01, seed=0, ctx=DistContext(device=dev))
        assert tr.persistent
        xs = []
        if n > 1:
            half, ntiles = C.MlpRunner.persist_xchg_size(n, a.algo)
            xs = make_local_group(None, [0] * n, 5000.0, half_floats=half, ntiles=ntiles)
            if not a.mirror:
                for x in xs:
                    x.fill_flags(1 << 62)
            tr.runner.set_world_size(n)
            if a.algo >= 2:
                from hipdsml.parallel.xchg import swizzle_inputs

                nb = tr.nbatches
                Xs = tr.X[: nb * 64, :784].reshape(1, nb, 64, 784).expand(n, nb, 64, 784)
                tr.runner.set_persist_gram(C.gram_table(Xs.reshape(n, nb * 64, 784).contiguous(),
                                                        tr.X, nb, 64, 784))
                if a.algo == 4:
                    xall = swizzle_inputs(Xs.reshape(n, nb * 64, 784), 64)
                    tr.runner.set_persist_xall(xall, xall[0].numel())
                C.mlp_persist_set_probe(1)
            if a.mirror:
                C.mlp_persist_set_probe(2)
            tr.runner.set_persist(tr.pk_buf, tr.pk_err, 5000.0, xs[0], a.algo)
        torch.cuda.synchronize()

        def run(k):
            per = a.launch or k
            while k > 0:
                tr.train_steps(min(per, k))
                k -= per

        def timed():
            run(200)
            tr.synchronize()
            t0 = time.perf_counter()
            run(a.steps)
            tr.synchronize()
            return (time.perf_counter() - t0) / a.steps

        if a.hop_us:
            assert C.measure_build, "--hop-us needs the measurement build (python -m hipdsml._build --measure)"
            for hop in hops:
                C.mlp_persist_set_hop(hop)  # takes effect at the next launch (tags keep rising)
                dt = timed()
                print(json.dumps({"mode": ["pk", "pk2", "pkg", "pkg2", "pkx"][a.algo] if n > 1 else "none",
                                  "ranks": n, "mirror": True, "hop_us": hop,
                                  "us_per_step": round(dt * 1e6, 2)}), flush=True)
            C.mlp_persist_set_hop(0)
            C.mlp_persist_set_probe(0)
            del tr, xs
            torch.cuda.synchronize()
            continue
        place_us = []
        cands = [tr.pk_buf]
        best_dt, best_buf = None, tr.pk_buf
        for k in range(max(1, a.place)):
            if k:
                cands.append(torch.zeros_like(tr.pk_buf))
                tr.pk_buf = cands[-1]
                if n > 1:
                    tr.runner.set_persist(tr.pk_buf, tr.pk_err, 5000.0, xs[0], a.algo)
                else:
                    tr.runner.set_persist(tr.pk_buf, tr.pk_err, 5000.0)
            t = timed()
            place_us.append(round(t * 1e6, 2))
            if best_dt is None or t < best_dt:
                best_dt, best_buf = t, tr.pk_buf
        if best_buf is not tr.pk_buf:  # stamps (below) on the fastest buffer
            tr.pk_buf = best_buf
            if n > 1:
                tr.runner.set_persist(tr.pk_buf, tr.pk_err, 5000.0, xs[0], a.algo)
            else:
                tr.runner.set_persist(tr.pk_buf, tr.pk_err, 5000.0)
        dt = best_dt
        stamps = None
        if a.stamps:
            from pk_stamps import decode

            C.mlp_persist_set_stamping(True)
            run(32)
            tr.synchronize()
            C.mlp_persist_set_stamping(False)
            stamps = decode(C.mlp_persist_stamps(), tr.spec)
            if a.push_stamps:
                assert C.measure_build, "--push-stamps needs the measurement build"
                import statistics
                raw, ps = C.mlp_persist_stamps(), C.mlp_persist_push_stamps()
                keys = ["pusher_poll_start", "pusher_staged_seen", "pusher_pushes_issued", "pusher_pushes_acked",
                        "gather_loads_issued", "gather_first_data", "gather_done"]
                rel = {k: [] for k in keys}
                for row in range(6):
                    g0 = raw[(3 * 8 + 2 + row) * 8 + 0]
                    gs = [raw[(3 * 8 + 2 + row) * 8 + k] for k in range(4)]
                    pr = [ps[row * 4 + k] for k in range(4)]
                    if not g0 or not all(gs) or not all(pr[:3]):
                        continue
                    for k, v in zip(keys, pr + gs[1:]):
                        if v:
                            rel[k].append((v - g0) / 100.0)
                with open(a.push_stamps, "a") as f:
                    f.write(json.dumps({"ranks": n, "mirror": a.mirror,
                                        "us_after_tile0_gather_entry": {k: round(statistics.median(v), 2)
                                                                        for k, v in rel.items() if v},
                                        "rows": len(rel["gather_done"])}) + "\n")
            with open(a.stamps, "a") as f:
                f.write(json.dumps({"mode": ["pk", "pk2", "pkg", "pkg2", "pkx"][a.algo], "ranks": n,
                                    "mirror": a.mirror, "l1push": a.l1push,
                                    "stamps": stamps}) + "\n")
        C.mlp_persist_set_probe(0)
        name = ["pk", "pk2", "pkg", "pkg2", "pkx"][a.algo]
        print(json.dumps({"mode": name if n > 1 else "none", "ranks": n, "mirror": a.mirror, "l1push": a.l1push,
                          "us_per_step": round(dt * 1e6, 2), "place_us": place_us,
                          "bytes_out_per_step": pk_bytes_out(n, a.algo),
                          "bytes_per_peer_per_step": pk_bytes_out(n, a.algo) // max(n - 1, 1)}),
              flush=True)
        del tr, xs, cands, best_buf
        torch.cuda.synchronize()
    return 0


if __name__ == "__main__":
    sys.exit(main())

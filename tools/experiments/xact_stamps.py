#!/usr/bin/env python3
"""Phase timeline of the activation-exchange K_C (kernels/mlp_f32_xact.hip) from
in-kernel s_memrealtime stamps (100 MHz), lone-replica probe setup (peers'
exchange buffers on the same GPU, every flag preset): pusher block 0 and the
first tile block, us relative to the pusher's entry.  Diagnostic only."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main() -> int:
    import torch

    from hipdsml.data.mnist import synthetic_mnist
    from hipdsml.engine.trainer import MlpTrainer
    from hipdsml.models.mlp import MlpSpec
    from hipdsml.ops.native import require_native
    from hipdsml.parallel.dist import DistContext
    from hipdsml.parallel.xchg import make_local_act_group, swizzle_inputs

    C = require_native()
    dev = torch.device("cuda", 0)
    names = {0: "P.entry", 1: "P.loaded", 2: "P.stores_issued", 3: "P.drained",
             8: "T.entry", 9: "T.pre_poll", 10: "T.polled", 11: "T.mfma_done", 12: "T.reduced",
             13: "T.stored"}
    out = {}
    for n in [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "2,8").split(",")]:
        tr = MlpTrainer(MlpSpec((784, 128, 64, 10)), synthetic_mnist(64 * 100, seed=0), batch=64,
                        lr=0.01, seed=0, ctx=DistContext(device=dev))
        rows = tr.nbatches * 64
        Xall = swizzle_inputs(torch.stack([tr.X[:rows]] * n), 64)
        xs = make_local_act_group(tr.layout, [0] * n)
        tr.runner.set_act_exchange(xs[0], Xall, Xall[0].numel())
        for x in xs:
            x.fill_flags(1 << 62)
        tr.train_steps(20)
        tr.runner.synchronize()
        C.mlp_set_stamping(True)
        acc = {k: 0.0 for k in names}
        reps = 50
        for _ in range(reps):
            tr.train_steps(1)
            tr.runner.synchronize()
            st = C.mlp_stamps_xact()
            for k in names:
                acc[k] += (st[k] - st[0]) * 10.0 / 1e3  # us
        C.mlp_set_stamping(False)
        out[f"N{n}"] = {names[k]: round(v / reps, 3) for k, v in acc.items()}
        del tr, xs
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())

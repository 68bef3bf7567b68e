"""Phase timeline of the fused wide forward (kernels/wide_fwd.hip): one
stamped launch inside a training step, per-workgroup s_memrealtime (100 MHz)
at entry, layer-1 tile published, slice ready, A + W2 landed, MFMAs done,
exit, layer-1 operands landed, layer-1 partials in LDS.  Prints one JSON line: medians / maxima in us from the first entry."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from hipdsml.data.mnist import synthetic_mnist  # noqa: E402
from hipdsml.engine.wide import WideMlpTrainer  # noqa: E402
from hipdsml.models.mlp import MlpSpec  # noqa: E402


def main() -> None:
    spec = MlpSpec.parse("784-4096-4096-10")
    tr = WideMlpTrainer(spec, synthetic_mnist(64 * 8, seed=1), batch=64, graph=False, fused_fwd=True)
    assert tr.fused_fwd, "fused forward unavailable"
    C = tr.C
    tr.train_steps(20)
    tr.synchronize()
    out = {}
    early = os.environ.get("WF_EARLY_DMA", "0") == "1"
    C.wide_fwd2_set_early_dma(early)
    out["early_dma"] = early
    for rep in range(3):
        C.wide_fwd2_set_stamping(True)
        tr.train_steps(1)
        tr.synchronize()
        C.wide_fwd2_set_stamping(False)
        v = torch.tensor(C.wide_fwd2_stamps(), dtype=torch.float64).view(256, 8)
        t0 = v[:, 0].min()
        rel = (v - t0) / 100.0  # us
        names = ["entry", "l1_published", "slice_ready", "operands_landed", "mfma_done", "exit", "l1_loaded",
                 "l1_partials"]
        out[f"rep{rep}"] = {n: {"med": round(rel[:, k].median().item(), 2), "max": round(rel[:, k].max().item(), 2)}
                            for k, n in enumerate(names)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()

"""Phase stamps of the fused input-layer launch (kernels/wide_input.hip,
measurement build): per workgroup s_memrealtime (100 MHz) at entry, loads
landed (dZ_1 summed), first barrier, update loop done, bias barrier, forward
MFMAs done, partials barrier, exit.  Prints the median over workgroups and
steps of each phase, in us, relative to the launch's first entry stamp."""
import json
import statistics
import sys

import torch

sys.path.insert(0, ".")
from hipdsml.data.mnist import synthetic_mnist  # noqa: E402
from hipdsml.engine.wide import WideMlpTrainer  # noqa: E402
from hipdsml.models.mlp import MlpSpec  # noqa: E402

NAMES = ["entry", "loads+dZ1", "barrier1", "update loop", "bias barrier", "forward mfma", "partials barrier",
         "exit"]


def main():
    t = WideMlpTrainer(MlpSpec((784, 4096, 4096, 10)), synthetic_mnist(64 * 64, seed=1), batch=64, graph=False)
    C = t.C
    assert C.measure_build, "needs the measurement build (python -m hipdsml._build --measure)"
    assert t.fused_input
    import os
    dbg = int(os.environ.get("WI_DBG", "0"))
    C.wide_input_set_dbg(dbg)  # measurement: drop load kinds (kernels/wide_input.hip g_wi_dbg)
    t.train_steps(10)
    t.synchronize()
    rows = {k: [] for k in NAMES}
    since_first = {k: [] for k in NAMES}
    for _ in range(20):
        C.wide_input_set_stamping(True)
        t.train_steps(1)
        t.synchronize()
        C.wide_input_set_stamping(False)
        v = C.wide_input_stamps()
        st = [v[8 * b:8 * b + 8] for b in range(256)]
        t0 = min(s[0] for s in st)
        for s in st:
            for k in range(8):
                since_first[NAMES[k]].append((s[k] - t0) / 100.0)
                if k:
                    rows[NAMES[k]].append((s[k] - s[k - 1]) / 100.0)
    ev = []
    for _ in range(3):  # launch time from events, 50 steps
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        t.train_steps(50)
        e1.record()
        t.synchronize()
        ev.append(e0.elapsed_time(e1) * 1000 / 50)
    out = {"dbg": dbg, "us_per_step": round(min(ev), 2), "phase_us_median": {k: round(statistics.median(v), 2) for k, v in rows.items() if v},
           "since_launch_us_median": {k: round(statistics.median(v), 2) for k, v in since_first.items()},
           "since_launch_us_max": {k: round(max(v), 2) for k, v in since_first.items()}}
    print(json.dumps(out))


if __name__ == "__main__":
    main()

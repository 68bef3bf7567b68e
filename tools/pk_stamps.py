"""Phase timeline of the persistent fused step (kernels/mlp_persist.hip):
layer-1 block 0 and chain block 0, steps 8..15 of one launch (s_memrealtime,
100 MHz -> us).  Prints per-phase medians and writes JSON to argv[1]."""
import json
import statistics
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from hipdsml.data.mnist import synthetic_mnist  # noqa: E402
from hipdsml.engine.trainer import MlpTrainer  # noqa: E402
from hipdsml.models.mlp import MlpSpec  # noqa: E402
from hipdsml.ops.native import require_native  # noqa: E402
from hipdsml.parallel.dist import DistContext  # noqa: E402

C = require_native()
t = MlpTrainer(MlpSpec((784, 128, 64, 10)), synthetic_mnist(64 * 100, seed=1), batch=64, lr=0.01,
               ctx=DistContext(device=torch.device("cuda", 0)))
assert t.persistent
t.train_steps(100)
t.synchronize()
C.mlp_persist_set_stamping(True)
t.train_steps(32)
t.synchronize()
C.mlp_persist_set_stamping(False)
v = C.mlp_persist_stamps()
st = [[[v[(r * 8 + s) * 8 + p] for p in range(8)] for s in range(8)] for r in range(3)]
L1 = ["fwd+publish", "dZ1 wait", "bwd+update"]
CH = ["partials wait", "L2/L3 fwd+softmax", "dZ2,dZ1 publish", "row exchange", "dW2/dW3+update"]
out = {"layer1": {}, "chain": {}, "step_us": None}
for name, role, labels in (("layer1", 0, L1), ("chain", 1, CH)):
    for k, lab in enumerate(labels):
        d = [(st[role][s][k + 1] - st[role][s][k]) / 100.0 for s in range(8)]
        out[name][lab] = round(statistics.median(d), 3)
steps = [(st[0][s + 1][0] - st[0][s][0]) / 100.0 for s in range(7)]
out["step_us"] = round(statistics.median(steps), 3)
# cross-role: chain partial-wait end vs layer-1 publish
out["l1_publish_to_chain_ready_us"] = round(statistics.median(
    [(st[1][s][1] - st[0][s][1]) / 100.0 for s in range(8)]), 3)
out["chain"]["dW2 MFMAs (wave 0)"] = round(statistics.median([(st[1][s][6] - st[1][s][4]) / 100.0 for s in range(8)]), 3)
out["chain"]["W2/W3/b updates (wave 0)"] = round(statistics.median([(st[1][s][7] - st[1][s][6]) / 100.0 for s in range(8)]), 3)
out["chain"]["barrier wait after wave 0"] = round(statistics.median([(st[1][s][5] - st[1][s][7]) / 100.0 for s in range(8)]), 3)
out["chain_dz1_publish_to_l1_ready_us"] = round(statistics.median(
    [(st[0][s][2] - st[1][s][3]) / 100.0 for s in range(8)]), 3)

print(json.dumps(out, indent=1))
if len(sys.argv) > 1:
    json.dump(out, open(sys.argv[1], "w"), indent=1)

"""Phase breakdown of the fused row-chain kernel from in-kernel s_memrealtime
stamps (block 0, 100 MHz clock).  Diagnostic only: the stamping build adds a
scalar branch per phase."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from hipdsml.data.mnist import synthetic_mnist  # noqa: E402
from hipdsml.engine.trainer import MlpTrainer  # noqa: E402
from hipdsml.models.mlp import MlpSpec  # noqa: E402
from hipdsml.ops.native import require_native  # noqa: E402
from hipdsml.parallel.dist import DistContext  # noqa: E402

C = require_native()
spec = MlpSpec.parse(sys.argv[1] if len(sys.argv) > 1 else "784-128-64-10")
tr = MlpTrainer(spec, synthetic_mnist(64 * 20, seed=0, dim=spec.dims[0]), batch=64,
                ctx=DistContext(device=torch.device("cuda", 0)), persist=False)
tr.train_steps(20)
tr.synchronize()
C.mlp_set_stamping(True)
generic = ["slabs+stage", "fwd", "softmax", "bwd"]
fast = ["loads+stage", "fwd-L2", "fwd-L3-partial", "softmax", "bwd-L3", "bwd-L2"]
fast_idx = [0, 1, 2, 3, 4, 5, 7]
acc_g = [0.0] * 4
acc_f = [0.0] * 6
clk = [0.0, 0.0]
n = 50
for _ in range(n):
    tr.train_steps(1)
    tr.synchronize()
    s = C.mlp_stamps()
    f = C.mlp_stamps_fast()
    for k in range(4):
        acc_g[k] += (s[k + 1] - s[k]) * 10.0  # ns
    for k in range(6):
        acc_f[k] += (f[fast_idx[k + 1]] - f[fast_idx[k]]) * 10.0
    clk[0] += f[16 + 7] - f[16 + 0]
    clk[1] += f[7] - f[0]
C.mlp_set_stamping(False)
if any(acc_g):
    print("generic rowchain (us, block 0):", {generic[k]: round(acc_g[k] / n / 1e3, 3) for k in range(4)})
if any(acc_f):
    print("fast rowchain (us, block 0):", {fast[k]: round(acc_f[k] / n / 1e3, 3) for k in range(6)},
          "total", round(sum(acc_f) / n / 1e3, 3),
          "shader clock MHz", round(100.0 * clk[0] / max(clk[1], 1), 1))

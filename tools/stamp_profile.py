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
                ctx=DistContext(device=torch.device("cuda", 0)))
tr.train_steps(20)
tr.synchronize()
C.mlp_set_stamping(True)
names = ["start", "slabs+stage", "fwd", "softmax", "bwd"]
acc = [0.0] * 4
n = 50
for _ in range(n):
    tr.train_steps(1)
    tr.synchronize()
    s = C.mlp_stamps()
    for k in range(4):
        acc[k] += (s[k + 1] - s[k]) * 10.0  # ns
C.mlp_set_stamping(False)
print("rowchain phase (us, block 0):", {names[k + 1]: round(acc[k] / n / 1e3, 3) for k in range(4)})

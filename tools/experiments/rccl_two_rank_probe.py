"""Probe: can two RCCL ranks share one GPU on this box (RCCL normally rejects
duplicate devices)?  Launch: python -m torch.distributed.run --nproc-per-node 2
--master-addr 127.0.0.1 tools/rccl_two_rank_probe.py  (both ranks use cuda:0)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from hipdsml.ops.native import require_native  # noqa: E402
from hipdsml.parallel.dist import DistContext  # noqa: E402

os.environ["LOCAL_RANK"] = "0"  # force both ranks onto GPU 0
ctx = DistContext.from_env(device="cuda", backend="gloo")
C = require_native()
uid = ctx.share_bytes("probe/uid", C.rccl_unique_id() if ctx.rank == 0 else None)
try:
    comm = C.RcclComm(uid, ctx.rank, ctx.world_size, 0, True)
    t = torch.full((1 << 18,), float(ctx.rank + 1), device="cuda:0")
    comm.ring_allreduce_(t, 0, 1 << 16)
    comm.allreduce_(t, 0)
    torch.cuda.synchronize()
    print(f"rank {ctx.rank}: OK value={t[0].item()} (want {2 * sum(range(1, ctx.world_size + 1))})", flush=True)
except Exception as e:
    print(f"rank {ctx.rank}: RCCL two-ranks-one-GPU FAILED: {e}", flush=True)
ctx.destroy()

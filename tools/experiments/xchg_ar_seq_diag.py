"""Replay the in-process standalone all-reduce test sequence and report the
first wrong result (stream kind selectable)."""
import sys

import torch

sys.path.insert(0, ".")
from hipdsml.ops.native import require_native  # noqa: E402
from hipdsml.parallel.xchg import make_local_group  # noqa: E402

DEV = torch.device("cuda", 0)
C = require_native()
mode = sys.argv[1]
pool = []


def streams(n):
    while len(pool) < n:
        if mode.startswith("dedicated"):
            pool.append(torch.cuda.ExternalStream(C.dedicated_stream(0), device=DEV))
        else:
            pool.append(torch.cuda.Stream(DEV))
    return pool[:n]


def case(world, n, algo):
    n = n // 4 * 4
    side = torch.cuda.Stream(DEV)
    with torch.cuda.stream(side):
        xs = make_local_group(None, [0] * world, 5000.0, half_floats=2 << 20, ntiles=256)
        g = torch.Generator().manual_seed(n)
        ss = streams(world)
        for it in range(3):
            host = [torch.randn(n, generator=g) for _ in range(world)]
            ins = [h.to(DEV) for h in host]
            outs = [torch.empty_like(i) for i in ins]
            torch.cuda.synchronize()
            for r in range(world):
                if mode.endswith("ev"):
                    ss[r].wait_stream(side)
                with torch.cuda.stream(ss[r]):
                    if it == 2:
                        xs[r].allreduce_(ins[r], algo)
                    else:
                        xs[r].allreduce(ins[r], outs[r], algo)
            if mode.endswith("ev"):
                for r in range(world):
                    side.wait_stream(ss[r])
            torch.cuda.synchronize()
            want = host[0].clone()
            for h in host[1:]:
                want = want + h
            for r in range(world):
                got = (ins[r] if it == 2 else outs[r]).cpu()
                bad = (got != want).nonzero().flatten()
                if bad.numel():
                    inn = ins[r].cpu()
                    print(f"BAD {mode} world={world} n={n} algo={algo} it={it} r={r} nbad={bad.numel()} "
                          f"first={bad[:3].tolist()} got={got[bad[:3]].tolist()} want={want[bad[:3]].tolist()} "
                          f"in={inn[bad[:3]].tolist()} host={host[r][bad[:3]].tolist()} err={[x.error() for x in xs]}",
                          flush=True)
                    return False
    return True


ok = True
for algo in (0, 1):
    for world, n in [(2, 262144), (3, 1000), (2, 4), (3, 1 << 20), (3, 12)]:
        ok &= case(world, n, algo)
print(mode, "ALL OK" if ok else "FAILURES", flush=True)

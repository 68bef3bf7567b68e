"""Multi-ring all-reduce schedule (csrc/runtime/ring_plan.h), checked on the
CPU by simulating every rank's ncclSend/ncclRecv groups with per-pair FIFO
matching (RCCL semantics): no deadlock, matched lengths, exact sums."""
from collections import defaultdict, deque

import numpy as np
import pytest

C = pytest.importorskip("hipdsml.ops.native").load_native()
if C is None:
    pytest.skip("native extension not built", allow_module_level=True)


def simulate(n, count, align, chunk, max_rings, seed=0):
    rng = np.random.default_rng(seed)
    init = [rng.integers(-1000, 1000, size=count).astype(np.int64) for _ in range(n)]
    buf = [b.copy() for b in init]
    plans = [C.ring_schedule(n, r, count, align, chunk, max_rings) for r in range(n)]
    pc = [0] * n
    posted = [False] * n
    q = defaultdict(deque)  # (src, dst) -> deque of arrays
    while True:
        progress = False
        for r in range(n):
            if pc[r] >= len(plans[r]):
                continue
            g = plans[r][pc[r]]
            if not posted[r]:
                for (_, sp, so, sl, _, _, _, _) in g:
                    if sl > 0:
                        q[(r, sp)].append(buf[r][so:so + sl].copy())
                posted[r] = True
                progress = True
            need = defaultdict(int)
            for (_, _, _, _, rp, _, rl, _) in g:
                if rl > 0:
                    need[rp] += 1
            if all(len(q[(p, r)]) >= k for p, k in need.items()):
                for (_, _, _, _, rp, ro, rl, red) in g:
                    if rl > 0:
                        data = q[(rp, r)].popleft()
                        assert len(data) == rl, "send/recv length mismatch"
                        if red:
                            buf[r][ro:ro + rl] += data
                        else:
                            buf[r][ro:ro + rl] = data
                pc[r] += 1
                posted[r] = False
                progress = True
        if all(pc[r] >= len(plans[r]) for r in range(n)):
            break
        assert progress, "deadlock"
    assert all(len(v) == 0 for v in q.values()), "unmatched sends"
    want = sum(init)
    for r in range(n):
        np.testing.assert_array_equal(buf[r], want)
    return plans


@pytest.mark.parametrize("n", [2, 3, 4, 5, 6, 7, 8])
@pytest.mark.parametrize("count,chunk", [(262144, 0), (262144, 8192), (109400, 4096), (37, 0),
                                         (4, 0), (1000, 12)])
@pytest.mark.parametrize("max_rings", [0, 1])
def test_ring_schedule_correct(n, count, chunk, max_rings):
    simulate(n, count, 4, chunk, max_rings, seed=n * 1000 + count)


def test_directed_rings_use_disjoint_links():
    for n in range(2, 9):
        rings = C.directed_rings(n)
        assert len(rings) == (1 if n == 2 else 2 * ((n - 1) // 2))
        links = set()
        for rg in rings:
            assert sorted(rg) == list(range(n))
            for i in range(n):
                e = (rg[i], rg[(i + 1) % n])
                if n > 2:
                    assert e not in links
                links.add(e)
    assert len(C.directed_rings(8)) == 6  # 6 of the 7 xGMI links per GPU

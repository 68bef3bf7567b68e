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


def simulate_pipelined(n, count, align, chunk, max_rings, lazy_reduce=True, seed=0):
    """Two streams per rank, as RcclComm::ring_allreduce runs the pipelined
    ring: the transfer groups in order on the comm stream (each first waiting
    for its ring_pipeline dependencies), the reduce-scatter's reduces in order
    on the reduce stream.  With lazy_reduce the reduces run only when no
    transfer can progress anywhere (the latest legal moment), so a missing
    dependency shows up as a wrong sum, a scratch slot overwritten before its
    reduce read it, or a deadlock.  Returns how many transfer groups completed
    while the previous group's reduce was still pending (the overlap)."""
    rng = np.random.default_rng(seed)
    init = [rng.integers(-1000, 1000, size=count).astype(np.int64) for _ in range(n)]
    buf = [b.copy() for b in init]
    plans = [C.ring_schedule(n, r, count, align, chunk, max_rings) for r in range(n)]
    deps = [C.ring_pipeline(n, r, count, align, chunk, max_rings) for r in range(n)]
    pc = [0] * n                      # next transfer group per rank
    posted = [False] * n
    red_q = [deque() for _ in range(n)]   # reduce stream: FIFO of group indices
    red_done = [set() for _ in range(n)]
    scratch = [dict() for _ in range(n)]  # (slot, ring) -> payload not yet reduced
    q = defaultdict(deque)
    overlap = 0
    while True:
        progress = False
        for r in range(n):
            if pc[r] >= len(plans[r]):
                continue
            i = pc[r]
            g = plans[r][i]
            wr, slot, sf = deps[r][i]
            red = bool(g) and g[0][7]
            if not posted[r]:
                if wr >= 0 and wr not in red_done[r]:
                    continue
                if red and sf >= 0 and sf not in red_done[r]:
                    continue
                for (_, sp, so, sl, _, _, _, _, *_rest) in g:
                    if sl > 0:
                        q[(r, sp)].append(buf[r][so:so + sl].copy())
                posted[r] = True
                progress = True
            need = defaultdict(int)
            for x in g:
                if x[6] > 0:
                    need[x[4]] += 1
            if all(len(q[(p, r)]) >= k for p, k in need.items()):
                for x in g:
                    ring, rp, ro, rl, red_x = x[0], x[4], x[5], x[6], x[7]
                    if rl > 0:
                        data = q[(rp, r)].popleft()
                        assert len(data) == rl
                        if red_x:
                            assert (slot, ring) not in scratch[r], "scratch slot overwritten before its reduce"
                            scratch[r][(slot, ring)] = (ro, data)
                        else:
                            buf[r][ro:ro + rl] = data
                if red:
                    red_q[r].append(i)
                if i > 0 and plans[r][i - 1] and plans[r][i - 1][0][7] and (i - 1) not in red_done[r]:
                    overlap += 1
                pc[r] += 1
                posted[r] = False
                progress = True
        if not progress or not lazy_reduce:
            # the reduce streams advance (one reduce per rank per round)
            for r in range(n):
                if red_q[r]:
                    i = red_q[r].popleft()
                    _, slot, _ = deps[r][i]
                    for x in plans[r][i]:
                        if x[7] and x[6] > 0:
                            ro, data = scratch[r].pop((slot, x[0]))
                            buf[r][ro:ro + len(data)] += data
                    red_done[r].add(i)
                    progress = True
        if all(pc[r] >= len(plans[r]) and not red_q[r] for r in range(n)):
            break
        assert progress, "deadlock"
    want = sum(init)
    for r in range(n):
        np.testing.assert_array_equal(buf[r], want)
    return overlap


@pytest.mark.parametrize("n", [2, 3, 4, 8])
@pytest.mark.parametrize("count,chunk", [(262144, 8192), (109400, 4096), (1000, 12), (4096, 0)])
@pytest.mark.parametrize("lazy", [True, False])
def test_pipelined_ring_dependencies_are_sufficient(n, count, chunk, lazy):
    ov = simulate_pipelined(n, count, 4, chunk, 0, lazy_reduce=lazy, seed=n + count)
    if lazy and chunk and count // (2 * n * max(1, len(C.directed_rings(n)))) > chunk:
        # several chunk rounds per step: transfers run ahead of the reduces
        assert ov > 0


def test_pipeline_slots_alternate_and_point_backwards():
    for n in (2, 3, 8):
        plan = C.ring_schedule(n, 1, 100000, 4, 2048, 0)
        deps = C.ring_pipeline(n, 1, 100000, 4, 2048, 0)
        reds = [i for i, g in enumerate(plan) if g and g[0][7]]
        assert [deps[i][1] for i in reds] == [k & 1 for k in range(len(reds))]
        for i, (wr, slot, sf) in enumerate(deps):
            assert wr < i and sf < i

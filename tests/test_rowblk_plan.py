"""Cost-balanced workgroup runs of the row-block global-batch update
(kernels/wgrad_sgd.hip wgrad_rowblk_plan, round 6: profiles/r6_rowblk_balance.json).
Host logic, checked on the CPU: the runs cover every unit once in launch order,
fit the workgroup budget, follow the documented cost model exactly (a Python
re-implementation of the greedy fill + bisection), and balance the modelled
cost better than the equal unit split they replaced."""
import pytest

native = pytest.importorskip("hipdsml.ops.native")

RBN, OV = 128, 1.5  # kRbN (W rows of an n block), segment overhead in k tiles


def _units(N, K):
    out = []  # (segment id) per unit, launch order
    us = 0
    for n, k in zip(N, K):
        kts, nbs = (k + 63) // 64, (n + RBN - 1) // RBN
        for nbk in range(nbs):
            out += [us + nbk * kts] * kts
        us += kts * nbs
    return out


def _fill(segs, T, starts=None):
    g, cur, prev = 0, 0.0, -1
    if starts is not None:
        starts.append(0)
    for uu, seg in enumerate(segs):
        c = 1.0 + (OV if (cur == 0.0 or seg != prev) else 0.0)
        if cur > 0.0 and cur + c > T:
            g += 1
            if starts is not None:
                starts.append(uu)
            cur, c = 0.0, 1.0 + OV
        cur += c
        prev = seg
    g += 1
    if starts is not None:
        starts.append(len(segs))
    return g


def _plan_ref(N, K, groups):
    segs = _units(N, K)
    lo, hi = 1.0, len(segs) * (1.0 + OV) + 1.0
    for _ in range(40):
        mid = 0.5 * (lo + hi)
        if _fill(segs, mid) <= groups:
            hi = mid
        else:
            lo = mid
    st = []
    _fill(segs, hi, st)
    return st


def _run_costs(segs, starts):
    costs = []
    for a, b in zip(starts[:-1], starts[1:]):
        c, prev = 0.0, -1
        for uu in range(a, b):
            c += 1.0 + (OV if (uu == a or segs[uu] != prev) else 0.0)
            prev = segs[uu]
        costs.append(c)
    return costs


SHAPES = [
    ([10, 4096, 4096], [4096, 4096, 784], 256),  # the wide model's update, launch order
    ([4096, 4096], [4096, 784], 256),
    ([10, 4096, 4096], [4096, 4096, 784], 100),
    ([128, 64], [784, 128], 256),                # fewer units than workgroups
]


@pytest.mark.parametrize("N,K,groups", SHAPES, ids=lambda v: str(v))
def test_rowblk_plan_matches_cost_model_and_balances(N, K, groups):
    C = native.require_native()
    st = list(C.wgrad_rowblk_plan(N, K, groups))
    segs = _units(N, K)
    assert st[0] == 0 and st[-1] == len(segs)
    assert all(b > a for a, b in zip(st[:-1], st[1:]))
    assert len(st) - 1 <= min(groups, len(segs))
    assert st == _plan_ref(N, K, groups)
    costs = _run_costs(segs, st)
    if len(segs) >= 4 * groups:
        # the model's point: no run carries much more than the mean, and the
        # longest run is shorter than the equal unit split's longest
        assert max(costs) <= 1.15 * (sum(costs) / len(costs))
        g = len(st) - 1
        eq = [len(segs) * i // g for i in range(g + 1)]
        assert max(costs) < max(_run_costs(segs, eq))

"""GPU: m = 8192 (between C3's 4096 and C5's 16384; y_w and the base row fill
k_price's LDS, WM 1 at its limit; 1,024 FTRAN workgroups) solved to
optimality and compared with an independent solver (the loop v4:286-359 run
to its exit).

Fixture: scipy HiGHS dual simplex on the seeded LP m = 8192, n = 24576
(``tests/golden/make_golden_c4.py 8192 24576 0`` in the build container;
``tests/golden/highs_8192x24576_0.json`` holds its wall time and memory).
Default path, and the same LP as a 4-shard column group (the sharded pricing
with the replicated window): |z - z*| <= 1e-9 |z*|, HiGHS's basic set, and the
shards' objectives bit-identical.
"""
import json
import os

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIXTURE = os.path.join(ROOT, "tests", "golden", "highs_8192x24576_0.json")


@pytest.fixture(scope="module")
def mid():
    with open(FIXTURE) as f:
        h = json.load(f)
    assert (h["m"], h["n"], h["seed"]) == (8192, 24576, 0)
    return h


def test_m8192_default_solves_to_highs_optimum(spx, mid):
    with spx.Context(m=mid["m"], n=mid["n"], seed=mid["seed"]) as ctx:
        cfg = ctx.config()
        assert cfg["window"] == 64 and cfg["defer_tail"] == 1 and cfg["price_lds"] == 2
        r = ctx.solve()
    print(f"m=8192 n=24576: {r.pivots} pivots, z={r.z:.15g} (HiGHS {mid['highs_z']:.15g})")
    assert r.status == spx.SolveStatus.OptimumFound
    assert abs(r.z - mid["highs_z"]) <= 1e-9 * abs(mid["highs_z"])
    assert sorted(int(j) for j in r.b_ixs) == mid["highs_basis"]


def test_m8192_group4_solves_to_highs_optimum(spx, mid):
    G = 4
    m, n, seed = mid["m"], mid["n"], mid["seed"]
    ctxs = [spx.Context(m=m, n=n, seed=seed, rank=r, nranks=G) for r in range(G)]
    try:
        st, piv = spx.group_iterate(ctxs, 0)
        while st == spx.SolveStatus.MaxIter:
            st, piv = spx.group_iterate(ctxs, 4096)
        assert st == spx.SolveStatus.OptimumFound
        zs = [c.objective() for c in ctxs]
        bases = [sorted(int(j) for j in c.state()["b_ixs"]) for c in ctxs]
    finally:
        for c in ctxs:
            c.close()
    print(f"m=8192 n=24576, 4 shards: {piv} pivots, z={zs[0]:.15g}")
    assert all(z == zs[0] for z in zs)  # replicas hold the same bits
    assert abs(zs[0] - mid["highs_z"]) <= 1e-9 * abs(mid["highs_z"])
    for b in bases:
        assert b == mid["highs_basis"]

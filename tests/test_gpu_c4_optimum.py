"""GPU: the north-star pricing-scaling shape (m = 4096, wide n) solved to
optimality and compared with an independent solver (the loop v4:286-359 run to
its exit).

The fixture comes from scipy HiGHS dual simplex in the build container
(``tests/golden/make_golden_c4.py``).  At the full C4 width (n = 131,072,
520 M nonzeros) HiGHS does not fit the build container: it failed with
std::bad_alloc at a 58 GB address-space limit, and its resident memory grows
about 135 bytes per nonzero (15.8 GB at n = 32,768), so C4 itself would need
about 70 GB of the container's 62.  The largest width pinned is therefore
n = 65,536 at m = 4096 (252 M nonzeros).  C4 itself is pinned to the oracle
through two folds (test_gpu_c45.py).

Checked on the default path (eta window, compact FTRAN, deferred tail,
captured hipGraphs) and as an in-process group of 8 column shards (the
north-star partitioning at 8 ranks: B^-1 replicated, MINLOC merge):
|z - z*| <= 1e-9 |z*| and the same basic set as HiGHS.
"""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIXTURE = os.path.join(ROOT, "tests", "golden", "highs_4096x65536_0.json")


@pytest.fixture(scope="module")
def wide():
    with open(FIXTURE) as f:
        h = json.load(f)
    assert (h["m"], h["n"], h["seed"]) == (4096, 65536, 0)
    return h


def test_wide_default_solves_to_highs_optimum(spx, wide):
    with spx.Context(m=wide["m"], n=wide["n"], seed=wide["seed"]) as ctx:
        cfg = ctx.config()
        assert cfg["window"] == 64 and cfg["defer_tail"] == 1
        r = ctx.solve()
    print(f"m=4096 n=65536: {r.pivots} pivots, z={r.z:.15g} (HiGHS {wide['highs_z']:.15g})")
    assert r.status == spx.SolveStatus.OptimumFound
    assert abs(r.z - wide["highs_z"]) <= 1e-9 * abs(wide["highs_z"])
    assert sorted(int(j) for j in r.b_ixs) == wide["highs_basis"]


def test_wide_group8_solves_to_highs_optimum(spx, wide):
    G = 8
    m, n, seed = wide["m"], wide["n"], wide["seed"]
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
    print(f"m=4096 n=65536, 8 shards: {piv} pivots, z={zs[0]:.15g}")
    assert all(z == zs[0] for z in zs)  # replicas hold the same bits
    assert abs(zs[0] - wide["highs_z"]) <= 1e-9 * abs(wide["highs_z"])
    for b in bases:
        assert b == wide["highs_basis"]

"""GPU parity at the BASELINE.json configurations themselves (C2, C3, C4),
through the C-ABI, against the oracle (oracle/simplex_oracle.c, the
restatement of src/v4_cub_reduction.cu:286-359) and the HiGHS golden optima
(tests/golden/highs_optima.json case 11 = C2, tests/golden/highs_c3.json = C3;
HiGHS stands in for solver_glpk.cpp, libglpk is absent).

Tolerances (fp64): pivot sequence (p, q) identical to the
oracle's; |z - z_highs| <= 1e-9 |z_highs|; basic set equal to HiGHS's; x_b, y,
B^-1 within 1e-9 (relative max-norm) of the oracle after K pivots.
"""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REL = 1e-9


def _rel(a, b):
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    return float(np.max(np.abs(a - b)) / max(1.0, float(np.max(np.abs(b)))))


@pytest.fixture(scope="module")
def c2_oracle(oracle, golden):
    case = golden["cases"][11]
    assert (case["m"], case["n"], case["seed"]) == (1024, 4096, 0)
    A, b, c = oracle.generate(1024, 4096, 0)
    ref = oracle.solve(A, b, c, eps=golden["eps"], trace_cap=1 << 14)
    assert ref.status == oracle.OPTIMUM_FOUND and ref.pivots == case["oracle_pivots"] == 2065
    return case, ref


@pytest.fixture(scope="module")
def c3_golden():
    path = os.path.join(ROOT, "tests", "golden", "highs_c3.json")
    with open(path) as f:
        g = json.load(f)
    assert (g["m"], g["n"], g["seed"]) == (4096, 16384, 0)
    return g


# C2 (m=1024, n=4096, seed 0): the default (auto) path, the eta window and the
# explicit rank-1 update (v4:331-333), each solved to optimality
@pytest.mark.parametrize("kw", [dict(), dict(window=64), dict(window=-1), dict(window=64, persist=True)],
                         ids=["auto", "window64", "explicit", "window64-persistent"])
def test_c2_golden_full_solve(spx, golden, c2_oracle, kw):
    case, ref = c2_oracle
    with spx.Context(m=1024, n=4096, seed=0, eps=golden["eps"], trace=4096, **kw) as ctx:
        r = ctx.solve()
        tp, tq = ctx.trace()
    assert r.status == spx.SolveStatus.OptimumFound
    assert r.pivots == 2065
    assert abs(r.z - case["highs_z"]) <= REL * abs(case["highs_z"])
    assert sorted(int(j) for j in r.b_ixs) == case["highs_basis"]
    assert list(tp) == list(ref.trace_p) and list(tq) == list(ref.trace_q)


# C3 (m=4096, n=16384, seed 0), the headline: 130 pivots = two folds of the
# default 64-window, pivot for pivot against the oracle, then the state
@pytest.mark.parametrize("kw", [dict(), dict(window=-1)], ids=["default-window64", "explicit"])
def test_c3_pivots_and_state_match_oracle(spx, oracle, kw):
    m, n, K = 4096, 16384, 130
    A, b, c = oracle.generate(m, n, 0)
    ref = oracle.solve(A, b, c, eps=1e-7, max_iter=K, trace_cap=K, want_state=True)
    assert ref.pivots == K
    with spx.Context(m=m, n=n, seed=0, eps=1e-7, trace=K, **kw) as ctx:
        if not kw:
            assert ctx.config()["window"] == 64  # the bench's default representation
        st, piv = ctx.iterate(K)
        assert st == spx.SolveStatus.MaxIter and piv == K
        tp, tq = ctx.trace()
        s = ctx.state(binv=True)
    assert list(tp) == list(ref.trace_p) and list(tq) == list(ref.trace_q)
    assert list(s["b_ixs"]) == list(ref.b_ixs)
    assert _rel(s["x_b"], ref.x_b) <= REL
    assert _rel(s["y"], ref.y) <= REL
    assert _rel(s["binv"], ref.binv) <= REL


# C3 solved to optimality (18,291 pivots) against the committed HiGHS optimum and
# the oracle's whole pivot sequence
@pytest.mark.parametrize("kw", [dict(), dict(window=-1), dict(tableau=True)],
                         ids=["default-window64", "explicit", "tableau"])
def test_c3_golden_full_solve(spx, c3_golden, kw):
    g = c3_golden
    cap = g["oracle_pivots"] + 64
    with spx.Context(m=4096, n=16384, seed=0, eps=g["eps"], trace=cap, **kw) as ctx:
        r = ctx.solve()
        tp, tq = ctx.trace()
    assert r.status == spx.SolveStatus.OptimumFound
    assert abs(r.z - g["highs_z"]) <= REL * abs(g["highs_z"])
    assert sorted(int(j) for j in r.b_ixs) == g["highs_basis"]
    assert r.pivots == g["oracle_pivots"]
    assert list(tp) == g["oracle_trace_p"] and list(tq) == g["oracle_trace_q"]


# C4 (m=4096, n=131072): column-sharded pricing over G in-process shards with
# B^-1 replicated and the default 64-window (the north-star partitioning,
# SURVEY.md §8e), bit for bit against one rank
@pytest.mark.parametrize("G", [2, 4, 8])
def test_c4_shard_group_matches_single_rank(spx, G):
    m, n, k = 4096, 131072, 20
    with spx.Context(m=m, n=n, seed=0, window=64, trace=k) as ref:
        rst, rpiv = ref.iterate(k)
        rp, rq = ref.trace()
        rs = ref.state()
        rz = ref.objective()
    assert rpiv == k
    ctxs = [spx.Context(m=m, n=n, seed=0, rank=g, nranks=G, window=64, trace=k) for g in range(G)]
    try:
        st, piv = spx.group_iterate(ctxs, k)
        assert st == rst and piv == rpiv
        for c in ctxs:
            p, q = c.trace()
            assert np.array_equal(p, rp) and np.array_equal(q, rq)
        for c in ctxs:
            s = c.state()
            assert np.array_equal(s["b_ixs"], rs["b_ixs"])
            assert np.array_equal(s["x_b"], rs["x_b"])
            assert np.array_equal(s["y"], rs["y"])
            assert c.objective() == rz
    finally:
        for c in ctxs:
            c.close()


def test_trace_requires_cap(spx):
    with spx.Context(m=8, n=16, seed=1) as ctx:
        ctx.iterate(2)
        with pytest.raises(spx.SimplexError):
            ctx.trace()

"""GPU: Devex and steepest-edge pricing (README.md:16-17) on column-shard
groups -- the north-star partitioning (pricing sharded by
columns, B^-1 replicated, a MINLOC merge of one record per rank) with the
weighted pricing rules.

Each rank keeps the weights of its own columns; the winning rank's record
carries the entering column's reduced cost and weight (Params::pr_stride,
dvx_payload), and steepest edge's B_w^T alpha is formed on every rank from
the replicated B^-1.  A column's key is computed by the same arithmetic on
whichever rank owns it and the merge is a total order, so a group takes the
pivots of one rank with the same bits: the trace, the basis, x_b, y and z
are compared for equality, through several folds, to optimality.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

DEVEX, STEEP = 1, 2


def _single(spx, kw, k):
    with spx.Context(trace=k, **kw) as ref:
        st, piv = ref.iterate(k)
        p, q = ref.trace()
        return st, piv, p, q, ref.state(), ref.objective()


def _group(spx, G, kw, k):
    ctxs = [spx.Context(rank=g, nranks=G, trace=k, **kw) for g in range(G)]
    try:
        st, piv = spx.group_iterate(ctxs, k)
        return st, piv, [c.trace() for c in ctxs], [c.state() for c in ctxs], [c.objective() for c in ctxs]
    finally:
        for c in ctxs:
            c.close()


def _check(spx, G, kw, k, want_optimum):
    rst, rpiv, rp, rq, rs, rz = _single(spx, kw, k)
    if want_optimum:
        assert rst == spx.SolveStatus.OptimumFound
    st, piv, traces, states, zs = _group(spx, G, kw, k)
    assert st == rst and piv == rpiv
    for p, q in traces:
        assert np.array_equal(p, rp) and np.array_equal(q, rq)
    for s in states:
        for key in ("b_ixs", "x_b", "y"):
            assert np.array_equal(s[key], rs[key]), key
    assert all(z == rz for z in zs)
    return rpiv


@pytest.mark.parametrize("G", [2, 4])
@pytest.mark.parametrize("pricing", [DEVEX, STEEP], ids=["devex", "steepest"])
def test_weighted_pricing_group_to_optimum(spx, G, pricing):
    """m=300, n=1200 (window 32: a fold every 31 pivots) solved to optimality."""
    kw = dict(m=300, n=1200, seed=8, window=32, eps=1e-7, pricing=pricing)
    piv = _check(spx, G, kw, 4096, want_optimum=True)
    assert piv > 62  # (more than two folds)


def test_steepest_c3_group8_first_130(spx):
    """The headline shape (C3, m=4096 n=16384, window 64) as 8 column shards
    with steepest edge: the first 130 pivots (two folds) as one rank."""
    kw = dict(m=4096, n=16384, seed=0, window=64, pricing=STEEP)
    assert _check(spx, 8, kw, 130, want_optimum=False) == 130


def test_weighted_pricing_group_refuses_split_tail(spx):
    """The split ratio-test tail (and so Harris) is not wired for a group's
    weighted pricing: refused at creation, not run."""
    with pytest.raises(spx.SimplexError):
        spx.Context(m=64, n=256, seed=0, window=16, pricing=STEEP, rank=0, nranks=2, ratio_test=2)

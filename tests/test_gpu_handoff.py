"""GPU: the cross-workgroup hand-offs of the pass kernels give the same bits
in every form.  k_price's partials reach the entering-column merge either in
k_update (deferred, the default with one rank and the window), in k_price's
own last workgroup by tagged words (the default where k_price merges: several
ranks, explicit B^-1 at m > 2048, SPX_FLAG_PRICE_TAIL), or by drained stores +
a last-arrival count (SPX_FLAG_COUNTED_TAIL); k_update's ratio-test partials
likewise (tagged or counted).  Pivot traces and state must be identical."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

FORMS = [dict(), dict(price_tail=True), dict(counted_tail=True), dict(price_tail=True, counted_tail=True)]


def _run(spx, m, n, k, **kw):
    with spx.Context(m=m, n=n, seed=3, trace=k, **kw) as ctx:
        st, piv = ctx.iterate(k)
        tp, tq = ctx.trace()
        s = ctx.state()
    return st, piv, np.asarray(tp), np.asarray(tq), s


@pytest.mark.parametrize("window", [64, -1])
def test_handoff_forms_bit_identical(spx, window):
    m, n, k = 2304, 9000, 150  # explicit at m > 2048 merges in k_price
    ref = _run(spx, m, n, k, window=window)
    assert ref[1] == k
    for kw in FORMS[1:]:
        got = _run(spx, m, n, k, window=window, **kw)
        assert got[0] == ref[0] and got[1] == ref[1], kw
        assert np.array_equal(got[2], ref[2]) and np.array_equal(got[3], ref[3]), kw
        for key in ("b_ixs", "x_b", "y"):
            assert np.array_equal(got[4][key], ref[4][key]), (kw, key)


@pytest.mark.parametrize("counted", [False, True])
def test_handoff_shard_group_matches_single_rank(spx, counted):
    """Column shards (k_price merges its own partials, then the candidate
    exchange) against one rank, both hand-off forms."""
    m, n, k, G = 1024, 6000, 60, 3
    ref = _run(spx, m, n, k, window=64)
    ctxs = [spx.Context(m=m, n=n, seed=3, rank=g, nranks=G, window=64, trace=k, counted_tail=counted)
            for g in range(G)]
    try:
        st, piv = spx.group_iterate(ctxs, k)
        assert st == ref[0] and piv == ref[1]
        for c in ctxs:
            p, q = c.trace()
            assert np.array_equal(p, ref[2]) and np.array_equal(q, ref[3])
            s = c.state()
            for key in ("b_ixs", "x_b", "y"):
                assert np.array_equal(s[key], ref[4][key]), key
    finally:
        for c in ctxs:
            c.close()

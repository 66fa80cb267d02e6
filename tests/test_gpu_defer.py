"""The deferred ratio-test tail (Params::defer_tail, TailRec in spx_device.h):
the compact FTRAN pass publishes its workgroup partials and ends; the next
pricing pass reduces them in every workgroup and its workgroup 0 applies the
bookkeeping, and k_apply_tail applies a pending tail before a fold and at
the end of every iterate call.  The reduction is the FTRAN tail's own (512
threads, the same order), so the pivots and every state word must be the
bits of the tail run inside the FTRAN pass (SPX_DEFER_TAIL=0).

It is active for compact window passes with 512-thread workgroups, i.e. at
m >= 2048 (smaller m gives the update pass 256-thread workgroups), so these
cases run at m = 2048.  Reference: the pivot tail v4:317-342.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _ctx(spx, defer, *args, **kw):
    old = os.environ.get("SPX_DEFER_TAIL")
    os.environ["SPX_DEFER_TAIL"] = "1" if defer else "0"
    try:
        return spx.Context(*args, **kw)
    finally:
        if old is None:
            del os.environ["SPX_DEFER_TAIL"]
        else:
            os.environ["SPX_DEFER_TAIL"] = old


def _run_chunks(ctx, chunks):
    for k in chunks:
        ctx.iterate(k)
    st = ctx.state(binv=True)
    tp, tq = ctx.trace()
    return st, tp, tq, ctx.objective()


# mixed chunk sizes: eager lead passes, whole captured windows, a remainder,
# single passes (a pending tail applied at every call's end)
CHUNKS = [1, 5, 63, 70, 7, 1, 130]


@pytest.mark.parametrize("graph_batch,price_block", [(0, 0), (-1, 0), (0, 256), (-1, 256)])
def test_deferred_tail_same_bits(spx, graph_batch, price_block):
    """price_block 256: each pricing thread holds two of the 512-thread
    shape's partials (reduce_partial_pair), so the deferred tail keeps the
    in-pass tail's bits with 256-thread pricing workgroups too."""
    m, n, seed = 2048, 6144, 3
    kw = dict(m=m, n=n, seed=seed, trace=sum(CHUNKS))
    if graph_batch < 0:
        kw["graph_batch"] = -1  # eager passes only
    if price_block:
        kw["price_block"] = price_block
    with _ctx(spx, True, **kw) as a, _ctx(spx, False, **kw) as b:
        assert a.config()["defer_tail"] == 1, a.config()
        assert b.config()["defer_tail"] == 0, b.config()
        sa, pa, qa, za = _run_chunks(a, CHUNKS)
        sb, pb, qb, zb = _run_chunks(b, CHUNKS)
    assert np.array_equal(pa, pb) and np.array_equal(qa, qb)
    for key in ("b_ixs", "x_b", "y", "binv"):
        assert np.array_equal(sa[key], sb[key]), key
    assert za == zb


def _unbounded_lp(m, k_struct, seed):
    """max c x, A x <= b, x >= 0 with slack identity; one structural column
    is non-positive with a positive cost, so the LP is unbounded, but its
    small cost lets other columns enter first."""
    rng = np.random.default_rng(seed)
    n = k_struct + m
    A = np.zeros((n, m))
    A[:k_struct] = rng.uniform(0.0, 1.0, size=(k_struct, m))
    A[k_struct // 2] = -rng.uniform(0.5, 1.0, size=m)
    A[k_struct:] = np.eye(m)
    b = rng.uniform(1.0, 2.0, size=m)
    c = np.zeros(n)
    c[:k_struct] = rng.uniform(0.5, 1.0, size=k_struct)
    c[k_struct // 2] = 0.05
    return A, b, c


def test_deferred_tail_unbounded(spx):
    """The Unbounded exit found by a pricing pass's deferred reduction (or by
    k_apply_tail) is the one the FTRAN tail reports, at the same pivot."""
    A, b, c = _unbounded_lp(2048, 1024, 5)
    res = []
    for defer in (True, False):
        with _ctx(spx, defer, A, b, c, trace=20000) as ctx:
            assert ctx.config()["defer_tail"] == (1 if defer else 0)
            r = ctx.solve()
            tp, tq = ctx.trace()
            res.append((r.status, r.pivots, tp, tq))
    (sa, na, pa, qa), (sb, nb, pb, qb) = res
    assert sa == spx.SolveStatus.Unbounded and sb == sa
    assert na == nb and na > 0
    assert np.array_equal(pa, pb) and np.array_equal(qa, qb)


def test_deferred_tail_limit_and_resume(spx):
    """Passes stopped by the iteration limit leave no tail pending: k + k'
    pivots in two calls give the bits of one call."""
    m, n, seed = 2048, 4096, 8
    with _ctx(spx, True, m=m, n=n, seed=seed) as a, _ctx(spx, True, m=m, n=n, seed=seed) as b:
        a.iterate(200)
        b.iterate(77)
        b.iterate(123)
        sa, sb = a.state(), b.state()
    for key in ("b_ixs", "x_b", "y"):
        assert np.array_equal(sa[key], sb[key]), key


def test_deferred_tail_price_block_256_same_bits_as_512(spx):
    """Pricing geometry does not enter the bits: each column's dot is one
    wave's, the entering argmin breaks ties by index, and the deferred
    ratio-test tail reduces the same 512-thread shape with 256 or 512
    threads.  Covers C3-shaped m = 4096 over two folds."""
    kw = dict(m=4096, n=16384, seed=0, trace=140)
    with _ctx(spx, True, price_block=256, **kw) as a, _ctx(spx, True, **kw) as b:
        assert a.config()["defer_tail"] == 1 and b.config()["defer_tail"] == 1
        assert a.config()["price_block"] == 256 and b.config()["price_block"] == 512
        sa, pa, qa, za = _run_chunks(a, [3, 137])
        sb, pb, qb, zb = _run_chunks(b, [3, 137])
    assert np.array_equal(pa, pb) and np.array_equal(qa, qb)
    for key in ("b_ixs", "x_b", "y", "binv"):
        assert np.array_equal(sa[key], sb[key]), key
    assert za == zb


@pytest.mark.parametrize("G", [2, 3])
def test_deferred_tail_shard_group(spx, G):
    """Column-sharded in-process groups (replicated B_w, pricing tail in the
    launch for the exchange) with the deferred ratio-test tail: identical to
    the in-pass tail's group and to one rank, through two folds and mixed
    iterate chunks."""
    m, n, seed = 2048, 6144, 3
    kw = dict(m=m, n=n, seed=seed, trace=sum(CHUNKS))
    with _ctx(spx, True, **kw) as ref:
        rs, rp, rq, rz = _run_chunks(ref, CHUNKS)
    for defer in (True, False):
        ctxs = [_ctx(spx, defer, rank=g, nranks=G, **kw) for g in range(G)]
        try:
            assert all(c.config()["defer_tail"] == (1 if defer else 0) for c in ctxs)
            for k in CHUNKS:
                spx.group_iterate(ctxs, k)
            for c in ctxs:
                s = c.state(binv=True)
                p, q = c.trace()
                assert np.array_equal(p, rp) and np.array_equal(q, rq), defer
                for key in ("b_ixs", "x_b", "y", "binv"):
                    assert np.array_equal(s[key], rs[key]), (defer, key)
                assert c.objective() == rz
        finally:
            for c in ctxs:
                c.close()

"""GPU: non-basic slack columns priced as unit vectors (Params::slack_unit,
A[:, n-m:] = I) against the same columns streamed densely
(SPX_DENSE_SLACKS=1): the same bits in every representation and dispatch,
through whole solves in which most slacks leave the basis."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _run(spx, dense, k, **kw):
    old = os.environ.get("SPX_DENSE_SLACKS")
    os.environ["SPX_DENSE_SLACKS"] = "1" if dense else "0"
    try:
        with spx.Context(**kw) as ctx:
            st, piv = ctx.iterate(k)
            s = ctx.state(binv=True)
            e = ctx.reduced_costs()
            r = ctx.solve()
            return piv, s, e, r
    finally:
        if old is None:
            del os.environ["SPX_DENSE_SLACKS"]
        else:
            os.environ["SPX_DENSE_SLACKS"] = old


@pytest.mark.parametrize("window,graph_batch,persist", [(-1, 16, None), (16, 16, False), (64, -1, False),
                                                        (64, 0, None)])
def test_unit_slacks_match_dense_stream(spx, window, graph_batch, persist):
    kw = dict(m=300, n=1200, seed=5, window=window, graph_batch=graph_batch, persist=persist)
    a = _run(spx, False, 200, **kw)
    b = _run(spx, True, 200, **kw)
    assert a[0] == b[0] == 200
    for key in ("b_ixs", "x_b", "y", "binv"):
        assert np.array_equal(a[1][key], b[1][key]), key
    assert np.array_equal(a[2], b[2])
    assert a[3].pivots == b[3].pivots and a[3].z == b[3].z and a[3].status == b[3].status


def test_unit_slacks_host_lp_matches_oracle(spx, oracle):
    """An LP given from the host (spx_create checks the slack block) solves to
    the oracle's pivot count and optimum, with slacks priced as unit columns."""
    m, n, seed = 256, 1024, 11
    A, b, c = oracle.generate(m, n, seed)
    o = oracle.solve(A, b, c, eps=1e-7)
    with spx.Context(A, b, c, window=16) as ctx:  # A: (n, m), column j of A per row
        r = ctx.solve()
    assert r.status == spx.SolveStatus.OptimumFound and r.pivots == o.pivots
    assert abs(r.z - o.z) <= 1e-9 * abs(o.z)

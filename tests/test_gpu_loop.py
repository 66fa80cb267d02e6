"""GPU: the persistent loop kernel (k_loop, csrc/spx_loop.hip; SPX_FLAG_PERSIST)
against the oracle and the two-kernel pass.  Same tolerances as
test_gpu_parity.py: identical pivot paths, state within 1e-9 of the oracle,
within 1e-12 of the two-kernel pass (the ratio test's c_B.alpha sum is grouped
by the launch geometry)."""
import numpy as np
import pytest

from lpgen import degenerate_lp, highs_opt

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    return float(np.max(np.abs(a - b)) / max(1.0, float(np.max(np.abs(b)))))


@pytest.mark.parametrize("window", [8, 64])
@pytest.mark.parametrize("m,n,seed", [(64, 256, 0), (300, 900, 3)])
def test_loop_solves_to_oracle_optimum(spx, oracle, window, m, n, seed):
    A, b, c = oracle.generate(m, n, seed)
    ref = oracle.solve(A, b, c, eps=1e-7)
    with spx.Context(A, b, c, eps=1e-7, window=window, persist=True) as ctx:
        assert ctx.config()["persistent"] == 1
        r = ctx.solve()
    assert r.status == spx.SolveStatus.OptimumFound and r.pivots == ref.pivots
    assert list(r.b_ixs) == list(ref.b_ixs)
    assert abs(r.z - ref.z) <= 1e-9 * abs(ref.z)
    assert _rel(r.x_b, ref.x_b) <= 1e-9


def test_loop_devex_and_guarded(spx, oracle):
    A, b, c = oracle.generate(257, 771, 2)
    ref = oracle.solve(A, b, c, eps=1e-7, pricing=oracle.PRICING_DEVEX)
    with spx.Context(A, b, c, eps=1e-7, pricing=spx.PRICING_DEVEX, persist=True) as ctx:
        assert ctx.config()["persistent"] == 1
        r = ctx.solve()
    assert r.pivots == ref.pivots and list(r.b_ixs) == list(ref.b_ixs)
    A, b, c = degenerate_lp(300, 900, 4)
    z_star = highs_opt(A, b, c)
    with spx.Context(A, b, c, eps=1e-7, window=16, ratio_test=1, persist=True) as ctx:
        r = ctx.solve(max_iter=20000)
    assert r.status == spx.SolveStatus.OptimumFound and abs(r.z - z_star) <= 1e-9 * abs(z_star)


def test_loop_unbounded(spx, oracle):
    m, n = 3, 6
    A = np.zeros((n, m))
    A[0] = [-1.0, 0.0, -2.0]
    A[1] = [1.0, 1.0, 1.0]
    A[2] = [2.0, 0.5, 1.0]
    A[3:] = np.eye(m)
    b = np.array([4.0, 3.0, 5.0])
    c = np.array([1.0, 0.5, 0.25, 0, 0, 0])
    o = oracle.solve(A, b, c)
    with spx.Context(A, b, c, window=8, persist=True) as ctx:
        r = ctx.solve()
    assert r.status == spx.SolveStatus.Unbounded and r.pivots == o.pivots


def test_loop_mixed_with_two_kernel_steps(spx, oracle):
    """Step-wise passes (spx_price / spx_pivot, the two-kernel path),
    reinversion and persistent launches share one device state."""
    m, n, seed = 200, 800, 5
    A, b, c = oracle.generate(m, n, seed)
    ref = oracle.solve(A, b, c, eps=1e-7, trace_cap=2000)
    with spx.Context(A, b, c, eps=1e-7, window=32, persist=True) as ctx:
        ctx.iterate(40)
        for k in range(40, 45):
            p, e, opt = ctx.price()
            assert p == ref.trace_p[k]
            q, st = ctx.pivot()
            assert q == ref.trace_q[k]
        ctx.reinvert()
        ctx.iterate(50)
        r = ctx.solve()
    assert r.pivots == ref.pivots and abs(r.z - ref.z) <= 1e-9 * abs(ref.z)


def test_loop_refactor_and_timing(spx, oracle):
    A, b, c = oracle.generate(300, 900, 1)
    ref = oracle.solve(A, b, c, eps=1e-7, refactor_every=50)
    with spx.Context(A, b, c, eps=1e-7, window=64, refactor_every=50, persist=True, timing=True) as ctx:
        r = ctx.solve()
        lt = ctx.loop_times()
    assert r.pivots == ref.pivots and list(r.b_ixs) == list(ref.b_ixs)
    assert lt["loop_passes"] >= r.pivots and lt["loop_ms"] > 0
    assert lt["clock_passes"] > 0 and lt["price_us"] > 0 and lt["ftran_us"] > 0


def test_loop_opt_in_only(spx):
    """Two-kernel passes are the default at every size, so a single GPU runs
    the dispatch that N ranks run (the persistent loop is single-rank); the
    loop is opt-in.  Both forms read only B_w's non-unit columns (the compact
    operand: none yet at the slack basis)."""
    with spx.Context(m=1000, n=3000, seed=0, window=64) as ctx:
        assert ctx.config()["persistent"] == 0 and ctx.ftran_cols() == 0
    with spx.Context(m=12000, n=13000, seed=0, window=64) as ctx:
        assert ctx.config()["persistent"] == 0 and ctx.ftran_cols() == 0
        assert ctx.config()["price_block"] == 512
    with spx.Context(m=12000, n=13000, seed=0, window=64, persist=True) as ctx:
        assert ctx.config()["persistent"] == 1 and ctx.ftran_cols() == 0


@pytest.mark.parametrize("tableau", [False, True], ids=["k_loop", "k_tab_loop"])
def test_loop_not_coresident_falls_back(spx, oracle, monkeypatch, tableau):
    """A persistent launch whose grid is not all resident (SPX_LOOP_OVERSUB=1
    launches 4,096 workgroups more than the co-resident grid) must not hang in a grid barrier:
    the entry check (spx_grid.h grid_arrive) sends every workgroup home
    within 2 ms without touching the state, and the context makes those
    pivots as two-kernel passes -- the oracle's pivots and optimum."""
    m, n, seed = 300, 900, 3
    A, b, c = oracle.generate(m, n, seed)
    ref = oracle.solve(A, b, c, eps=1e-7, trace_cap=4096)
    monkeypatch.setenv("SPX_LOOP_OVERSUB", "1")
    with spx.Context(A, b, c, eps=1e-7, window=16, persist=True, tableau=tableau, trace=4096) as ctx:
        assert ctx.config()["persistent"] == 1
        st, piv = ctx.iterate(50)
        assert piv == 50
        ds = ctx.dispatch_stats()
        assert ds["persist_fallbacks"] >= 1 and ctx.config()["persistent"] == 0
        r = ctx.solve()
        tp, tq = ctx.trace()
    assert r.status == spx.SolveStatus.OptimumFound and r.pivots == ref.pivots
    assert list(tp) == list(ref.trace_p) and list(tq) == list(ref.trace_q)
    assert abs(r.z - ref.z) <= 1e-9 * abs(ref.z)


@pytest.mark.parametrize("tableau", [False, True], ids=["k_loop", "k_tab_loop"])
def test_loop_first_launch_not_coresident_mid_window(spx, oracle, monkeypatch, tableau):
    """only the FIRST persistent launch of a call is not resident
    (SPX_LOOP_OVERSUB=2), and the call starts mid-window.  The later launches
    of that call would find a resident grid; the failure is sticky
    (spx_grid.h grid_arrive reads LoopState::nores), so they leave at entry too
    instead of running from a window the host already counted as advanced,
    and the fallback makes every pivot of the call -- the oracle's pivots."""
    m, n, seed = 300, 900, 3
    A, b, c = oracle.generate(m, n, seed)
    ref = oracle.solve(A, b, c, eps=1e-7, trace_cap=4096)
    with spx.Context(A, b, c, eps=1e-7, window=16, persist=True, tableau=tableau, trace=4096) as ctx:
        assert ctx.config()["persistent"] == 1
        st, piv = ctx.iterate(6)  # resident: the window is now mid-way
        assert piv == 6 and ctx.dispatch_stats()["persist_fallbacks"] == 0
        monkeypatch.setenv("SPX_LOOP_OVERSUB", "2")
        st, piv = ctx.iterate(60)  # 4+ launches; only the first is oversubscribed
        assert piv == 66
        assert ctx.dispatch_stats()["persist_fallbacks"] == 1
        r = ctx.solve()
        tp, tq = ctx.trace()
    assert r.status == spx.SolveStatus.OptimumFound and r.pivots == ref.pivots
    assert list(tp) == list(ref.trace_p) and list(tq) == list(ref.trace_q)
    assert abs(r.z - ref.z) <= 1e-9 * abs(ref.z)

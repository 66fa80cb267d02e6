"""GPU: the large-size code paths (chunked tail, big LDS y, global-y pricing)
and the BASELINE configurations C4/C5 through size-independent invariants.

Tolerances as in test_gpu_parity.py; at C4/C5 the oracle cannot run a window
in test time, so the checks are B^-1 B = I on sampled basis columns (columns
regenerated on the host from the seeded generator), x_b = B^-1 b, z = c_B.x_b,
x_b >= 0 and e_j ~ 0 on basic columns.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    return float(np.max(np.abs(a - b)) / max(1.0, float(np.max(np.abs(b)))))


def test_every_geometry_consistent(spx):
    """LDS-y and global-y pricing and every pricing block give the same bits;
    every update geometry (its c_B.alpha sum order) the same pivots and values
    within 1e-12."""
    m, n, seed, k = 1100, 3300, 4, 150
    runs = []
    for kw in [dict(), dict(global_y=True), dict(price_block=256, global_y=True), dict(price_block=1024),
               dict(update_block=256), dict(update_block=512, update_rows=2), dict(update_block=1024, update_rows=4)]:
        with spx.Context(m=m, n=n, seed=seed, **kw) as ctx:
            st, piv = ctx.iterate(k)
            s = ctx.state(binv=True)
            s["z"] = ctx.objective()
            runs.append((kw, piv, s))
    kw0, piv0, s0 = runs[0]
    assert piv0 == k
    for kw, piv, s in runs[1:]:
        assert piv == piv0, kw
        assert np.array_equal(s["b_ixs"], s0["b_ixs"]), kw
        if any(key.startswith("update_") for key in kw):
            for key in ("x_b", "y", "binv"):
                assert _rel(s[key], s0[key]) <= 1e-12, (kw, key)
            assert abs(s["z"] - s0["z"]) <= 1e-12 * abs(s0["z"]), kw
        else:
            for key in ("x_b", "y", "binv"):
                assert np.array_equal(s[key], s0[key]), (kw, key)
            assert s["z"] == s0["z"], kw


def test_mid_size_against_oracle(spx, oracle):
    """m=6000 (chunked tail, L=6016) against the CPU restatement."""
    m, n, seed, k = 6000, 9000, 2, 40
    A, b, c = oracle.generate(m, n, seed)
    ref = oracle.solve(A, b, c, max_iter=k, want_state=True, trace_cap=k)
    with spx.Context(A, b, c) as ctx:
        ps, qs = [], []
        for _ in range(k):
            p, e, opt = ctx.price()
            q, st = ctx.pivot()
            ps.append(p)
            qs.append(q)
        s = ctx.state(binv=True)
    assert ps == list(ref.trace_p) and qs == list(ref.trace_q)
    assert _rel(s["x_b"], ref.x_b) <= 1e-9
    assert _rel(s["y"], ref.y) <= 1e-9
    assert _rel(s["binv"], ref.binv) <= 1e-9


def _check_invariants(spx, oracle, m, n, seed, k, ncols=24):
    with spx.Context(m=m, n=n, seed=seed) as ctx:
        st, piv = ctx.iterate(k)
        assert st == spx.SolveStatus.MaxIter and piv == k
        s = ctx.state(binv=True)
        z = ctx.objective()
        e = ctx.reduced_costs()
    b = (n - m) / 4.0 * (1.0 + oracle.uniform_np(seed, 2, np.arange(m, dtype=np.uint64)))
    c = np.zeros(n)
    c[: n - m] = oracle.uniform_np(seed, 3, np.arange(n - m, dtype=np.uint64))
    rows = np.linspace(0, m - 1, ncols).astype(np.int64)
    Bcols = np.stack([oracle.column_np(m, n, seed, int(s["b_ixs"][i])) for i in rows], axis=1)
    I = s["binv"] @ Bcols
    E = np.zeros_like(I)
    E[rows, np.arange(len(rows))] = 1.0
    assert np.max(np.abs(I - E)) < 1e-9
    assert _rel(s["binv"] @ b, s["x_b"]) < 1e-10
    assert abs(z - float(c[s["b_ixs"]] @ s["x_b"])) <= 1e-10 * abs(z)
    assert np.all(s["x_b"] > -1e-9)
    assert np.max(np.abs(e[s["b_ixs"]])) < 1e-9  # basic columns price to zero
    assert len(set(s["b_ixs"].tolist())) == m


def test_c4_invariants(spx, oracle):
    """C4 (m=4096, n=131072): 127k priced columns per iteration."""
    _check_invariants(spx, oracle, 4096, 131072, 0, 40)


def test_c5_invariants(spx, oracle):
    """C5 (m=16384, n=65536): y in 128 KiB of LDS, B^-1 2.1 GB x 2."""
    _check_invariants(spx, oracle, 16384, 65536, 0, 30, ncols=16)


def test_global_y_large_m(spx, oracle):
    """m=20000: y no longer fits LDS, pricing reads it from global memory."""
    _check_invariants(spx, oracle, 20000, 21000, 1, 12, ncols=8)


def test_dynamic_pricing_tail_same_bits(spx, monkeypatch):
    """Eta-window pricing with the base row read from L2 (k_price WM 2, m large
    enough that y_w and the base row do not both fit LDS: the C5 shape) hands
    out its last columns by ticket in whatever order the waves finish
    (Params::price_dyn).  Every column's terms and the argmin's total order do
    not depend on which wave prices it, so the trace, the state and B^-1 are
    those of the static grid stride (SPX_PRICE_DYN=0) bit for bit, through two
    folds.  Then the stepped API prices twice at one iteration count (the
    ticket counter of that pass parity must start from zero again) and
    pivots."""
    m, n, seed, k = 10000, 20000, 3, 130
    outs = []
    for dyn in ("1", "0"):
        monkeypatch.setenv("SPX_PRICE_DYN", dyn)
        with spx.Context(m=m, n=n, seed=seed, trace=k) as ctx:
            cfg = ctx.config()
            assert cfg["window"] == 64 and cfg["price_lds"] == 1  # y_w in LDS, the base row from L2
            st, piv = ctx.iterate(k)
            tp, tq = ctx.trace()
            s = ctx.state()
            p1, p2 = ctx.price(), ctx.price()
            assert p1 == p2
            q = ctx.pivot()
            outs.append((piv, tp, tq, s, ctx.objective(), p1, q))
    (pa, tpa, tqa, sa, za, p1a, qa), (pb, tpb, tqb, sb, zb, p1b, qb) = outs
    assert pa == pb == k
    assert p1a == p1b and qa == qb
    assert np.array_equal(tpa, tpb) and np.array_equal(tqa, tqb)
    for key in ("b_ixs", "x_b", "y"):
        assert np.array_equal(sa[key], sb[key]), key
    assert za == zb


def test_dynamic_pricing_tail_wm1_same_bits(spx, monkeypatch):
    """The ticketed tail with the base row in LDS (k_price WM 1), where a wave
    prices at least 16 columns (the C4 shape; m=2048, n=40960: 19 per wave):
    the same trace, state and objective bits as the static grid stride
    (SPX_PRICE_DYN=0), through two folds."""
    m, n, seed, k = 2048, 40960, 4, 130
    outs = []
    for dyn in ("1", "0"):
        monkeypatch.setenv("SPX_PRICE_DYN", dyn)
        with spx.Context(m=m, n=n, seed=seed, trace=k) as ctx:
            cfg = ctx.config()
            assert cfg["window"] == 64 and cfg["price_lds"] == 2  # y_w and the base row in LDS
            st, piv = ctx.iterate(k)
            tp, tq = ctx.trace()
            outs.append((piv, tp, tq, ctx.state(), ctx.objective()))
    (pa, tpa, tqa, sa, za), (pb, tpb, tqb, sb, zb) = outs
    assert pa == pb == k
    assert np.array_equal(tpa, tpb) and np.array_equal(tqa, tqb)
    for key in ("b_ixs", "x_b", "y"):
        assert np.array_equal(sa[key], sb[key]), key
    assert za == zb


@pytest.mark.parametrize("grid", [1, 2, 3])
def test_dynamic_pricing_tail_small_grids(spx, monkeypatch, grid):
    """The ticketed tail with 1-3 pricing workgroups (8-24 waves; the
    counters capped to the waves that draw from them, none left without
    one): the static order's bits (m=300, n=1200, window 16, 130 pivots)."""
    m, n, seed, k = 300, 1200, 7, 130
    outs = []
    for dyn in ("2", "0"):
        monkeypatch.setenv("SPX_PRICE_DYN", dyn)
        with spx.Context(m=m, n=n, seed=seed, window=16, persist=False, price_grid=grid, trace=k) as ctx:
            st, piv = ctx.iterate(k)
            tp, tq = ctx.trace()
            outs.append((piv, tp, tq, ctx.state()))
    (pa, tpa, tqa, sa), (pb, tpb, tqb, sb) = outs
    assert pa == pb == k
    assert np.array_equal(tpa, tpb) and np.array_equal(tqa, tqb)
    for key in ("b_ixs", "x_b", "y"):
        assert np.array_equal(sa[key], sb[key]), key


def test_ticketed_tail_unpriced_slots_fail_loudly(spx, monkeypatch):
    """the ticketed tail's coverage is checked on the
    device, not only by the host's cap.  A deliberately broken geometry -- 16
    counters for one 8-wave pricing workgroup, the cap skipped
    (SPX_TK_UNSAFE=1), so counters 8..15 have no wave drawing from them and
    their slots go unpriced -- must stop the solve with an error
    (SPX_ERR_STATE via DevState::uncovered or the host's last-pass check),
    not return wrong pivots; the capped geometry on the same LP runs clean."""
    m, n, seed = 300, 1200, 7
    monkeypatch.setenv("SPX_PRICE_DYN", "2")
    monkeypatch.setenv("SPX_TK_SHARDS", "16")
    with spx.Context(m=m, n=n, seed=seed, window=16, persist=False, price_grid=1) as ctx:
        st, piv = ctx.iterate(40)  # (capped: 8 counters, every one drawn from)
        assert piv == 40
    monkeypatch.setenv("SPX_TK_UNSAFE", "1")
    with spx.Context(m=m, n=n, seed=seed, window=16, persist=False, price_grid=1) as ctx:
        with pytest.raises(spx.SimplexError, match="unpriced"):
            ctx.iterate(40)
        with pytest.raises(spx.SimplexError, match="unpriced"):  # sticky until a reset
            ctx.iterate(1)
        monkeypatch.delenv("SPX_TK_UNSAFE")
        ctx.reset()
        ctx.iterate(0)  # (the flag is cleared; the context's counters are still 16)

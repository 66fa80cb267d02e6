"""GPU: the window tableau (SPX_FLAG_TABLEAU) against the CPU
oracle (oracle/simplex_oracle.c, the v4 loop with B^-1 rewritten every pivot,
v4:268-368) and against the eta window it extends.

The tableau computes the same quantities as the eta window — reduced costs
e_j = y.A_j - c_j (v4:288-290), alpha = B^-1 A_p (v4:306-308) — from T_w =
B_w A and dw = y_w A - c kept in HBM instead of from the A and B_w streams,
so it reassociates the same sums.  Bar, as for the window
(test_gpu_window.py): the oracle's pivot path exactly, x_b / y / B^-1 within
1e-9 relative, the HiGHS optimum within 1e-9 with the same basis set;
graph replay and eager launches bit-identical.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

WINDOWS = [8, 16, 32, 64]


def _rel(a, b):
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    return float(np.max(np.abs(a - b)) / max(1.0, float(np.max(np.abs(b)))))


@pytest.mark.parametrize("persist", [False, True])
@pytest.mark.parametrize("window", WINDOWS)
@pytest.mark.parametrize("m,n,seed,k", [(257, 771, 2, 150), (1000, 3000, 3, 140), (64, 200, 5, 90)])
def test_tableau_state_matches_oracle(spx, oracle, window, m, n, seed, k, persist):
    """Two-kernel passes (k_price WM 3 + k_update) and the persistent tableau
    loop (k_tab_loop) both follow the oracle."""
    A, b, c = oracle.generate(m, n, seed)
    ref = oracle.solve(A, b, c, max_iter=k, eps=1e-7, want_state=True, trace_cap=k)
    with spx.Context(A, b, c, eps=1e-7, window=window, tableau=True, persist=persist) as ctx:
        assert ctx.config()["tableau"] == 1 and ctx.config()["persistent"] == int(persist)
        st, piv = ctx.iterate(k)
        s = ctx.state(binv=True)
        e = ctx.reduced_costs()
        z = ctx.objective()
    assert piv == ref.pivots
    assert list(s["b_ixs"]) == list(ref.b_ixs)
    assert _rel(s["x_b"], ref.x_b) <= 1e-9
    assert _rel(s["y"], ref.y) <= 1e-9
    assert _rel(s["binv"], ref.binv) <= 1e-9
    assert _rel(e, oracle.price(A, c, s["y"])) <= 1e-12
    assert abs(z - ref.z) <= 1e-9 * abs(ref.z)


@pytest.mark.parametrize("window", [8, 64])
def test_tableau_step_api_trace(spx, oracle, window):
    """spx_price / spx_pivot one pass at a time: the oracle's (p, q) sequence."""
    m, n, seed, K = 100, 300, 1, 90
    A, b, c = oracle.generate(m, n, seed)
    ref = oracle.solve(A, b, c, eps=1e-7, trace_cap=K)
    with spx.Context(A, b, c, window=window, tableau=True) as ctx:
        ps, qs = [], []
        for _ in range(min(K, ref.pivots)):
            p, e, opt = ctx.price()
            assert not opt
            q, st = ctx.pivot()
            ps.append(p)
            qs.append(q)
    assert ps == list(ref.trace_p[: len(ps)]) and qs == list(ref.trace_q[: len(qs)])


def test_tableau_readback_mid_window_then_continue(spx, oracle):
    """A readback folds the window early (T_w and dw with it); the run goes on
    along the oracle's path."""
    m, n, seed = 300, 1200, 7
    A, b, c = oracle.generate(m, n, seed)
    ref = oracle.solve(A, b, c, max_iter=100, want_state=True)
    with spx.Context(A, b, c, window=16, tableau=True) as ctx:
        for k in (13, 1, 2, 40, 44):
            ctx.iterate(k)
            s = ctx.state(binv=True)
            ctx.reduced_costs()
    assert list(s["b_ixs"]) == list(ref.b_ixs)
    assert _rel(s["x_b"], ref.x_b) <= 1e-9
    assert _rel(s["y"], ref.y) <= 1e-9
    assert _rel(s["binv"], ref.binv) <= 1e-9


def test_tableau_graph_eager_bit_identical(spx):
    """Two-kernel passes: graph replay, eager launches and every pricing
    geometry give the same bits.  The persistent loop groups the ratio test's
    c_B.alpha sum by its own geometry: same pivots, values within 1e-12."""
    m, n, seed, k = 300, 1200, 7, 160
    runs = []
    for kw in (dict(), dict(graph_batch=-1), dict(graph_batch=5), dict(price_grid=3), dict(price_block=1024)):
        with spx.Context(m=m, n=n, seed=seed, window=32, tableau=True, persist=False, **kw) as ctx:
            assert ctx.config()["persistent"] == 0
            ctx.iterate(k)
            runs.append((kw, ctx.state(binv=True)))
    s0 = runs[0][1]
    for kw, s in runs[1:]:
        for key in ("b_ixs", "x_b", "y", "binv"):
            assert np.array_equal(s[key], s0[key]), (kw, key)
    with spx.Context(m=m, n=n, seed=seed, window=32, tableau=True) as ctx:
        assert ctx.config()["persistent"] == 1
        st, piv = ctx.iterate(k)
        s = ctx.state(binv=True)
    assert piv == k and np.array_equal(s["b_ixs"], s0["b_ixs"])
    for key in ("x_b", "y", "binv"):
        assert _rel(s[key], s0[key]) <= 1e-12, key


def test_tableau_matches_window(spx):
    m, n, seed, k = 1100, 3300, 4, 200
    out = {}
    for tab in (False, True):
        with spx.Context(m=m, n=n, seed=seed, window=32, tableau=tab, persist=False) as ctx:
            st, piv = ctx.iterate(k)
            out[tab] = (piv, ctx.state(binv=True), ctx.objective())
    (p0, s0, z0), (p1, s1, z1) = out[False], out[True]
    assert p0 == p1 == k
    assert np.array_equal(s0["b_ixs"], s1["b_ixs"])
    # B^-1 and x_b come from the same U/Wt/xw arithmetic; y from the same
    # fold; the tableau only changes how r_tau.A_j and alpha are summed
    for key in ("x_b", "y", "binv"):
        assert _rel(s1[key], s0[key]) <= 1e-10, key
    assert abs(z1 - z0) <= 1e-10 * abs(z0)


@pytest.mark.parametrize("case_i", [0, 3, 6, 9, 10])
def test_tableau_golden_optimum(spx, golden, case_i):
    case = golden["cases"][case_i]
    with spx.Context(m=case["m"], n=case["n"], seed=case["seed"], eps=golden["eps"], window=64,
                     tableau=True) as ctx:
        r = ctx.solve()
    assert r.status == spx.SolveStatus.OptimumFound
    assert abs(r.z - case["highs_z"]) <= 1e-9 * abs(case["highs_z"])
    assert sorted(int(j) for j in r.b_ixs) == case["highs_basis"]
    assert r.pivots == case["oracle_pivots"]


def test_tableau_sample(spx, oracle):
    """input/sample.txt (the reference's only known answer: z = 9, x0 = 1, x1 = 3)."""
    m, n, A, b, c = spx.read_lp("tests/golden/sample.txt")
    with spx.Context(A, b, c, window=8, tableau=True) as ctx:
        r = ctx.solve()
    assert r.status == spx.SolveStatus.OptimumFound and abs(r.z - 9.0) < 1e-12
    assert dict(zip((int(j) for j in r.b_ixs), r.x_b)) == pytest.approx({0: 1.0, 1: 3.0})


def test_tableau_unbounded(spx, oracle):
    m, n = 3, 6
    A = np.zeros((n, m))
    A[0] = [-1.0, 0.0, -2.0]
    A[1] = [1.0, 1.0, 1.0]
    A[2] = [2.0, 0.5, 1.0]
    A[3:] = np.eye(m)
    b = np.array([4.0, 3.0, 5.0])
    c = np.array([1.0, 0.5, 0.25, 0, 0, 0])
    o = oracle.solve(A, b, c)
    with spx.Context(A, b, c, window=8, tableau=True) as ctx:
        r = ctx.solve()
    assert r.status == spx.SolveStatus.Unbounded and r.pivots == o.pivots


def test_tableau_reinvert_and_warm_start(spx, oracle):
    """spx_reinvert and spx_set_basis rebuild T_w = B_w A (k_tab_build) and
    dw: the run continues on the oracle's path and reaches its optimum."""
    m, n, seed = 200, 700, 3
    A, b, c = oracle.generate(m, n, seed)
    ref = oracle.solve(A, b, c, eps=1e-7, want_state=True)
    mid = oracle.solve(A, b, c, eps=1e-7, max_iter=60, want_state=True)
    with spx.Context(A, b, c, window=16, tableau=True) as ctx:
        ctx.iterate(37)
        ctx.reinvert()
        ctx.iterate(23)
        s = ctx.state(binv=True)
        assert list(s["b_ixs"]) == list(mid.b_ixs)
        assert _rel(s["binv"], mid.binv) <= 1e-9
        r = ctx.solve()
        assert r.status == spx.SolveStatus.OptimumFound and r.pivots == ref.pivots
        assert abs(r.z - ref.z) <= 1e-9 * abs(ref.z)
    with spx.Context(A, b, c, window=16, tableau=True) as ctx:
        ctx.set_basis(mid.b_ixs)
        r = ctx.solve()
        assert r.status == spx.SolveStatus.OptimumFound
        assert abs(r.z - ref.z) <= 1e-9 * abs(ref.z)
        assert sorted(int(j) for j in r.b_ixs) == sorted(int(j) for j in ref.b_ixs)


def test_tableau_refactor_every(spx, oracle):
    m, n, seed = 257, 771, 2
    A, b, c = oracle.generate(m, n, seed)
    ref = oracle.solve(A, b, c, eps=1e-7, want_state=True)
    with spx.Context(A, b, c, window=32, tableau=True, refactor_every=50) as ctx:
        r = ctx.solve()
    assert r.status == spx.SolveStatus.OptimumFound and r.pivots == ref.pivots
    assert abs(r.z - ref.z) <= 1e-9 * abs(ref.z)


def test_tableau_devex_matches_window_devex(spx):
    """Devex weights come from the pass's r.A_j (Wt[j][tau]) in both modes."""
    m, n, seed, k = 300, 1200, 5, 150
    out = {}
    for tab, persist in ((False, False), (True, False), (True, True)):
        with spx.Context(m=m, n=n, seed=seed, window=16, pricing=spx.PRICING_DEVEX, tableau=tab,
                         persist=persist) as ctx:
            ctx.iterate(k)
            out[tab, persist] = ctx.state(binv=True)
    ref = out[False, False]
    for key in ((True, False), (True, True)):
        assert np.array_equal(out[key]["b_ixs"], ref["b_ixs"]), key
        assert _rel(out[key]["x_b"], ref["x_b"]) <= 1e-10, key


def test_tableau_rejects(spx):
    with pytest.raises(spx.SimplexError):
        spx.Context(m=64, n=256, seed=0, window=-1, tableau=True)
    with pytest.raises(spx.SimplexError):
        spx.Context(m=64, n=256, seed=0, rank=0, nranks=2, tableau=True)


@pytest.mark.parametrize("m,n,k,window", [(4096, 16384, 300, 64), (12000, 14000, 70, 32)])
def test_tableau_large_invariants(spx, oracle, m, n, k, window):
    """C3 over several folds, and m = 12000: B^-1 B = I on sampled basis
    columns, x_b = B^-1 b, z = c_B.x_b, and the pivots of the eta window."""
    seed = 0
    with spx.Context(m=m, n=n, seed=seed, window=window, persist=False) as ctx:
        ctx.iterate(k)
        s_w = ctx.state()
    with spx.Context(m=m, n=n, seed=seed, window=window, tableau=True) as ctx:
        st, piv = ctx.iterate(k)
        assert st == spx.SolveStatus.MaxIter and piv == k
        s = ctx.state(binv=True)
        z = ctx.objective()
    assert np.array_equal(s["b_ixs"], s_w["b_ixs"])
    b = (n - m) / 4.0 * (1.0 + oracle.uniform_np(seed, 2, np.arange(m, dtype=np.uint64)))
    c = np.zeros(n)
    c[: n - m] = oracle.uniform_np(seed, 3, np.arange(n - m, dtype=np.uint64))
    rows = np.linspace(0, m - 1, 12).astype(np.int64)
    Bcols = np.stack([oracle.column_np(m, n, seed, int(s["b_ixs"][i])) for i in rows], axis=1)
    I = s["binv"] @ Bcols
    E = np.zeros_like(I)
    E[rows, np.arange(len(rows))] = 1.0
    assert np.max(np.abs(I - E)) < 1e-9
    assert _rel(s["binv"] @ b, s["x_b"]) < 1e-10
    assert abs(z - float(c[s["b_ixs"]] @ s["x_b"])) <= 1e-10 * abs(z)
    assert np.all(s["x_b"] > -1e-9)


@pytest.mark.parametrize("keep_bw", ["0", "1"])
def test_tableau_bw_forms_match_oracle(spx, oracle, monkeypatch, keep_bw):
    """With A[:, n-m:] = I the tableau skips k_fold (B_w is T_w's slack block,
    rebuilt for readbacks by k_tab_binv); SPX_TAB_BW=1 keeps B_w and k_fold.
    Both follow the oracle across several folds (window 16, 150 pivots)."""
    monkeypatch.setenv("SPX_TAB_BW", keep_bw)
    m, n, k = 257, 771, 150
    A, b, c = oracle.generate(m, n, 2)
    ref = oracle.solve(A, b, c, max_iter=k, eps=1e-7, want_state=True, trace_cap=k)
    with spx.Context(A, b, c, eps=1e-7, window=16, tableau=True, persist=False) as ctx:
        st, piv = ctx.iterate(k)
        s = ctx.state(binv=True)
        z = ctx.objective()
        # a readback mid-solve, then more pivots: the rebuilt B_w stays consistent
        st2, piv2 = ctx.iterate(20)
        s2 = ctx.state(binv=True)
    assert piv == ref.pivots
    assert list(s["b_ixs"]) == list(ref.b_ixs)
    assert _rel(s["x_b"], ref.x_b) <= 1e-9
    assert _rel(s["y"], ref.y) <= 1e-9
    assert _rel(s["binv"], ref.binv) <= 1e-9
    assert abs(z - ref.z) <= 1e-9 * abs(ref.z)
    ref2 = oracle.solve(A, b, c, max_iter=k + piv2, eps=1e-7, want_state=True, trace_cap=k + piv2)
    assert list(s2["b_ixs"]) == list(ref2.b_ixs)
    assert _rel(s2["binv"], ref2.binv) <= 1e-9
    assert _rel(s2["x_b"], ref2.x_b) <= 1e-9

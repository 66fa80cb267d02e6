"""GPU: the eta-window representation of B^-1 (spx_opts.window)
against the CPU oracle (which rewrites B^-1 every pivot, v4:331-333) and
against the explicit in-place update.

Tolerances as in test_gpu_parity.py: pivot path identical, state within 1e-9
relative of the oracle; explicit vs window within 1e-10 (same arithmetic,
different association).  Graph vs eager and sharded vs single-rank runs of
the same window are bit-identical.
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
@pytest.mark.parametrize("m,n,seed,k", [(257, 771, 2, 150), (1000, 3000, 3, 140)])
def test_window_state_matches_oracle(spx, oracle, window, m, n, seed, k, persist):
    A, b, c = oracle.generate(m, n, seed)
    ref = oracle.solve(A, b, c, max_iter=k, eps=1e-7, want_state=True, trace_cap=k)
    with spx.Context(A, b, c, eps=1e-7, window=window, persist=persist) as ctx:
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
    Bmat = A[s["b_ixs"]].T
    assert np.max(np.abs(s["binv"] @ Bmat - np.eye(m))) < 1e-8


@pytest.mark.parametrize("window", [8, 32])
def test_window_step_api_trace(spx, oracle, window):
    """spx_price / spx_pivot one pass at a time (folds on the host's schedule)."""
    m, n, seed, K = 100, 300, 1, 70
    A, b, c = oracle.generate(m, n, seed)
    ref = oracle.solve(A, b, c, eps=1e-7, trace_cap=K)
    with spx.Context(A, b, c, window=window) as ctx:
        ps, qs = [], []
        for _ in range(min(K, ref.pivots)):
            p, e, opt = ctx.price()
            assert not opt
            q, st = ctx.pivot()
            ps.append(p)
            qs.append(q)
    assert ps == list(ref.trace_p[: len(ps)]) and qs == list(ref.trace_q[: len(qs)])


def test_window_readback_mid_window_then_continue(spx, oracle):
    """A readback folds the window early; the run continues on the same path."""
    m, n, seed = 300, 1200, 7
    A, b, c = oracle.generate(m, n, seed)
    ref = oracle.solve(A, b, c, max_iter=100, want_state=True)
    with spx.Context(A, b, c, window=16) as ctx:
        for k in (13, 1, 2, 40, 44):
            ctx.iterate(k)
            s = ctx.state(binv=True)
            ctx.reduced_costs()
    assert list(s["b_ixs"]) == list(ref.b_ixs)
    assert _rel(s["x_b"], ref.x_b) <= 1e-9
    assert _rel(s["y"], ref.y) <= 1e-9
    assert _rel(s["binv"], ref.binv) <= 1e-9


@pytest.mark.parametrize("window", [16, 32])
def test_window_graph_eager_bit_identical(spx, window):
    """Two-kernel passes (persist=False): graph replay, eager launches and every
    pricing geometry give the same bits.  The persistent loop kernel (k_loop,
    both workgroup sizes) groups the ratio test's c_B.alpha sum by its own
    geometry: same pivots, values within 1e-12."""
    m, n, seed, k = 300, 1200, 7, 130
    runs = []
    for kw in (dict(), dict(graph_batch=-1), dict(graph_batch=5), dict(price_grid=3), dict(price_block=1024)):
        with spx.Context(m=m, n=n, seed=seed, window=window, persist=False, **kw) as ctx:
            assert ctx.config()["persistent"] == 0
            ctx.iterate(k)
            runs.append((kw, ctx.state(binv=True)))
    s0 = runs[0][1]
    for kw, s in runs[1:]:
        for key in ("b_ixs", "x_b", "y", "binv"):
            assert np.array_equal(s[key], s0[key]), (kw, key)
    with spx.Context(m=m, n=n, seed=seed, window=window, persist=True) as ctx:
        assert ctx.config()["persistent"] == 1
        st, piv = ctx.iterate(k)
        s = ctx.state(binv=True)
    assert piv == k and np.array_equal(s["b_ixs"], s0["b_ixs"])
    for key in ("x_b", "y", "binv"):
        assert _rel(s[key], s0[key]) <= 1e-12, key


def test_window_matches_explicit_update(spx):
    m, n, seed, k = 1100, 3300, 4, 150
    out = {}
    for w in (-1, 32):
        with spx.Context(m=m, n=n, seed=seed, window=w) as ctx:
            st, piv = ctx.iterate(k)
            out[w] = (piv, ctx.state(binv=True), ctx.objective())
    (p0, s0, z0), (p1, s1, z1) = out[-1], out[32]
    assert p0 == p1 == k
    assert np.array_equal(s0["b_ixs"], s1["b_ixs"])
    for key in ("x_b", "y", "binv"):
        assert _rel(s1[key], s0[key]) <= 1e-10, key
    assert abs(z1 - z0) <= 1e-10 * abs(z0)


@pytest.mark.parametrize("case_i", [0, 3, 6, 9, 10])
def test_window_golden_optimum(spx, golden, case_i):
    case = golden["cases"][case_i]
    with spx.Context(m=case["m"], n=case["n"], seed=case["seed"], eps=golden["eps"], window=16) as ctx:
        r = ctx.solve()
    assert r.status == spx.SolveStatus.OptimumFound
    assert abs(r.z - case["highs_z"]) <= 1e-9 * abs(case["highs_z"])
    assert sorted(int(j) for j in r.b_ixs) == case["highs_basis"]
    assert r.pivots == case["oracle_pivots"]


def test_window_unbounded(spx, oracle):
    m, n = 3, 6
    A = np.zeros((n, m))
    A[0] = [-1.0, 0.0, -2.0]
    A[1] = [1.0, 1.0, 1.0]
    A[2] = [2.0, 0.5, 1.0]
    A[3:] = np.eye(m)
    b = np.array([4.0, 3.0, 5.0])
    c = np.array([1.0, 0.5, 0.25, 0, 0, 0])
    o = oracle.solve(A, b, c)
    with spx.Context(A, b, c, window=8) as ctx:
        r = ctx.solve()
    assert r.status == spx.SolveStatus.Unbounded and r.pivots == o.pivots


@pytest.mark.parametrize("G,m,n,k", [(2, 300, 1200, 150), (3, 257, 771, 120), (4, 5, 7, 10)])
def test_window_shard_group_matches_single_rank(spx, G, m, n, k):
    """Column-sharded pricing: the winner's window coefficients travel in the
    MINLOC record; every shard reproduces the single-rank window run bitwise."""
    seed = 11
    with spx.Context(m=m, n=n, seed=seed, window=16, persist=False) as ref:
        rst, rpiv = ref.iterate(k)
        rs = ref.state(binv=True)
    ctxs = [spx.Context(m=m, n=n, seed=seed, rank=g, nranks=G, window=16) for g in range(G)]
    try:
        st, piv = spx.group_iterate(ctxs, k)
        assert st == rst and piv == rpiv
        for c in ctxs:
            s = c.state(binv=True)
            for key in ("b_ixs", "x_b", "y", "binv"):
                assert np.array_equal(s[key], rs[key]), key
    finally:
        for c in ctxs:
            c.close()


def test_window_rejects_row_shard_and_bad_size(spx):
    with pytest.raises(spx.SimplexError):
        spx.Context(m=64, n=256, seed=0, window=12)
    with pytest.raises(spx.SimplexError):
        spx.Context(m=64, n=256, seed=0, rank=0, nranks=2, row_shard=True, window=16)


@pytest.mark.parametrize("m,n,k,window", [(4096, 16384, 100, 32), (12000, 14000, 40, 32), (20000, 21000, 12, 16)])
def test_window_large_invariants(spx, oracle, m, n, k, window):
    """C3 (base row in LDS), m=12000 (base row read from L2) and m=20000
    (global y): B^-1 B = I on sampled basis columns, x_b = B^-1 b, z = c_B.x_b."""
    seed = 0
    with spx.Context(m=m, n=n, seed=seed, window=window) as ctx:
        st, piv = ctx.iterate(k)
        assert st == spx.SolveStatus.MaxIter and piv == k
        s = ctx.state(binv=True)
        z = ctx.objective()
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


@pytest.mark.parametrize("m,n,want", [(1024, 4096, 0), (2047, 4096, 0), (2048, 4096, 64), (4096, 16384, 64),
                                      (4096, 131072, 64)])
def test_auto_representation(spx, m, n, want):
    """window = 0 picks the eta window of 64 at m >= 2048 (C3, C4, C5) and the
    explicit rank-1 update below (C2); row-sharded B^-1 is always explicit."""
    with spx.Context(m=m, n=n, seed=0) as ctx:
        assert ctx.config()["window"] == want

"""Parity of the HIP path (libsimplex, through its C-ABI) against the CPU oracle
(oracle/simplex_oracle.c, a restatement of src/v4_cub_reduction.cu:219-380) and
the golden fixtures (input/sample.txt known answer; HiGHS optima).

Tolerances (fp64):
  * objective   |z_gpu - z_ref| <= 1e-9 |z_ref|, basis SET identical
  * pivot path  entering/leaving indices identical to the oracle's
  * state       x_b, y, B^-1 within 1e-9 relative (max-norm) after K pivots
  * e_j         max|e_gpu - e_cpu| <= 1e-12 * max|e_cpu| (pricing GEMV)
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REL_Z = 1e-9


def _rel(a, b):
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    return float(np.max(np.abs(a - b)) / max(1.0, float(np.max(np.abs(b)))))


def test_sample_known_answer(spx, oracle):
    # input/sample.txt:15-16 — "Optimum: 9 / For x0 = 1, x1 = 3"
    m, n, A, b, c = spx.read_lp("tests/golden/sample.txt")
    r = spx.solve(A, b, c, max_iter=5, eps=1e-4)  # reference constants (v4:18-19)
    assert r.status == spx.SolveStatus.OptimumFound
    assert r.z == 9.0
    assert list(r.b_ixs) == [1, 0]
    assert list(r.x_b) == [3.0, 1.0]
    assert r.pivots == 2


def test_sample_max_iter_semantics(spx, oracle):
    m, n, A, b, c = spx.read_lp("tests/golden/sample.txt")
    for k in range(0, 4):
        r = spx.solve(A, b, c, max_iter=k, eps=1e-4)
        o = oracle.solve(A, b, c, max_iter=k, eps=1e-4)
        assert int(r.status) == o.status, k
        assert r.pivots == o.pivots, k


@pytest.mark.parametrize("case_i", range(11))
def test_golden_optimum(spx, oracle, golden, case_i):
    case = golden["cases"][case_i]
    m, n, seed = case["m"], case["n"], case["seed"]
    with spx.Context(m=m, n=n, seed=seed, eps=golden["eps"]) as ctx:
        r = ctx.solve()
    assert r.status == spx.SolveStatus.OptimumFound
    assert abs(r.z - case["highs_z"]) <= REL_Z * abs(case["highs_z"])
    assert sorted(int(j) for j in r.b_ixs) == case["highs_basis"]
    assert r.pivots == case["oracle_pivots"]


def test_generator_bit_identical(spx, oracle):
    m, n, seed = 37, 101, 5
    A, b, c = oracle.generate(m, n, seed)
    with spx.Context(m=m, n=n, seed=seed) as ctx:
        st = ctx.state()
        # y = c_B, x_b = b at the slack basis
        assert np.array_equal(st["x_b"], b)
        assert np.array_equal(st["c_B"], c[n - m:])
        e = ctx.reduced_costs()
    e_ref = oracle.price(A, c, c[n - m:].copy())
    assert _rel(e, e_ref) <= 1e-12


@pytest.mark.parametrize("m,n,seed", [(64, 256, 0), (100, 300, 1), (257, 771, 2), (512, 2048, 0)])
def test_pivot_trace_matches_oracle(spx, oracle, golden, m, n, seed):
    A, b, c = oracle.generate(m, n, seed)
    K = 64
    ref = oracle.solve(A, b, c, eps=1e-7, trace_cap=K)
    with spx.Context(A, b, c, eps=1e-7) as ctx:
        ps, qs = [], []
        for _ in range(min(K, ref.pivots)):
            p, e, opt = ctx.price()
            assert not opt
            q, st = ctx.pivot()
            ps.append(p)
            qs.append(q)
    k = len(ps)
    assert ps == list(ref.trace_p[:k])
    assert qs == list(ref.trace_q[:k])


@pytest.mark.parametrize("m,n,seed,k", [(64, 256, 0, 20), (257, 771, 2, 60), (1000, 3000, 3, 150)])
def test_state_after_k_pivots(spx, oracle, m, n, seed, k):
    A, b, c = oracle.generate(m, n, seed)
    ref = oracle.solve(A, b, c, max_iter=k, eps=1e-7, want_state=True)
    with spx.Context(A, b, c, eps=1e-7) as ctx:
        st, piv = ctx.iterate(k)
        s = ctx.state(binv=True)
        e = ctx.reduced_costs()
    assert piv == ref.pivots
    assert list(s["b_ixs"]) == list(ref.b_ixs)
    assert _rel(s["x_b"], ref.x_b) <= 1e-9
    assert _rel(s["y"], ref.y) <= 1e-9
    assert _rel(s["binv"], ref.binv) <= 1e-9
    # pricing GEMV against the CPU restatement from the GPU's own y
    e_ref = oracle.price(A, c, s["y"])
    assert _rel(e, e_ref) <= 1e-12
    # structural invariants: B^-1 B = I, x_b = B^-1 b, y = c_B B^-1
    Bmat = A[s["b_ixs"]].T  # columns of the basis
    I = s["binv"] @ Bmat
    assert np.max(np.abs(I - np.eye(m))) < 1e-8
    assert _rel(s["binv"] @ b, s["x_b"]) < 1e-9
    assert _rel(c[s["b_ixs"]] @ s["binv"], s["y"]) < 1e-9


def test_graph_eager_and_tunings_bit_identical(spx):
    """Deterministic kernels: graph replay, eager launches and every pricing
    geometry produce the same bits (the property that keeps multi-GPU replicas
    identical).  The update geometry (rows per workgroup) fixes the order of the
    c_B.alpha sum behind s_y, so those variants agree to 1e-12 with identical
    pivots."""
    m, n, seed, k = 300, 1200, 7, 120
    runs = []
    variants = [dict(), dict(graph_batch=-1), dict(graph_batch=5), dict(price_block=1024), dict(price_grid=3),
                dict(split_tail=True), dict(update_rows=4), dict(update_rows=8), dict(update_block=256)]
    for kw in variants:
        with spx.Context(m=m, n=n, seed=seed, **kw) as ctx:
            ctx.iterate(k)
            s = ctx.state(binv=True)
            runs.append((kw, s))
    s0 = runs[0][1]
    for kw, s in runs[1:]:
        assert np.array_equal(s["b_ixs"], s0["b_ixs"]), kw
        same = not any(key.startswith("update_") for key in kw)
        for key in ("x_b", "y", "binv"):
            if same:
                assert np.array_equal(s[key], s0[key]), (kw, key)
            else:
                assert _rel(s[key], s0[key]) <= 1e-12, (kw, key)


def test_unbounded(spx, oracle):
    # column 0 has A <= 0 and c > 0: x0 can grow forever
    m, n = 3, 6
    A = np.zeros((n, m))
    A[0] = [-1.0, 0.0, -2.0]
    A[1] = [1.0, 1.0, 1.0]
    A[2] = [2.0, 0.5, 1.0]
    A[3:] = np.eye(m)
    b = np.array([4.0, 3.0, 5.0])
    c = np.array([1.0, 0.5, 0.25, 0, 0, 0])
    o = oracle.solve(A, b, c)
    r = spx.solve(A, b, c)
    assert o.status == oracle.UNBOUNDED
    assert r.status == spx.SolveStatus.Unbounded
    assert r.pivots == o.pivots


def test_all_slack_m_equals_n(spx, oracle):
    m = n = 5
    A = np.eye(m)
    b = np.arange(1.0, 6.0)
    c = np.zeros(n)
    r = spx.solve(A, b, c)
    assert r.status == spx.SolveStatus.OptimumFound
    assert r.pivots == 0 and r.z == 0.0


def test_degenerate_ties_first_index(spx, oracle):
    # duplicated columns and equal ratios force ties in both argmins
    m, n = 4, 10
    rng = np.random.default_rng(3)
    U = rng.integers(1, 4, size=(n - m, m)).astype(np.float64)
    U[1] = U[0]
    U[3] = U[2]
    A = np.vstack([U, np.eye(m)])
    b = np.full(m, 6.0)
    c = np.zeros(n)
    c[: n - m] = [3, 3, 2, 2, 1, 1]
    o = oracle.solve(A, b, c, trace_cap=32)
    with spx.Context(A, b, c) as ctx:
        ps, qs = [], []
        while True:
            p, e, opt = ctx.price()
            if opt:
                break
            q, st = ctx.pivot()
            ps.append(p)
            qs.append(q)
            if st != spx.SolveStatus.MaxIter:
                break
    assert ps == list(o.trace_p) and qs == list(o.trace_q)


def test_large_headline_properties(spx):
    """C3 (m=4096, n=16384): size-independent invariants after a window of pivots."""
    m, n = 4096, 16384
    with spx.Context(m=m, n=n, seed=0) as ctx:
        st, piv = ctx.iterate(200)
        assert st == spx.SolveStatus.MaxIter and piv == 200
        s = ctx.state(binv=True)
        z = ctx.objective()
    import oracle as orc

    A, b, c = orc.generate(m, n, 0)
    # B^-1 B = I on a sample of columns, x_b = B^-1 b, objective monotone & = c_B.x_b
    Bmat = A[s["b_ixs"]].T
    cols = np.arange(0, m, 97)
    I = s["binv"] @ Bmat[:, cols]
    E = np.zeros_like(I)
    E[cols, np.arange(len(cols))] = 1.0
    assert np.max(np.abs(I - E)) < 1e-9
    assert _rel(s["binv"] @ b, s["x_b"]) < 1e-10
    assert abs(z - float(c[s["b_ixs"]] @ s["x_b"])) <= 1e-10 * abs(z)
    assert np.all(s["x_b"] > -1e-9)  # primal feasibility maintained


@pytest.mark.parametrize("G,m,n,k", [(2, 300, 1200, 150), (3, 257, 771, 120), (8, 512, 2048, 200), (4, 5, 7, 10)])
def test_shard_group_matches_single_rank(spx, G, m, n, k):
    """Column-sharded pricing over G shards + G-way MINLOC merge + replicated
    update reproduces the single-rank trajectory bit for bit on every shard."""
    seed = 11
    with spx.Context(m=m, n=n, seed=seed) as ref:
        rst, rpiv = ref.iterate(k)
        rs = ref.state(binv=True)
        rz = ref.objective()
    ctxs = [spx.Context(m=m, n=n, seed=seed, rank=g, nranks=G) for g in range(G)]
    try:
        st, piv = spx.group_iterate(ctxs, k)
        assert st == rst and piv == rpiv
        for c in ctxs:
            s = c.state(binv=True)
            assert np.array_equal(s["b_ixs"], rs["b_ixs"])
            assert np.array_equal(s["x_b"], rs["x_b"])
            assert np.array_equal(s["y"], rs["y"])
            assert np.array_equal(s["binv"], rs["binv"])
            assert c.objective() == rz
    finally:
        for c in ctxs:
            c.close()


def test_shard_group_solves_to_golden_optimum(spx, golden):
    case = [c for c in golden["cases"] if c["m"] == 256][0]
    G = 4
    ctxs = [spx.Context(m=case["m"], n=case["n"], seed=case["seed"], rank=g, nranks=G) for g in range(G)]
    try:
        st = spx.SolveStatus.MaxIter
        while st == spx.SolveStatus.MaxIter:
            st, piv = spx.group_iterate(ctxs, 64)
        assert st == spx.SolveStatus.OptimumFound and piv == case["oracle_pivots"]
        r = ctxs[0].solve(0)
        assert abs(r.z - case["highs_z"]) <= 1e-9 * abs(case["highs_z"])
        assert sorted(int(j) for j in r.b_ixs) == case["highs_basis"]
    finally:
        for c in ctxs:
            c.close()


@pytest.mark.parametrize("G,m,n,k", [(2, 300, 1200, 150), (3, 257, 771, 120), (8, 512, 2048, 200),
                                     (4, 1100, 3300, 100), (2, 5000, 7000, 30)])
def test_row_sharded_group_matches_single_rank(spx, G, m, n, k):
    """B^-1 row-sharded over G in-process shards (pivot row carried by the
    ratio-test all-gather): same pivots as one rank; values within 1e-9 (s_y is
    evaluated from the gathered c_B.alpha sum, a reassociation)."""
    seed = 13
    with spx.Context(m=m, n=n, seed=seed) as ref:
        rst, rpiv = ref.iterate(k)
        rs = ref.state(binv=True)
        rz = ref.objective()
    ctxs = [spx.Context(m=m, n=n, seed=seed, rank=g, nranks=G, row_shard=True) for g in range(G)]
    try:
        st, piv = spx.group_iterate(ctxs, k)
        assert st == rst and piv == rpiv
        spx.group_sync(ctxs)
        binv = np.zeros((m, m))
        mb = (m + G - 1) // G
        for g, c in enumerate(ctxs):
            s = c.state(binv=True)
            assert np.array_equal(s["b_ixs"], rs["b_ixs"])
            assert _rel(s["x_b"], rs["x_b"]) <= 1e-9
            assert _rel(s["y"], rs["y"]) <= 1e-9
            assert abs(c.objective() - rz) <= 1e-9 * abs(rz)
            binv[g * mb:(g + 1) * mb] = s["binv"][g * mb:(g + 1) * mb]
        assert _rel(binv, rs["binv"]) <= 1e-9
    finally:
        for c in ctxs:
            c.close()


def test_row_sharded_group_solves_to_golden_optimum(spx, golden):
    case = [c for c in golden["cases"] if c["m"] == 512][0]
    G = 4
    ctxs = [spx.Context(m=case["m"], n=case["n"], seed=case["seed"], rank=g, nranks=G, row_shard=True)
            for g in range(G)]
    try:
        st = spx.SolveStatus.MaxIter
        while st == spx.SolveStatus.MaxIter:
            st, piv = spx.group_iterate(ctxs, 128)
        assert st == spx.SolveStatus.OptimumFound and piv == case["oracle_pivots"]
        spx.group_sync(ctxs)
        r = ctxs[2].solve(0)
        assert abs(r.z - case["highs_z"]) <= 1e-9 * abs(case["highs_z"])
        assert sorted(int(j) for j in r.b_ixs) == case["highs_basis"]
    finally:
        for c in ctxs:
            c.close()


def test_row_sharded_unbounded(spx, oracle):
    m, n = 3, 6
    A = np.zeros((n, m))
    A[0] = [-1.0, 0.0, -2.0]
    A[1] = [1.0, 1.0, 1.0]
    A[2] = [2.0, 0.5, 1.0]
    A[3:] = np.eye(m)
    b = np.array([4.0, 3.0, 5.0])
    c = np.array([1.0, 0.5, 0.25, 0, 0, 0])
    o = oracle.solve(A, b, c)
    ctxs = [spx.Context(A, b, c, rank=g, nranks=3, row_shard=True) for g in range(3)]
    try:
        st, piv = spx.group_iterate(ctxs, 20)
        assert st == spx.SolveStatus.Unbounded and piv == o.pivots
    finally:
        for c in ctxs:
            c.close()

"""GPU: steepest-edge pricing with the Goldfarb-Reid recurrence
(SPX_PRICING_STEEPEST; README.md:16-17 "Steepest edge with a recurrence")
against the oracle's restatement (oracle/simplex_oracle.c se_choose), through
the C-ABI.

The GPU forms A_j . B^-T alpha as a third dot on the pricing pass's A stream
(B_w^T alpha in LDS, plus the window terms), the oracle with its explicit
B^-1, so the weights agree to rounding, not bits.  Tolerances: the same (p, q)
sequence as the oracle; z within 1e-9 of the HiGHS optimum (golden
fixtures); weights within 1e-9 (relative) of the oracle's and of the
definition 1 + ||B^-1 A_j||^2 from the GPU's own B^-1.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

STEEP = 2


class _env:
    def __init__(self, **kv):
        self.kv = kv

    def __enter__(self):
        self.old = {k: os.environ.get(k) for k in self.kv}
        os.environ.update({k: str(v) for k, v in self.kv.items()})

    def __exit__(self, *exc):
        for k, v in self.old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


def _nonbasic(n, basis):
    mask = np.ones(n, dtype=bool)
    mask[np.asarray(basis, dtype=np.int64)] = False
    return np.nonzero(mask)[0]


@pytest.mark.parametrize("case_ix,window,dense", [(0, 16, False), (3, 64, False), (6, 32, False), (8, 64, True)],
                         ids=["c0-w16", "c3-w64", "c6-w32", "c8-w64-dense"])
def test_steepest_matches_oracle_full_solve(spx, oracle, golden, case_ix, window, dense):
    case = golden["cases"][case_ix]
    m, n, seed = case["m"], case["n"], case["seed"]
    A, b, c = oracle.generate(m, n, seed)
    ref = oracle.solve(A, b, c, pricing=oracle.PRICING_STEEPEST, trace_cap=1 << 14)
    assert ref.status == oracle.OPTIMUM_FOUND
    with _env(SPX_DENSE_FTRAN="1" if dense else "0"):
        with spx.Context(m=m, n=n, seed=seed, window=window, pricing=STEEP, trace=1 << 14) as ctx:
            assert ctx.config()["persistent"] == 0
            r = ctx.solve()
            tp, tq = ctx.trace()
    assert r.status == spx.SolveStatus.OptimumFound
    assert r.pivots == ref.pivots
    assert list(tp) == list(ref.trace_p) and list(tq) == list(ref.trace_q)
    assert abs(r.z - case["highs_z"]) <= 1e-9 * abs(case["highs_z"])
    assert sorted(int(j) for j in r.b_ixs) == case["highs_basis"]


@pytest.mark.parametrize("m,n,seed,k,window", [(300, 1200, 2, 90, 64), (512, 2048, 1, 150, 16),
                                               (1024, 4096, 0, 130, 64)])
def test_steepest_weights_match_oracle_and_definition(spx, oracle, m, n, seed, k, window):
    """After k pivots and one more pricing pass (which applies the last
    pivot's update): the GPU's weights of the non-basic columns against the
    oracle's, and against 1 + ||B^-1 A_j||^2 from the GPU's B^-1."""
    A, b, c = oracle.generate(m, n, seed)
    ref = oracle.solve(A, b, c, pricing=oracle.PRICING_STEEPEST, max_iter=k, trace_cap=k, want_state=True)
    assert ref.pivots == k
    with spx.Context(m=m, n=n, seed=seed, window=window, pricing=STEEP, trace=k) as ctx:
        st, piv = ctx.iterate(k)
        assert piv == k
        tp, tq = ctx.trace()
        s = ctx.state(binv=True)
        ctx.price()
        w = ctx.weights()
    assert list(tp) == list(ref.trace_p) and list(tq) == list(ref.trace_q)
    nb = _nonbasic(n, s["b_ixs"])
    assert np.max(np.abs(w[nb] - ref.weights[nb]) / ref.weights[nb]) <= 1e-9
    exact = 1.0 + np.sum((s["binv"] @ A[nb].T) ** 2, axis=0)
    assert np.max(np.abs(w[nb] - exact) / exact) <= 1e-9


def test_steepest_degenerate_guarded(spx, oracle):
    """A degenerate LP (tests/lpgen.py) with the guarded ratio test: the HiGHS
    optimum in fewer pivots than Dantzig.  Degenerate pivots leave many
    entering candidates whose keys differ only in rounding, so the GPU's
    weights (the same recurrence, summed in another order) may take another
    path than the oracle's after a while: the first pivots agree."""
    from lpgen import degenerate_lp, highs_opt

    A, b, c = degenerate_lp(300, 900, 4)
    z_star = highs_opt(A, b, c)
    ref = oracle.solve(A, b, c, ratio=oracle.RATIO_GUARDED, pricing=oracle.PRICING_STEEPEST, trace_cap=1 << 14)
    dz = oracle.solve(A, b, c, ratio=oracle.RATIO_GUARDED)
    with spx.Context(A, b, c, window=64, pricing=STEEP, ratio_test=1, trace=1 << 14) as ctx:
        r = ctx.solve()
        tp, tq = ctx.trace()
    assert r.status == spx.SolveStatus.OptimumFound
    assert abs(r.z - z_star) <= 1e-9 * abs(z_star)
    assert r.pivots < dz.pivots and ref.pivots < dz.pivots
    k = min(len(tp), len(ref.trace_p))
    diff = np.nonzero((tp[:k] != ref.trace_p[:k]) | (tq[:k] != ref.trace_q[:k]))[0]
    agree = int(diff[0]) if len(diff) else k
    assert agree >= 50, agree


def test_steepest_refused_configs(spx):
    with pytest.raises(spx.SimplexError):
        spx.Context(m=64, n=256, seed=0, window=-1, pricing=STEEP)  # needs the eta window
    with pytest.raises(spx.SimplexError):
        spx.Context(m=64, n=256, seed=0, window=16, pricing=STEEP, tableau=True)


def test_steepest_large_m_global_v(spx, oracle):
    """m = 6000 (L = 6016): y, the base row and B_w^T alpha no longer fit LDS
    together, so v is read from global memory (k_price WM 5); the oracle's
    pivot path for 60 pivots."""
    m, n, seed, k = 6000, 9000, 2, 60
    A, b, c = oracle.generate(m, n, seed)
    ref = oracle.solve(A, b, c, pricing=oracle.PRICING_STEEPEST, max_iter=k, trace_cap=k)
    with spx.Context(A, b, c, window=64, pricing=STEEP, trace=k) as ctx:
        ctx.iterate(k)
        tp, tq = ctx.trace()
    assert list(tp) == list(ref.trace_p) and list(tq) == list(ref.trace_q)


def test_steepest_c3_matches_oracle_fixture(spx):
    """The headline config (C3: m=4096, n=16384, seed 0) with steepest edge:
    the oracle's first 130 pivots (two eta-window folds; the committed
    fixture tests/golden/oracle_c3se_k130.npz from make_golden_c45.py C3SE),
    x_b / y / z within 1e-9, and after one more pricing pass the weights of
    every non-basic column within 1e-9 (relative) of the oracle's."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    g = np.load(os.path.join(root, "tests", "golden", "oracle_c3se_k130.npz"))
    K = int(g["k"])
    m, n, seed = int(g["m"]), int(g["n"]), int(g["seed"])
    assert (m, n, seed, int(g["pricing"])) == (4096, 16384, 0, STEEP)
    with spx.Context(m=m, n=n, seed=seed, eps=float(g["eps"]), pricing=STEEP, trace=K) as ctx:
        cfg = ctx.config()
        assert cfg["window"] == 64 and cfg["persistent"] == 0
        st, piv = ctx.iterate(K)
        assert st == spx.SolveStatus.MaxIter and piv == K
        tp, tq = ctx.trace()
        s = ctx.state()
        z = ctx.objective()
        ctx.price()
        w = ctx.weights()
    assert np.array_equal(tp, g["trace_p"]), int(np.argmax(tp != g["trace_p"]))
    assert np.array_equal(tq, g["trace_q"]), int(np.argmax(tq != g["trace_q"]))
    assert np.array_equal(s["b_ixs"], g["b_ixs"])
    for key in ("x_b", "y"):
        ref = g[key]
        assert np.max(np.abs(s[key] - ref)) <= 1e-9 * max(1.0, float(np.max(np.abs(ref)))), key
    assert abs(z - float(g["z"])) <= 1e-9 * abs(float(g["z"]))
    nb = _nonbasic(n, s["b_ixs"])
    wr = g["weights"]
    assert np.max(np.abs(w[nb] - wr[nb]) / wr[nb]) <= 1e-9


def test_steepest_c3_solves_to_highs_optimum(spx):
    """C3 solved to optimality with steepest edge: the HiGHS optimum and basis
    set of the committed fixture (tests/golden/highs_c3.json), in fewer pivots
    than Dantzig's 18,291 (the oracle's C3 trace)."""
    import json

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with open(os.path.join(root, "tests", "golden", "highs_c3.json")) as f:
        h = json.load(f)
    with spx.Context(m=h["m"], n=h["n"], seed=h["seed"], eps=h["eps"], pricing=STEEP) as ctx:
        r = ctx.solve()
    print(f"C3 steepest edge: {r.pivots} pivots (Dantzig {h['oracle_pivots']})")
    assert r.status == spx.SolveStatus.OptimumFound
    assert abs(r.z - h["highs_z"]) <= 1e-9 * abs(h["highs_z"])
    assert sorted(int(j) for j in r.b_ixs) == h["highs_basis"]
    assert r.pivots < h["oracle_pivots"]


@pytest.mark.parametrize("m,n,k", [(2048, 8192, 300), (4096, 16384, 200)])
def test_steepest_fused_partials_match_k_se_part(spx, m, n, k):
    """k_ftran_bc's fused sums of M^T alpha (Params::se_fused; k_se_part
    skipped on every pass but the first after a fold) against k_se_part's
    (SPX_SE_FUSE=0): the same pivots, x_b and y within 1e-12 and the weights
    within 1e-9 (relative; the oracle test's bound) -- the two group the same
    terms differently (8-row workgroups against 16-row blocks), so the bits
    differ, and the Goldfarb-Reid recurrence carries that rounding from pass
    to pass (measured: 1.8e-11 after 300 pivots at m = 2048)."""
    out = {}
    for fuse in ("1", "0"):
        with _env(SPX_SE_FUSE=fuse):
            with spx.Context(m=m, n=n, seed=1, pricing=STEEP, trace=k) as ctx:
                st, piv = ctx.iterate(k)
                tp, tq = ctx.trace()
                s = ctx.state()
                out[fuse] = (st, piv, tp, tq, s["x_b"], s["y"], ctx.weights(), s["b_ixs"])
    a, b = out["1"], out["0"]
    assert a[:2] == b[:2]
    assert np.array_equal(a[2], b[2]) and np.array_equal(a[3], b[3])
    assert np.array_equal(a[7], b[7])
    for i in (4, 5):
        assert np.max(np.abs(a[i] - b[i])) <= 1e-12 * max(1.0, float(np.max(np.abs(b[i]))))
    nb = _nonbasic(n, a[7])
    assert np.max(np.abs(a[6][nb] - b[6][nb]) / b[6][nb]) <= 1e-9

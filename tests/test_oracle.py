"""CPU: the oracle (fp64 restatement of src/v4_cub_reduction.cu:219-380) pinned
against the reference's known answer and the golden fixtures."""
import numpy as np
import pytest


def test_sample_known_answer(oracle):
    # input/sample.txt:15-16: "Optimum: 9 / For x0 = 1, x1 = 3"
    m, n, A, b, c = oracle.read_lp_text("tests/golden/sample.txt")
    r = oracle.solve(A, b, c, max_iter=5, eps=1e-4, trace_cap=8)  # v4:18-19 constants
    assert r.status == oracle.OPTIMUM_FOUND
    assert r.z == 9.0
    assert list(r.b_ixs) == [1, 0] and list(r.x_b) == [3.0, 1.0]
    # 3 loop passes, 2 pivots: (p=0, q=1) then (p=1, q=0)  
    assert r.pivots == 2 and list(r.trace_p) == [0, 1] and list(r.trace_q) == [1, 0]


def test_sample_max_iter(oracle):
    m, n, A, b, c = oracle.read_lp_text("tests/golden/sample.txt")
    assert oracle.solve(A, b, c, max_iter=2, eps=1e-4).status == oracle.MAX_ITER
    assert oracle.solve(A, b, c, max_iter=3, eps=1e-4).status == oracle.OPTIMUM_FOUND
    r0 = oracle.solve(A, b, c, max_iter=0)
    assert r0.status == oracle.MAX_ITER and r0.pivots == 0


def test_generator_c_equals_numpy(oracle):
    for (m, n, seed) in [(1, 1, 0), (3, 7, 1), (64, 256, 0), (33, 97, 4)]:
        A1, b1, c1 = oracle.generate(m, n, seed)
        A2, b2, c2 = oracle.generate_np(m, n, seed)
        assert np.array_equal(A1, A2) and np.array_equal(b1, b2) and np.array_equal(c1, c2)


def test_generator_known_values(oracle):
    # splitmix64 reference value (Vigna): splitmix64 of state 0 -> 0xE220A8397B1DCDAF
    assert oracle.lib().orc_splitmix64(0) == 0xE220A8397B1DCDAF
    A, b, c = oracle.generate(4, 8, 0)
    assert np.array_equal(A[4:], np.eye(4))
    assert np.all((A[:4] >= 0) & (A[:4] < 1))
    assert np.all((b >= 1.0) & (b < 2.0))  # (n-m)/4 = 1
    assert np.all(c[4:] == 0)


def test_golden_cases(oracle, golden):
    for case in golden["cases"]:
        if case["m"] > 512:
            continue
        A, b, c = oracle.generate(case["m"], case["n"], case["seed"])
        r = oracle.solve(A, b, c, eps=golden["eps"], trace_cap=len(case["oracle_trace_p"]))
        assert r.status == oracle.OPTIMUM_FOUND
        assert abs(r.z - case["highs_z"]) <= 1e-9 * abs(case["highs_z"])
        assert sorted(int(j) for j in r.b_ixs) == case["highs_basis"]
        assert r.pivots == case["oracle_pivots"]
        assert list(r.trace_p) == case["oracle_trace_p"]
        assert list(r.trace_q) == case["oracle_trace_q"]


@pytest.mark.slow
def test_golden_m1024(oracle, golden):
    case = [c for c in golden["cases"] if c["m"] == 1024][0]
    A, b, c = oracle.generate(case["m"], case["n"], case["seed"])
    r = oracle.solve(A, b, c, eps=golden["eps"])
    assert abs(r.z - case["highs_z"]) <= 1e-9 * abs(case["highs_z"])
    assert sorted(int(j) for j in r.b_ixs) == case["highs_basis"]


def test_reference_eps_stops_early(oracle, golden):
    """The reference's fp32 EPS = 1e-4 (v4:18) stops before the true optimum on
    larger LPs — the reason the build defaults to 1e-7."""
    case = [c for c in golden["cases"] if c["m"] == 512][0]
    A, b, c = oracle.generate(case["m"], case["n"], case["seed"])
    r = oracle.solve(A, b, c, eps=1e-4)
    assert r.pivots <= case["oracle_pivots"]
    assert r.z <= case["highs_z"] * (1 + 1e-12)


def test_thread_count_invariance(oracle):
    A, b, c = oracle.generate(96, 300, 9)
    r1 = oracle.solve(A, b, c, threads=1, want_state=True)
    r4 = oracle.solve(A, b, c, threads=4, want_state=True)
    assert r1.z == r4.z and np.array_equal(r1.binv, r4.binv) and r1.pivots == r4.pivots


def test_unbounded(oracle):
    m, n = 2, 4
    A = np.array([[-1.0, -1.0], [1.0, 2.0], [1.0, 0.0], [0.0, 1.0]])  # (n, m) columns
    b = np.array([1.0, 1.0])
    c = np.array([1.0, 0.0, 0.0, 0.0])
    r = oracle.solve(A, b, c)
    assert r.status == oracle.UNBOUNDED and r.pivots == 0


def test_invariants_after_pivots(oracle):
    A, b, c = oracle.generate(80, 240, 2)
    r = oracle.solve(A, b, c, max_iter=30, want_state=True)
    B = A[r.b_ixs].T
    assert np.allclose(r.binv @ B, np.eye(80), atol=1e-10)
    assert np.allclose(r.binv @ b, r.x_b, rtol=1e-11)
    assert np.allclose(c[r.b_ixs] @ r.binv, r.y, rtol=1e-11)


def test_price_matches_numpy(oracle):
    A, b, c = oracle.generate(50, 200, 1)
    y = np.linspace(-1, 1, 50)
    e = oracle.price(A, c, y)
    assert np.allclose(e, A @ y - c, rtol=1e-13, atol=1e-13)


def test_reader_rejects_m_gt_n(oracle, tmp_path):
    p = tmp_path / "bad.txt"
    p.write_text("3 2\n1 2\n3 4\n5 6\n1 1 1\n1 1\n")
    with pytest.raises(ValueError):
        oracle.read_lp_text(str(p))


# ---------------------------------------------------------------- §8f row 4
def test_ratio_rules_agree_on_nondegenerate(oracle):
    A, b, c = oracle.generate(128, 512, 0)
    ref = oracle.solve(A, b, c, trace_cap=400)
    for rule in (oracle.RATIO_GUARDED, oracle.RATIO_HARRIS):
        r = oracle.solve(A, b, c, ratio=rule, trace_cap=400)
        assert r.pivots == ref.pivots and list(r.b_ixs) == list(ref.b_ixs)
        assert np.array_equal(r.trace_q, ref.trace_q)


@pytest.mark.parametrize("m,n,seed", [(96, 300, 1), (128, 512, 2), (300, 900, 4)])
def test_ratio_rules_on_degenerate_lps(oracle, m, n, seed):
    """The reference rule (v4:199-208: no pivot guard, no x_b >= 0 filter)
    loses feasibility on these degenerate LPs; the guarded and Harris rules
    reach the HiGHS optimum."""
    from lpgen import degenerate_lp, highs_opt

    A, b, c = degenerate_lp(m, n, seed)
    z_star = highs_opt(A, b, c)
    cap = 20 * n
    r0 = oracle.solve(A, b, c, max_iter=cap)
    assert not (r0.status == oracle.OPTIMUM_FOUND and abs(r0.z - z_star) <= 1e-6 * abs(z_star))
    for rule in (oracle.RATIO_GUARDED, oracle.RATIO_HARRIS):
        r = oracle.solve(A, b, c, ratio=rule, max_iter=cap)
        assert r.status == oracle.OPTIMUM_FOUND
        assert abs(r.z - z_star) <= 1e-9 * abs(z_star)
        assert r.x_b.min() >= -1e-9


def test_reinvert_matches_numpy_inverse(oracle):
    A, b, c = oracle.generate(120, 400, 5)
    r = oracle.solve(A, b, c, max_iter=90, want_state=True)
    Bi, xb, y = oracle.reinvert(A, b, c, r.b_ixs)
    B = A[r.b_ixs].T
    ref = np.linalg.inv(B)
    assert np.max(np.abs(Bi - ref)) <= 1e-11 * max(1.0, np.max(np.abs(ref)))
    assert np.allclose(xb, ref @ b, rtol=1e-11, atol=1e-11)
    assert np.allclose(y, c[r.b_ixs] @ ref, rtol=1e-11, atol=1e-11)
    assert np.max(np.abs(Bi - r.binv)) <= 1e-11 * max(1.0, np.max(np.abs(ref)))


def test_reinvert_rejects_bad_bases(oracle):
    m, n = 30, 90
    A, b, c = oracle.generate(m, n, 0)
    basis = np.arange(n - m, n)
    dup = basis.copy()
    dup[0] = dup[1]
    with pytest.raises(ValueError, match="bad basis"):
        oracle.reinvert(A, b, c, dup)
    A2 = A.copy()
    A2[1] = A2[0]
    sing = basis.copy()
    sing[2], sing[7] = 0, 1
    with pytest.raises(ValueError, match="singular"):
        oracle.reinvert(A2, b, c, sing)
    Bi, xb, y = oracle.reinvert(A, b, c, basis)  # the slack basis: identity
    assert np.array_equal(Bi, np.eye(m)) and np.array_equal(xb, b)


def test_refactor_every_keeps_path(oracle):
    A, b, c = oracle.generate(150, 450, 3)
    ref = oracle.solve(A, b, c, trace_cap=1000)
    r = oracle.solve(A, b, c, refactor_every=20, trace_cap=1000)
    assert r.pivots == ref.pivots and np.array_equal(r.trace_q, ref.trace_q)
    assert abs(r.z - ref.z) <= 1e-11 * abs(ref.z)


def test_devex_reaches_optimum(oracle, golden):
    from lpgen import degenerate_lp, highs_opt

    for case in golden["cases"][:9]:
        A, b, c = oracle.generate(case["m"], case["n"], case["seed"])
        r = oracle.solve(A, b, c, pricing=oracle.PRICING_DEVEX)
        assert r.status == oracle.OPTIMUM_FOUND
        assert abs(r.z - case["highs_z"]) <= 1e-9 * abs(case["highs_z"])
        assert sorted(int(j) for j in r.b_ixs) == case["highs_basis"]
    A, b, c = degenerate_lp(300, 900, 4)
    z_star = highs_opt(A, b, c)
    d = oracle.solve(A, b, c, ratio=oracle.RATIO_GUARDED)
    x = oracle.solve(A, b, c, ratio=oracle.RATIO_GUARDED, pricing=oracle.PRICING_DEVEX)
    assert abs(x.z - z_star) <= 1e-9 * abs(z_star)
    assert x.pivots < d.pivots  # Devex needs fewer pivots on this degenerate LP (347 vs 1124)


def _exact_se_weights(A, basis, binv):
    """gamma_j = 1 + ||B^-1 A_j||^2 for the non-basic columns (the definition)."""
    n = A.shape[0]
    bs = set(int(j) for j in basis)
    nb = np.array([j for j in range(n) if j not in bs])
    return nb, 1.0 + np.sum((binv @ A[nb].T) ** 2, axis=0)


@pytest.mark.parametrize("m,n,seed,k", [(120, 480, 1, 30), (200, 800, 3, 60), (160, 640, 7, 100)])
def test_steepest_edge_recurrence_is_exact(oracle, m, n, seed, k):
    """The Goldfarb-Reid recurrence (se_choose) keeps the exact weights: after
    k steepest-edge pivots they equal 1 + ||B^-1 A_j||^2 from the final B^-1
    within 1e-10 (relative)."""
    A, b, c = oracle.generate(m, n, seed)
    r = oracle.solve(A, b, c, pricing=oracle.PRICING_STEEPEST, max_iter=k, want_state=True)
    assert r.pivots >= min(k, 30)
    nb, ex = _exact_se_weights(A, r.b_ixs, r.binv)
    assert np.max(np.abs(r.weights[nb] - ex) / ex) <= 1e-10


def test_steepest_edge_reaches_optimum(oracle, golden):
    """Steepest edge reaches the HiGHS optima (golden cases; a degenerate LP
    with the guarded ratio test), with fewer pivots than Dantzig and Devex on
    the degenerate LP."""
    from lpgen import degenerate_lp, highs_opt

    for case in golden["cases"][:9]:
        A, b, c = oracle.generate(case["m"], case["n"], case["seed"])
        r = oracle.solve(A, b, c, pricing=oracle.PRICING_STEEPEST)
        assert r.status == oracle.OPTIMUM_FOUND
        assert abs(r.z - case["highs_z"]) <= 1e-9 * abs(case["highs_z"])
        assert sorted(int(j) for j in r.b_ixs) == case["highs_basis"]
    A, b, c = degenerate_lp(300, 900, 4)
    z_star = highs_opt(A, b, c)
    d = oracle.solve(A, b, c, ratio=oracle.RATIO_GUARDED)
    x = oracle.solve(A, b, c, ratio=oracle.RATIO_GUARDED, pricing=oracle.PRICING_DEVEX)
    s = oracle.solve(A, b, c, ratio=oracle.RATIO_GUARDED, pricing=oracle.PRICING_STEEPEST)
    assert s.status == oracle.OPTIMUM_FOUND and abs(s.z - z_star) <= 1e-9 * abs(z_star)
    assert s.pivots < d.pivots and s.pivots <= x.pivots


def test_steepest_edge_refactor_keeps_weights(oracle):
    """Reinversion changes B^-1's bits, not the weights' recurrence: the same
    optimum, weights still exact."""
    A, b, c = oracle.generate(150, 450, 3)
    r = oracle.solve(A, b, c, pricing=oracle.PRICING_STEEPEST, refactor_every=20, want_state=True, max_iter=70)
    nb, ex = _exact_se_weights(A, r.b_ixs, r.binv)
    assert np.max(np.abs(r.weights[nb] - ex) / ex) <= 1e-10

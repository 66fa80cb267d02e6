"""GPU: the compact FTRAN operand (Params::bc: B_w stored by its non-unit
columns, gathered after every fold) against the dense B_w stream
(SPX_DENSE_FTRAN=1).  The two sum B_w[i,:].A_p in different orders, so they
agree within rounding: the same pivot path, states within 1e-10, the same
optimum.  Within the compact form every dispatch and geometry gives the
same bits."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


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


def _run(spx, dense, k, **kw):
    with _env(SPX_DENSE_FTRAN="1" if dense else "0"):
        with spx.Context(trace=4096, **kw) as ctx:
            st, piv = ctx.iterate(k)
            s = ctx.state(binv=True)
            tr = ctx.trace()
            r = ctx.solve()
            return piv, s, tr, r


def _close(a, b, tol=1e-10):
    return np.max(np.abs(a - b)) <= tol * max(1.0, np.max(np.abs(b)))


@pytest.mark.parametrize("window,m,n,seed,k", [(16, 300, 1200, 5, 200), (64, 512, 2048, 1, 400),
                                               (64, 1024, 4096, 0, 300), (32, 256, 1024, 7, 250)])
def test_compact_matches_dense_ftran(spx, window, m, n, seed, k):
    a = _run(spx, False, k, m=m, n=n, seed=seed, window=window, persist=False)
    d = _run(spx, True, k, m=m, n=n, seed=seed, window=window, persist=False)
    assert a[0] == d[0] == k
    assert np.array_equal(a[1]["b_ixs"], d[1]["b_ixs"])
    assert np.array_equal(a[2], d[2])  # the same (p, q) per pivot
    for key in ("x_b", "y", "binv"):
        assert _close(a[1][key], d[1][key]), key
    assert a[3].status == d[3].status and a[3].pivots == d[3].pivots
    assert abs(a[3].z - d[3].z) <= 1e-9 * abs(d[3].z)


@pytest.mark.parametrize("kw", [dict(graph_batch=-1), dict(update_rows=2), dict(update_block=256),
                                dict(refactor_every=100)], ids=["eager", "rows2", "block256", "reinvert"])
def test_compact_same_bits_every_dispatch(spx, kw):
    base = dict(m=400, n=1600, seed=2, window=16, persist=False)
    ref = _run(spx, False, 300, **base)
    got = _run(spx, False, 300, **base, **kw)
    if "refactor_every" in kw:  # a reinverted B_w has its own bits: same path, close values
        assert np.array_equal(got[1]["b_ixs"], ref[1]["b_ixs"])
        assert _close(got[1]["x_b"], ref[1]["x_b"], 1e-9)
        assert got[3].pivots == ref[3].pivots and abs(got[3].z - ref[3].z) <= 1e-9 * abs(ref[3].z)
        return
    for key in ("b_ixs", "x_b", "binv"):
        assert np.array_equal(got[1][key], ref[1][key]), key
    if "update_rows" in kw:
        # two rows per wave group the ratio-test sum T = sum c_B alpha (and so
        # s_y, y) differently, with the dense B_w stream as well
        assert _close(got[1]["y"], ref[1]["y"], 1e-12)
        assert got[3].pivots == ref[3].pivots and abs(got[3].z - ref[3].z) <= 1e-12 * abs(ref[3].z)
    else:
        assert np.array_equal(got[1]["y"], ref[1]["y"])
        assert got[3].pivots == ref[3].pivots and got[3].z == ref[3].z


def test_compact_set_basis_and_oracle(spx, oracle):
    """Warm start (reinversion builds the column list from the basis), then
    the solve reaches the oracle's optimum."""
    m, n, seed = 300, 1200, 9
    A, b, c = oracle.generate(m, n, seed)
    o = oracle.solve(A, b, c, eps=1e-7)
    with spx.Context(A, b, c, window=16, persist=False) as ctx:
        ctx.iterate(150)
        basis = ctx.state()["b_ixs"].copy()
    with spx.Context(A, b, c, window=16, persist=False) as ctx:
        ctx.set_basis(basis)
        r = ctx.solve()
    assert r.status == spx.SolveStatus.OptimumFound
    assert abs(r.z - o.z) <= 1e-9 * abs(o.z)


def test_compact_blocks_of_columns(spx, monkeypatch):
    """m = 9000 (L > 8,192): the A_p gather runs in LDS blocks once S passes
    8,192 columns; here a reinversion onto a basis of 8,500 structural
    columns makes S = 8,500 at once.  Same pivots and close values as the
    dense stream."""
    m, n, seed = 9000, 18000, 4
    with spx.Context(m=m, n=n, seed=seed, window=16, persist=False) as ctx:
        basis = np.arange(n - m, n, dtype=np.int64)
        basis[:8500] = np.arange(8500)  # structural columns 0..8499 in rows 0..8499
        try:
            ctx.set_basis(basis)
        except spx.SimplexError:
            pytest.skip("that basis is singular for this seed")
        assert ctx.ftran_cols() == 8500
        ctx.iterate(40)
        a = ctx.state()
    monkeypatch.setenv("SPX_DENSE_FTRAN", "1")
    with spx.Context(m=m, n=n, seed=seed, window=16, persist=False) as ctx:
        ctx.set_basis(basis)
        assert ctx.ftran_cols() == m
        ctx.iterate(40)
        d = ctx.state()
    assert np.array_equal(a["b_ixs"], d["b_ixs"])
    assert _close(a["x_b"], d["x_b"], 1e-8)


@pytest.mark.parametrize("window", [16, 64])
def test_compact_persistent_loop_same_bits(spx, window):
    """The persistent loop kernel (k_loop) runs the compact FTRAN with the
    same per-lane order as k_update: the same alpha bits (so the same U and
    B^-1) as two-kernel passes.  Its ratio-test partials group T = sum c_B
    alpha by its own workgroups, so s_y and y agree to rounding (as with the
    dense stream)."""
    base = dict(m=600, n=2400, seed=3, window=window)
    a = _run(spx, False, 300, persist=True, **base)
    b = _run(spx, False, 300, persist=False, **base)
    for key in ("b_ixs", "binv"):
        assert np.array_equal(a[1][key], b[1][key]), key
    for key in ("x_b", "y"):
        assert _close(a[1][key], b[1][key], 1e-12), key
    assert a[3].pivots == b[3].pivots and abs(a[3].z - b[3].z) <= 1e-12 * abs(b[3].z)


@pytest.mark.parametrize("kw", [dict(m=257, n=1001, seed=6, window=16),
                                dict(m=300, n=1200, seed=8, window=32, pricing=1),
                                dict(m=300, n=1200, seed=8, window=16, ratio_test=2),
                                dict(m=300, n=1200, seed=8, window=16, ratio_test=1)],
                         ids=["odd-m", "devex", "harris", "guarded"])
def test_compact_rules_and_odd_sizes(spx, kw):
    """Odd m (a half-used last chunk), Devex pricing and the guarded / Harris
    ratio tests: the compact operand takes the dense stream's pivots."""
    a = _run(spx, False, 150, persist=False, **kw)
    d = _run(spx, True, 150, persist=False, **kw)
    assert np.array_equal(a[1]["b_ixs"], d[1]["b_ixs"])
    assert np.array_equal(a[2], d[2])
    assert _close(a[1]["x_b"], d[1]["x_b"], 1e-9)
    assert a[3].status == d[3].status and a[3].pivots == d[3].pivots
    assert abs(a[3].z - d[3].z) <= 1e-9 * max(1.0, abs(d[3].z))


@pytest.mark.parametrize("rows,m,n,window", [(2, 401, 1604, 16), (4, 257, 1028, 16), (8, 401, 1604, 64),
                                             (4, 403, 1612, 8), (2, 301, 1204, 64)],
                         ids=["r2-m401", "r4-m257", "r8-m401-w64", "r4-m403-w8", "r2-m301-w64"])
def test_compact_partial_last_wave(spx, rows, m, n, window):
    """m not a multiple of the rows per wave (nor of 16): the last wave of
    k_update holds fewer than R rows, and its prefetched compact chunks and
    unit terms must still belong to its own rows.  The
    compact operand takes the dense stream's pivot path, with R rows per
    wave and with one."""
    kw = dict(m=m, n=n, seed=11, window=window, persist=False)
    a = _run(spx, False, 200, update_rows=rows, **kw)
    d = _run(spx, True, 200, update_rows=rows, **kw)
    one = _run(spx, False, 200, **kw)
    assert np.array_equal(a[2], d[2]) and np.array_equal(a[2], one[2])
    assert np.array_equal(a[1]["b_ixs"], d[1]["b_ixs"])
    for key in ("x_b", "binv"):
        assert _close(a[1][key], d[1][key], 1e-10), key
        assert np.array_equal(a[1][key], one[1][key]), key  # alpha has the per-lane order of R = 1
    assert a[3].status == d[3].status and a[3].pivots == d[3].pivots
    assert abs(a[3].z - d[3].z) <= 1e-9 * max(1.0, abs(d[3].z))


@pytest.mark.parametrize("kw", [dict(m=401, n=1604, seed=11, window=64), dict(m=400, n=1600, seed=2, window=16),
                                dict(m=1024, n=4096, seed=0, window=64), dict(m=300, n=1200, seed=8, window=32, pricing=1),
                                dict(m=257, n=1001, seed=6, window=16, ratio_test=2)],
                         ids=["m401-w64", "m400-w16", "m1024-w64", "devex", "harris"])
def test_compact_entry_kernel_same_bits(spx, kw):
    """k_ftran_bc (the one-row-per-wave compact pass with every p-independent
    load at kernel entry) against k_update<..., BC> (SPX_FTRAN_BC_ENTRY=0):
    the same arithmetic in the same order, so the same bits everywhere."""
    a = _run(spx, False, 200, persist=False, **kw)
    with _env(SPX_FTRAN_BC_ENTRY="0"):
        b = _run(spx, False, 200, persist=False, **kw)
    assert np.array_equal(a[2], b[2])
    for key in ("b_ixs", "x_b", "y", "binv"):
        assert np.array_equal(a[1][key], b[1][key]), key
    assert a[3].pivots == b[3].pivots and a[3].z == b[3].z


@pytest.mark.parametrize("rpw", [2, 4])
@pytest.mark.parametrize("kw", [dict(m=2051, n=6000, seed=5, window=64), dict(m=4096, n=16384, seed=0),
                                dict(m=2304, n=9000, seed=3, window=16)],
                         ids=["m2051-w64", "C3", "m2304-w16"])
def test_ftran_rows_per_wave_same_bits(spx, kw, rpw):
    """k_ftran_bc with RPW rows per wave (SPX_FTRAN_RPW; the deferred tail's
    form): each workgroup covers RPW of the one-row grid's partial slots with
    the same rows and the same merges, so states, traces and optima are those
    of one row per wave bit for bit -- including a last workgroup whose slots
    run past the grid (m = 2051: 257 slots) and a sliver of a last wave."""
    a = _run(spx, False, 200, persist=False, **kw)
    with _env(SPX_FTRAN_RPW=str(rpw)):
        with spx.Context(persist=False, **kw) as ctx:
            assert ctx.config()["defer_tail"] == 1
        b = _run(spx, False, 200, persist=False, **kw)
    assert np.array_equal(a[2], b[2])
    for key in ("b_ixs", "x_b", "y", "binv"):
        assert np.array_equal(a[1][key], b[1][key]), key
    assert a[3].pivots == b[3].pivots and a[3].z == b[3].z


@pytest.mark.parametrize("kw", [dict(m=401, n=1604, seed=11, window=64), dict(m=400, n=1600, seed=2, window=16),
                                dict(m=1024, n=4096, seed=0, window=64), dict(m=300, n=1200, seed=8, window=32, pricing=1),
                                dict(m=257, n=1001, seed=6, window=8, ratio_test=2),
                                dict(m=300, n=1200, seed=3, window=64, pricing=2),
                                dict(m=2051, n=6000, seed=5, window=64), dict(m=4096, n=16384, seed=0)],
                         ids=["m401-w64", "m400-w16", "m1024-w64", "devex", "harris-w8", "steepest", "m2051", "C3"])
def test_compact_fold_same_bits(spx, kw):
    """The compact fold (k_cfold: the listed columns of B_w only, R rebuilt
    one lane per column, the fold's MFMA tiles, the dense B_w kept by a
    scatter) against the dense fold plus the gather (SPX_DENSE_FOLD=1): the
    same R, the same tiles, so the same bits -- states, B^-1, traces and the
    optimum -- through many folds, lists growing past several pitches of 64
    and (at optimality) hundreds of columns."""
    a = _run(spx, False, 300, persist=False, **kw)
    with _env(SPX_DENSE_FOLD="1"):
        b = _run(spx, False, 300, persist=False, **kw)
    assert np.array_equal(a[2], b[2])
    for key in ("b_ixs", "x_b", "y", "binv"):
        assert np.array_equal(a[1][key], b[1][key]), key
    assert a[3].status == b[3].status and a[3].pivots == b[3].pivots and a[3].z == b[3].z


def test_compact_fold_persistent_and_reinversion(spx, oracle):
    """The compact fold between persistent k_loop launches, and a reinversion
    (which regathers the operand into buffer 0 whichever buffer was active)
    in the middle: the dense fold's bits, and the oracle's optimum."""
    kw = dict(m=300, n=1200, seed=3, window=16)
    outs = []
    for dense in ("0", "1"):
        with _env(SPX_DENSE_FOLD=dense):
            with spx.Context(persist=True, trace=4096, **kw) as ctx:
                ctx.iterate(37)
                ctx.reinvert()
                ctx.iterate(41)
                s = ctx.state(binv=True)
                r = ctx.solve()
                outs.append((s, ctx.trace(), r))
    (sa, ta, ra), (sb, tb, rb) = outs
    assert np.array_equal(ta, tb)
    for key in ("b_ixs", "x_b", "y", "binv"):
        assert np.array_equal(sa[key], sb[key]), key
    A, b, c = oracle.generate(kw["m"], kw["n"], kw["seed"])
    o = oracle.solve(A, b, c, eps=1e-7)
    assert ra.status == spx.SolveStatus.OptimumFound and abs(ra.z - o.z) <= 1e-9 * abs(o.z)


@pytest.mark.parametrize("kw,env", [(dict(update_rows=2), {}), (dict(), dict(SPX_FTRAN_BC_ENTRY="0"))],
                         ids=["rows2", "k_update-bc"])
def test_compact_fold_wide_list_k_update(spx, kw, env):
    """k_update<..., BC> (update_rows > 1, or SPX_FTRAN_BC_ENTRY=0) with a
    column list past BC_PF2 chunks (S > 512) after odd and even numbers of
    compact folds: every chunk of a row comes from the active operand buffer
    at its pitch (the chunks past the prefetch were read
    from buffer 0), so the bits are those of the dense fold plus the gather
    (SPX_DENSE_FOLD=1, one buffer)."""
    m, n, seed = 2048, 8192, 7
    basis = np.arange(n - m, n, dtype=np.int64)
    basis[:600] = np.arange(600)  # structural columns 0..599 in rows 0..599: S = 600
    outs = []
    for dense in ("0", "1"):
        with _env(SPX_DENSE_FOLD=dense, **env):
            with spx.Context(m=m, n=n, seed=seed, window=16, persist=False, trace=4096, **kw) as ctx:
                try:
                    ctx.set_basis(basis)
                except spx.SimplexError:
                    pytest.skip("that basis is singular for this seed")
                assert ctx.ftran_cols() == 600
                outs.append([])
                for k in (15, 15, 15, 52):  # folds before each: 0, 1, 2, 3 (odd and even buffers)
                    st, piv = ctx.iterate(k)
                    s = ctx.state(binv=True)
                    outs[-1].append((piv, s))
                outs[-1].append(ctx.trace())
    a, b = outs
    assert a[-1][0].size > 60
    assert np.array_equal(a[-1][0], b[-1][0]) and np.array_equal(a[-1][1], b[-1][1])
    for (pa, sa), (pb, sb) in zip(a[:-1], b[:-1]):
        assert pa == pb
        for key in ("b_ixs", "x_b", "y", "binv"):
            assert np.array_equal(sa[key], sb[key]), key

"""GPU: the MINLOC exchange through peer mailboxes (spx_mbox_export /
spx_mbox_attach, k_exchange) instead of the RCCL all-gather.

- One rank (SPX_FLAG_COMM1, its own mailbox only): eager and captured
  passes, and the stepping API, bit-identical to the single-rank loop.
- Two and three processes on ONE GPU (ranks of a column-sharded group that
  share the device; RCCL refuses two ranks on one device, the mailboxes do
  not): each rank maps the others' mailboxes over IPC, and every rank reaches
  the single-rank state bit for bit, then the oracle's optimum.  This runs
  the multi-process sharded path on hardware: separate processes, separate
  contexts, candidate records crossing between them every pass."""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.parametrize("fused", ["1", "0"], ids=["fused", "k_exchange"])
@pytest.mark.parametrize("window", [-1, 16])
@pytest.mark.parametrize("graph_batch", [-1, 16])
def test_mbox_one_rank_matches_single_rank(spx, monkeypatch, window, graph_batch, fused):
    """fused: window passes exchange inside k_price / k_ftran_bc (the
    default); k_exchange: SPX_MBOX_FUSED=0, one exchange kernel per pass."""
    monkeypatch.setenv("SPX_MBOX_FUSED", fused)
    m, n, seed, k = 300, 1200, 3, 150
    with spx.Context(m=m, n=n, seed=seed, window=window, persist=False) as ref:
        ref.iterate(k)
        rs = ref.state(binv=True)
        rp = ref.price()
    with spx.Context(m=m, n=n, seed=seed, window=window, comm1=True, graph_batch=graph_batch) as ctx:
        ctx.mbox_attach([ctx.mbox_export()])
        st, piv = ctx.iterate(k)
        cfg = ctx.config()
        s = ctx.state(binv=True)
        p = ctx.price()
    assert piv == k
    assert cfg["mbox_fused"] == (1 if fused == "1" and window > 0 else 0)
    if graph_batch > 0:  # a plain kernel: the capture never falls back
        assert cfg["graph_batch"] == (16 if window < 0 else 30)
    for key in ("b_ixs", "x_b", "y", "binv"):
        assert np.array_equal(s[key], rs[key]), key
    assert p == rp


@pytest.mark.parametrize("graph_batch", [-1, 64])
def test_mbox_one_rank_fused_deferred_tail(spx, graph_batch):
    """The fused exchange with the deferred ratio-test tail (m = 2048, compact
    window passes, 512-thread FTRAN workgroups): k_price's pricing tail stores
    the record into the mailbox, k_ftran_bc polls it, no k_exchange launch;
    through two folds the state is the single-rank loop's bit for bit, and so
    are a reset and a second run (the reset advances the tag epoch, so the
    first run's words cannot match the second's)."""
    m, n, seed, k = 2048, 6144, 5, 140
    with spx.Context(m=m, n=n, seed=seed, window=64, persist=False) as ref:
        ref.iterate(k)
        rs = ref.state(binv=True)
    with spx.Context(m=m, n=n, seed=seed, window=64, comm1=True, graph_batch=graph_batch) as ctx:
        ctx.mbox_attach([ctx.mbox_export()])
        cfg = ctx.config()
        assert cfg["mbox_fused"] == 1 and cfg["defer_tail"] == 1
        for rep in range(2):
            if rep:
                ctx.reset()
            st, piv = ctx.iterate(k)
            assert piv == k
            s = ctx.state(binv=True)
            for key in ("b_ixs", "x_b", "y", "binv"):
                assert np.array_equal(s[key], rs[key]), (rep, key)


def test_mbox_attach_errors(spx):
    with spx.Context(m=64, n=256, seed=0) as ctx:  # one rank, no COMM1: no exchange at all
        with pytest.raises(spx.SimplexError, match="nranks > 1"):
            ctx.mbox_export()
    with spx.Context(m=64, n=256, seed=0, comm1=True) as ctx:
        with pytest.raises(spx.SimplexError, match="export first"):
            ctx.mbox_attach([bytes(64)])
        with pytest.raises(ValueError):
            ctx.mbox_attach([b"short"])


@pytest.mark.parametrize("G,window,graph_batch", [(2, -1, 16), (2, 16, 16), (2, 64, -1), (3, 16, 16)])
def test_mbox_processes_share_one_gpu(spx, oracle, tmp_path, G, window, graph_batch):
    m, n, seed, k = 300, 1200, 3, 120
    with spx.Context(m=m, n=n, seed=seed, window=window, persist=False) as ref:
        ref.iterate(k)
        rs = ref.state(binv=True)
        rr = ref.solve()
    env = dict(os.environ)
    procs = [subprocess.Popen([sys.executable, "-u", os.path.join(HERE, "mbox_rank.py"), str(tmp_path), str(g), str(G),
                               str(m), str(n), str(seed), str(window), str(k), str(graph_batch)],
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, env=env) for g in range(G)]
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=100)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append(out.decode(errors="replace"))
    for g, p in enumerate(procs):
        assert p.returncode == 0, f"rank {g}:\n{outs[g][-3000:]}"
    A, b, c = oracle.generate(m, n, seed)
    o = oracle.solve(A, b, c, eps=1e-7)
    for g in range(G):
        r = np.load(tmp_path / f"r{g}.npz")
        assert int(r["piv"]) == k
        for key in ("b_ixs", "x_b", "y", "binv"):
            assert np.array_equal(r[key], rs[key]), (g, key)
        assert int(r["status"]) == int(spx.SolveStatus.OptimumFound)
        assert int(r["pivots"]) == rr.pivots == o.pivots
        assert float(r["z"]) == rr.z
        assert abs(rr.z - o.z) <= 1e-9 * abs(o.z)
        assert int(r["mbox_fused"]) == 0  # ranks sharing one GPU keep the k_exchange launch


@pytest.mark.parametrize("graph_batch", [16, -1])
def test_mbox_processes_deferred_tail(spx, tmp_path, graph_batch):
    """m = 2048 (512-thread FTRAN workgroups, compact window passes): the
    ranks run the deferred ratio-test tail -- each reduces its own replicated
    FTRAN partials in the next pricing pass, whose pricing tail stays in the
    launch for the exchange -- and reach the single-rank state bit for bit
    through two folds."""
    m, n, seed, k, G = 2048, 6144, 5, 140, 2
    with spx.Context(m=m, n=n, seed=seed, window=64, persist=False) as ref:
        assert ref.config()["defer_tail"] == 1
        ref.iterate(k)
        rs = ref.state(binv=True)
        rz = ref.objective()
    procs = [subprocess.Popen([sys.executable, "-u", os.path.join(HERE, "mbox_rank.py"), str(tmp_path), str(g), str(G),
                               str(m), str(n), str(seed), "64", str(k), str(graph_batch), "0"],
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, env=dict(os.environ)) for g in range(G)]
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=100)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append(out.decode(errors="replace"))
    for g, p in enumerate(procs):
        assert p.returncode == 0, f"rank {g}:\n{outs[g][-3000:]}"
    for g in range(G):
        r = np.load(tmp_path / f"r{g}.npz")
        assert int(r["defer_tail"]) == 1
        assert int(r["mbox_fused"]) == 0  # (peers on this device: k_exchange, see spx_mbox_attach)
        assert int(r["piv"]) == k
        for key in ("b_ixs", "x_b", "y", "binv"):
            assert np.array_equal(r[key], rs[key]), (g, key)
        assert float(r["z"]) == rz


@pytest.mark.parametrize("pricing", [1, 2], ids=["devex", "steepest"])
def test_mbox_processes_weighted_pricing(spx, tmp_path, pricing):
    """Devex and steepest edge across two processes on one GPU (mailbox
    exchange, captured passes): each record carries its winner's reduced cost
    and weight; every rank reaches the single-rank state after K pivots and
    the single rank's optimum, bit for bit."""
    m, n, seed, k, G = 300, 1200, 8, 90, 2
    with spx.Context(m=m, n=n, seed=seed, window=64, pricing=pricing) as ref:
        ref.iterate(k)
        rs = ref.state(binv=True)
        rr = ref.solve()
    procs = [subprocess.Popen([sys.executable, "-u", os.path.join(HERE, "mbox_rank.py"), str(tmp_path), str(g), str(G),
                               str(m), str(n), str(seed), "64", str(k), "16", "1", str(pricing)],
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, env=dict(os.environ)) for g in range(G)]
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=100)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append(out.decode(errors="replace"))
    for g, p in enumerate(procs):
        assert p.returncode == 0, f"rank {g}:\n{outs[g][-3000:]}"
    assert rr.status == spx.SolveStatus.OptimumFound
    for g in range(G):
        r = np.load(tmp_path / f"r{g}.npz")
        assert int(r["piv"]) == k
        for key in ("b_ixs", "x_b", "y", "binv"):
            assert np.array_equal(r[key], rs[key]), (g, key)
        assert int(r["status"]) == int(spx.SolveStatus.OptimumFound)
        assert int(r["pivots"]) == rr.pivots
        assert float(r["z"]) == rr.z

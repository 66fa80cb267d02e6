"""GPU: the RCCL MINLOC path on one GPU (SPX_FLAG_COMM1: a one-rank
communicator, so ncclAllGather runs exactly as in the multi-GPU bench),
eager and captured into hipGraphs, against the plain single-rank loop —
bit-identical (a one-rank all-gather is a copy)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("window", [-1, 16])
@pytest.mark.parametrize("graph_batch", [-1, 16])
def test_comm1_matches_single_rank(spx, window, graph_batch):
    m, n, seed, k = 300, 1200, 3, 150
    with spx.Context(m=m, n=n, seed=seed, window=window, persist=False) as ref:
        ref.iterate(k)
        rs = ref.state(binv=True)
    with spx.Context(m=m, n=n, seed=seed, window=window, comm1=True, graph_batch=graph_batch) as ctx:
        ctx.attach_comm(spx.comm_unique_id())
        st, piv = ctx.iterate(k)
        cfg = ctx.config()
        s = ctx.state(binv=True)
        p, e, opt = ctx.price()
        q, st2 = ctx.pivot()
    assert piv == k
    if graph_batch > 0:
        assert cfg["graph_batch"] in (0, 16 if window < 0 else 30)  # 0: capture fell back to eager
    for key in ("b_ixs", "x_b", "y", "binv"):
        assert np.array_equal(s[key], rs[key]), key


def test_comm1_graph_capture_used(spx):
    """Report whether RCCL accepted the capture (the multi-GPU bench relies on it
    for launch-free passes; a refusal falls back to eager launches)."""
    with spx.Context(m=256, n=1024, seed=0, window=-1, comm1=True) as ctx:
        ctx.attach_comm(spx.comm_unique_id())
        ctx.iterate(40)
        cfg = ctx.config()
    print(f"RCCL capture: graph_batch={cfg['graph_batch']}")
    assert cfg["graph_batch"] in (0, 16)


@pytest.mark.parametrize("graph_batch", [-1, 16])
def test_comm1_row_shard_matches_single_rank(spx, oracle, graph_batch):
    """The multi-GPU bench's default (row-sharded B^-1, two all-gathers per
    pass, k_finalize_rs) through RCCL on one rank: same pivots as the single
    rank, values within 1e-9 (the sharded s_y is reassociated), the optimum
    of the oracle."""
    m, n, seed, k = 300, 1200, 3, 150
    with spx.Context(m=m, n=n, seed=seed, window=-1) as ref:
        ref.iterate(k)
        rs = ref.state(binv=True)
    with spx.Context(m=m, n=n, seed=seed, window=-1, comm1=True, row_shard=True, graph_batch=graph_batch) as ctx:
        ctx.attach_comm(spx.comm_unique_id())
        st, piv = ctx.iterate(k)
        s = ctx.state(binv=True)
        r = ctx.solve()
    assert piv == k and np.array_equal(s["b_ixs"], rs["b_ixs"])
    for key in ("x_b", "y", "binv"):
        a, b = s[key], rs[key]
        assert np.max(np.abs(a - b)) <= 1e-9 * max(1.0, np.max(np.abs(b))), key
    A, b, c = oracle.generate(m, n, seed)
    o = oracle.solve(A, b, c, eps=1e-7)
    assert r.status == spx.SolveStatus.OptimumFound and r.pivots == o.pivots
    assert abs(r.z - o.z) <= 1e-9 * abs(o.z)


def test_comm_info_one_rank(spx):
    """spx_comm_info on a one-rank communicator: RCCL itself reports 1 rank,
    rank 0, bound to the context's device; the bus id is the device's; the
    captured graphs hold the all-gathers (or report the eager fallback).
    check_ranks accepts it, and refuses a record claiming another world."""
    with spx.Context(m=256, n=1024, seed=0, window=-1, comm1=True) as ctx:
        before = ctx.comm_info()
        ctx.attach_comm(spx.comm_unique_id())
        ctx.iterate(40)
        inf = ctx.comm_info()
        cfg = ctx.config()
    assert before["rccl_nranks"] == -1 and before["rccl_rank"] == -1
    assert inf["rccl_nranks"] == 1 and inf["rccl_rank"] == 0
    assert inf["rccl_device"] == inf["device"] >= 0
    assert len(inf["bus_id"]) >= 7 and ":" in inf["bus_id"]
    assert inf["graph"] == (cfg["graph_batch"] > 0) and inf["graph"] != inf["graph_fallback"]
    print(f"comm_info: {inf}")
    spx.check_ranks([inf], 1)
    with pytest.raises(RuntimeError):
        spx.check_ranks([inf], 2)
    with pytest.raises(RuntimeError):
        spx.check_ranks([inf, dict(inf, rank=1)], 2, exchange="mbox")  # same bus id twice


def test_comm_info_single_rank_context(spx):
    """Without a communicator: -1 for the RCCL fields, the device's bus id,
    graph replay for the default dispatch."""
    with spx.Context(m=256, n=1024, seed=0, window=-1) as ctx:
        ctx.iterate(40)
        inf = ctx.comm_info()
    assert inf["rccl_nranks"] == -1 and inf["nranks"] == 1 and inf["graph"] and not inf["graph_fallback"]
    spx.check_ranks([inf], 1, exchange="none")

"""GPU: what the library enqueues around a timed region (spx_dispatch_stats,
spx_prepare).  bench.py times whole windows of passes; the batch hipGraph
(capture + instantiate + upload, about 13 ms at C3) must be built before the
timed region, never inside it: graph_builds stays constant across iterate()."""
import pytest

pytestmark = pytest.mark.gpu


def test_one_rank_graph_built_at_create(spx):
    with spx.Context(m=2048, n=8192, seed=0) as ctx:
        d0 = ctx.dispatch_stats()
        assert d0["graph_builds"] == 1  # spx_create captured it
        ctx.prepare()  # no-op
        ctx.iterate(5)
        ctx.iterate(ctx.dispatch_stats()["window"] - ctx.dispatch_stats()["window_pos"])
        ctx.iterate(3 * 63)
        d1 = ctx.dispatch_stats()
    assert d1["graph_builds"] == 1
    assert d1["graph_launches"] - d0["graph_launches"] == 3


def test_comm1_graph_built_by_prepare(spx):
    """With a communicator the graph can only be captured after attach_comm:
    prepare() builds it, and no iterate() builds another."""
    with spx.Context(m=2048, n=8192, seed=0, comm1=True) as ctx:
        ctx.attach_comm(spx.comm_unique_id())
        assert ctx.dispatch_stats()["graph_builds"] == 0
        ctx.prepare()
        d0 = ctx.dispatch_stats()
        fallback = ctx.comm_info()["graph_fallback"]
        assert d0["graph_builds"] == (0 if fallback else 1)
        ctx.iterate(5)
        ctx.iterate(ctx.dispatch_stats()["window"] - ctx.dispatch_stats()["window_pos"])
        ctx.iterate(2 * 63)
        d1 = ctx.dispatch_stats()
    assert d1["graph_builds"] == d0["graph_builds"]
    if not fallback:
        assert d1["graph_launches"] - d0["graph_launches"] == 2


def test_explicit_graph_built_at_create(spx):
    with spx.Context(m=1024, n=4096, seed=0) as ctx:
        assert ctx.config()["window"] == 0
        assert ctx.dispatch_stats()["graph_builds"] == 1
        ctx.iterate(100)
        assert ctx.dispatch_stats()["graph_builds"] == 1

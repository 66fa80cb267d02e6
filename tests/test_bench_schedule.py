"""bench.py's whole-solve call schedule (run_to_exit / calls_passes) on the
CPU: the spx_iterate chunk sizes are spx_solve's (spx_api.cpp: 16 pivots,
doubling to 2,048 per call), the loop stops at the first terminal status, and
the passes it reports after the optimum are the ones its last call enqueued."""
import os
import re
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


class FakeCtx:
    """spx_iterate's contract: iterate(k) enqueues k passes; the solve
    terminates (status 1) once `total` pivots are made, and later passes make
    no pivot; iterate(0) only reads the state."""

    def __init__(self, total):
        self.total, self.piv, self.calls = total, 0, []

    def iterate(self, k):
        self.calls.append(k)
        self.piv = min(self.piv + k, self.total)
        return (1 if self.piv >= self.total else 0), self.piv


@pytest.mark.parametrize("total", [1, 16, 17, 4080, 18291, 40000])
def test_run_to_exit_chunks(total):
    ctx = FakeCtx(total)
    armed = []
    st, piv, calls = bench.run_to_exit(ctx, lambda k, p: armed.append((k, p)))
    assert (st, piv) == (1, total)
    ks = ctx.calls[1:]
    assert ctx.calls[0] == 0 and len(ks) == calls
    expect = [min(16 << i, 2048) for i in range(calls)]
    assert ks == expect
    assert [k for k, _ in armed] == expect  # the watchdog is armed once per call, with its size
    after = bench.calls_passes(calls) - piv
    assert 0 <= after < ks[-1]  # only the last call runs past the optimum
    assert sum(ks) == bench.calls_passes(calls)


def test_schedule_matches_spx_solve():
    src = open(os.path.join(ROOT, "simplex_method_gpu_amd", "csrc", "spx_api.cpp")).read()
    body = src[src.index("int spx_solve("):]
    body = body[:body.index("\n}\n")]
    assert re.search(r"int64_t chunk = 16;", body)
    assert re.search(r"chunk = std::min<int64_t>\(chunk \* 2, 2048\);", body)

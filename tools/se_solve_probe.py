"""The steepest-edge C3 solve timed window by window (63-pivot iterate calls,
device-synced), to see where a build's whole-solve time goes; SPX_LIB picks
the build.  python tools/se_solve_probe.py"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import simplex_method_gpu_amd as spx  # noqa: E402

ts, piv = [], 0
t_start = time.perf_counter()
with spx.Context(m=4096, n=16384, seed=0, device=0, pricing=spx.PRICING_STEEPEST) as ctx:
    t_made = time.perf_counter()
    st = spx.SolveStatus.MaxIter
    while st == spx.SolveStatus.MaxIter:
        t0 = time.perf_counter()
        st, p = ctx.iterate(63)
        ts.append((p - piv, round(1e3 * (time.perf_counter() - t0), 3)))
        piv = p
print(json.dumps({"lib": os.environ.get("SPX_LIB", "default")[-30:], "create_ms": round(1e3 * (t_made - t_start), 1),
                  "pivots": piv, "total_ms": round(sum(t for _, t in ts), 2), "chunks_ms": [t for _, t in ts]}))

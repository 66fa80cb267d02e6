"""The C3 solve from the slack basis under three call schedules, alternating in
one process: iterate(4096) calls (the bench up to round 6), spx_solve's chunks
(16 doubling to 2,048: bench.run_to_exit) and one spx_solve call; Dantzig and
steepest edge.  python tools/solve_sched.py [reps]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

import simplex_method_gpu_amd as spx  # noqa: E402
from bench import calls_passes, run_to_exit  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2


def by4096(ctx):
    st, p = ctx.iterate(0)
    calls = 0
    while st == 0:
        st, p = ctx.iterate(4096)
        calls += 1
    return p, calls * 4096 - p


def chunks(ctx):
    _, p, calls = run_to_exit(ctx)
    return p, calls_passes(calls) - p


def one_call(ctx):
    r = ctx.solve()
    return r.pivots, None


for pricing in (spx.PRICING_DANTZIG, spx.PRICING_STEEPEST):
    for r in range(reps):
        for name, f in (("iterate4096", by4096), ("chunks", chunks), ("spx_solve", one_call)):
            with spx.Context(m=4096, n=16384, seed=0, device=0, pricing=pricing) as ctx:
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                piv, after = f(ctx)
                torch.cuda.synchronize()
                dt = time.perf_counter() - t0
                ds = ctx.dispatch_stats()
            print(json.dumps({"pricing": pricing, "schedule": name, "pivots": piv, "seconds": round(dt, 4),
                              "it_per_s": round(piv / dt), "passes_after_optimum": after,
                              "graph_passes": ds["graph_passes"], "eager_passes": ds["eager_passes"]}), flush=True)

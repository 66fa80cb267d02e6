"""Quick iteration-rate probe: graph-mode ms/iteration plus event-timed kernel
averages, for A/B comparisons of builds (SPX_LIB=...) or launch geometries.
    python tools/itbench.py [--m 4096 --n 16384 --k 200 --reps 3] [--kw '{"update_rows":1}']"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import simplex_method_gpu_amd as spx  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--m", type=int, default=4096)
ap.add_argument("--n", type=int, default=16384)
ap.add_argument("--k", type=int, default=200)
ap.add_argument("--warm", type=int, default=20)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--kw", default="{}")
ap.add_argument("--tag", default=os.environ.get("SPX_LIB", "default"))
a = ap.parse_args()
kw = json.loads(a.kw)
res = []
with spx.Context(m=a.m, n=a.n, seed=0, device=0, **kw) as ctx:
    ctx.iterate(a.warm)
    for _ in range(a.reps):
        t0 = time.perf_counter()
        st, p0 = ctx.iterate(0)
        st, p1 = ctx.iterate(a.k)
        res.append(1e3 * (time.perf_counter() - t0) / max(p1 - p0, 1))
with spx.Context(m=a.m, n=a.n, seed=0, device=0, timing=True, **kw) as ctx:
    ctx.iterate(a.warm)
    ctx.kernel_times()
    ctx.iterate(a.k)
    kt = ctx.kernel_times()
nl = max(kt["price_launches"], 1)
print(json.dumps({"tag": a.tag, "kw": kw, "ms_per_iter": [round(x, 4) for x in res],
                  "it_per_s": round(1e3 / min(res), 1),
                  "price_us": round(1e3 * kt["price_ms"] / nl, 2),
                  "update_us": round(1e3 * kt["update_ms"] / nl, 2)}), flush=True)

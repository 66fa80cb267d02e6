"""Time of spx_reinvert at a given size with a basis of `k` pivots (mostly
structural columns once k ~ m): python tools/reinv_bench.py [--m 4096 --n 16384 --k 5000]"""
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
ap.add_argument("--k", type=int, default=5000)
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--full", action="store_true", help="warm-start a basis of m structural columns (0..m-1) instead")
a = ap.parse_args()
with spx.Context(m=a.m, n=a.n, seed=0, device=0) as ctx:
    if a.full:
        import numpy as np
        t0 = time.perf_counter()
        ctx.set_basis(np.arange(a.m, dtype=np.int64))
        print(json.dumps({"set_basis_full_s": round(time.perf_counter() - t0, 4)}), flush=True)
        piv = 0
    else:
        st, piv = ctx.iterate(a.k)
    s = ctx.state()
    nstruct = int((s["b_ixs"] < a.n - a.m).sum())
    ts = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        ctx.reinvert()
        ts.append(time.perf_counter() - t0)
    z0 = ctx.objective()
print(json.dumps({"m": a.m, "n": a.n, "pivots": piv, "structural_basic": nstruct,
                  "reinvert_s": [round(t, 4) for t in ts], "z": z0}), flush=True)

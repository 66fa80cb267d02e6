"""C3 pass rate late in the solve, and whole-solve time, with non-basic slack
columns priced as unit vectors (default) or streamed (SPX_DENSE_SLACKS=1).
python tools/slack_late.py"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import simplex_method_gpu_amd as spx  # noqa: E402


def measure(dense):
    os.environ["SPX_DENSE_SLACKS"] = "1" if dense else "0"
    out = {"dense_slacks": int(dense)}
    with spx.Context(m=4096, n=16384, seed=0, device=0) as ctx:
        _, p = ctx.iterate(0)
        for at in (64, 2016, 4032, 6048):
            ctx.iterate(at - p)
            t0 = time.perf_counter()
            _, p0 = ctx.iterate(0)
            st, p = ctx.iterate(252)
            out[f"it_s_from_{p0}"] = round((p - p0) / (time.perf_counter() - t0), 1)
            out[f"nonbasic_slacks_at_{p0}"] = int((ctx.state()["b_ixs"] < 16384 - 4096).sum())
            if st != spx.SolveStatus.MaxIter:
                break
    with spx.Context(m=4096, n=16384, seed=0, device=0) as ctx:
        t0 = time.perf_counter()
        r = ctx.solve()
        out["solve_s"] = round(time.perf_counter() - t0, 3)
        out["pivots"] = r.pivots
        out["z"] = r.z
    return out


for r in range(2):
    for dense in (False, True):
        print(json.dumps(measure(dense)), flush=True)

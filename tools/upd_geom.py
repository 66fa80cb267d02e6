"""C3 eta-window passes per second over update geometries (k_update block x
rows per wave), graph replay, whole windows.  python tools/upd_geom.py"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import simplex_method_gpu_amd as spx  # noqa: E402


def rate(**kw):
    with spx.Context(m=4096, n=16384, seed=0, device=0, **kw) as ctx:
        ctx.iterate(64)
        best = 0.0
        for _ in range(3):
            t0 = time.perf_counter()
            _, p0 = ctx.iterate(0)
            _, p1 = ctx.iterate(252)
            best = max(best, (p1 - p0) / (time.perf_counter() - t0))
        return best, ctx.config()


for blk, rows in [(512, 1), (256, 1), (1024, 1), (512, 2), (1024, 2), (256, 4), (512, 4), (1024, 4), (256, 8), (512, 8)]:
    try:
        r, cfg = rate(update_block=blk, update_rows=rows)
        print(json.dumps({"update_block": blk, "update_rows": rows, "it_s": round(r, 1),
                          "grid": cfg["update_grid"]}), flush=True)
    except Exception as e:  # geometry refused by the library
        print(json.dumps({"update_block": blk, "update_rows": rows, "error": str(e)[:200]}), flush=True)

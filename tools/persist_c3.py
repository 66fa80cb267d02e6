"""C3 pass rate: two-kernel passes vs the persistent loop kernel, both with
the compact FTRAN operand.  python tools/persist_c3.py"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import simplex_method_gpu_amd as spx  # noqa: E402

for r in range(2):
    for persist in (False, True):
        with spx.Context(m=4096, n=16384, seed=0, device=0, window=64, persist=persist) as ctx:
            ctx.iterate(64)
            t0 = time.perf_counter()
            _, p0 = ctx.iterate(0)
            _, p1 = ctx.iterate(252)
            dt = time.perf_counter() - t0
            print(json.dumps({"persist": persist, "it_s": round((p1 - p0) / dt, 1),
                              "persistent": ctx.config()["persistent"]}), flush=True)

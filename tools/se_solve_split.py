"""The bench's steepest-edge C3 solve split into its parts: context creation,
the pivoting passes (iterate(0) then exactly the pivots the solve takes), and
the passes after the optimum that a bench-style iterate(4096) call still
enqueues (they price nothing); SPX_LIB picks the build.
python tools/se_solve_split.py [pricing] [pivots]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

import simplex_method_gpu_amd as spx  # noqa: E402

pricing = int(sys.argv[1]) if len(sys.argv) > 1 else spx.PRICING_STEEPEST
npiv = int(sys.argv[2]) if len(sys.argv) > 2 else 1554


def seg(f):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = f()
    torch.cuda.synchronize()
    return r, round(1e3 * (time.perf_counter() - t0), 3)


out = {"lib": os.environ.get("SPX_LIB", "default")[-30:], "pricing": pricing}
for mode in ("bench", "split"):
    with spx.Context(m=4096, n=16384, seed=0, device=0, pricing=pricing) as ctx:
        if mode == "bench":
            def run():
                st, p = ctx.iterate(0)
                while st == 0:
                    st, p = ctx.iterate(4096)
                return st, p
            (st, p), ms = seg(run)
            out["bench_ms"], out["bench_pivots"] = ms, p
        else:
            (_, p0), ms0 = seg(lambda: ctx.iterate(0))
            (st1, p1), ms1 = seg(lambda: ctx.iterate(npiv))
            rest = -npiv % 4096  # the passes the bench's last iterate(4096) call has left
            (st2, p2), ms2 = seg(lambda: ctx.iterate(rest))
            out.update(first_ms=ms0, pivoting_ms=ms1, pivoting_status=int(st1), pivots=p1,
                       after_ms=ms2, after_passes=rest, after_status=int(st2), after_pivots=p2 - p1,
                       after_us_per_pass=round(1e3 * ms2 / max(rest, 1), 3))
print(json.dumps(out))

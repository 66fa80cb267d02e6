"""In-kernel phase stamps (SPX_FLAG_STAMPS) per pass for representation variants.
    python tools/phase_probe.py [--m 4096 --n 16384 --k 200]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import simplex_method_gpu_amd as spx  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--m", type=int, default=4096)
ap.add_argument("--n", type=int, default=16384)
ap.add_argument("--k", type=int, default=200)
ap.add_argument("--variants", default='[{"window": -1}, {"window": 64}]')
a = ap.parse_args()
for kw in json.loads(a.variants):
    with spx.Context(m=a.m, n=a.n, seed=0, device=0, stamps=True, graph_batch=-1, **kw) as ctx:
        ctx.iterate(20)
        ctx.phase_times()
        ctx.iterate(a.k)
        ph = ctx.phase_times()
    print(json.dumps({"kw": kw, **{k: (round(v / a.k, 2) if not isinstance(v, list) else [round(x / a.k, 2) for x in v]) for k, v in ph.items()}}), flush=True)

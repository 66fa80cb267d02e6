"""A/B of Context keyword variants on one LP: graph-mode ms per pivot, variants
interleaved over several rounds.
    python tools/ab.py --variants '[{}, {"counted_tail": true}, {"_env": {"SPX_FTRAN_BC_ENTRY": "0"}}]' [--m 4096 --n 16384 --k 252 --rounds 4]"""
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
ap.add_argument("--k", type=int, default=252)
ap.add_argument("--warm", type=int, default=64)
ap.add_argument("--rounds", type=int, default=4)
ap.add_argument("--variants", default='[{}]')
a = ap.parse_args()
vs = json.loads(a.variants)
def make(kw):
    # "_env": environment read by spx_create (e.g. SPX_FTRAN_BC_ENTRY=0), set only while creating
    kw = dict(kw)
    env = kw.pop("_env", {})
    old = {k: os.environ.get(k) for k in env}
    os.environ.update({k: str(v) for k, v in env.items()})
    try:
        return spx.Context(m=a.m, n=a.n, seed=0, device=0, **kw)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


ctxs = [make(kw) for kw in vs]
for c in ctxs:
    c.iterate(a.warm)
res = [[] for _ in vs]
for r in range(a.rounds):
    for i, c in enumerate(ctxs):
        st, p0 = c.iterate(0)
        t0 = time.perf_counter()
        st, p1 = c.iterate(a.k)
        res[i].append(1e6 * (time.perf_counter() - t0) / max(p1 - p0, 1))
for kw, r in zip(vs, res):
    print(json.dumps({"kw": kw, "us_per_pivot": [round(x, 2) for x in r], "best": round(min(r), 2)}), flush=True)
for c in ctxs:
    c.close()

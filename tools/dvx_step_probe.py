"""Devex / steepest edge: K pivots in one iterate() call against K calls of
one pivot, for one rank and for a G-shard group (the per-call flush of the
deferred tail must not change the pivots).   python tools/dvx_step_probe.py [pricing G K]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import simplex_method_gpu_amd as spx  # noqa: E402

pricing, G, K = (int(v) for v in sys.argv[1:4]) if len(sys.argv) >= 4 else (1, 2, 60)
kw = dict(m=300, n=1200, seed=8, window=32, eps=1e-7, pricing=pricing)


def single(step):
    with spx.Context(trace=K, **kw) as c:
        for _ in range(K if step else 1):
            c.iterate(1 if step else K)
        return c.trace()[0]


def group(step):
    cs = [spx.Context(rank=g, nranks=G, trace=K, **kw) for g in range(G)]
    try:
        for _ in range(K if step else 1):
            spx.group_iterate(cs, 1 if step else K)
        return cs[0].trace()[0]
    finally:
        for c in cs:
            c.close()


def interleaved():
    ref = spx.Context(trace=K, **kw)
    cs = [spx.Context(rank=g, nranks=G, trace=K, **kw) for g in range(G)]
    try:
        for _ in range(K):
            ref.iterate(1)
            spx.group_iterate(cs, 1)
        return ref.trace()[0], cs[0].trace()[0]
    finally:
        ref.close()
        for c in cs:
            c.close()


il_ref, il_grp = interleaved()
out = {"interleaved_single": il_ref, "interleaved_group": il_grp, "single_full": single(False), "single_step": single(True), "group_full": group(False), "group_step": group(True)}
base = out["single_full"]
for k, v in out.items():
    d = np.nonzero(v[:min(len(v), len(base))] != base[:min(len(v), len(base))])[0]
    print(k, len(v), "first differing pivot vs single_full:", int(d[0]) if len(d) else None)

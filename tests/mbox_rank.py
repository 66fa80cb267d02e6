"""One rank of a multi-process shard group on one device, for
tests/test_gpu_mbox.py (not a test module).  The ranks exchange their
mailbox handles through files in a directory, attach (spx_mbox_attach), run
the pivots and store the state they reach.

usage: python mbox_rank.py DIR RANK NRANKS M N SEED WINDOW K GRAPH_BATCH [SOLVE [PRICING]]
(SOLVE 0: the state after K pivots only, no solve to the optimum; PRICING:
spx_opts.pricing, 0 Dantzig by default)
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import simplex_method_gpu_amd as spx  # noqa: E402


def main():
    d, rank, G, m, n, seed, window, k, gb = sys.argv[1], *map(int, sys.argv[2:10])
    solve = int(sys.argv[10]) if len(sys.argv) > 10 else 1
    pricing = int(sys.argv[11]) if len(sys.argv) > 11 else 0
    with spx.Context(m=m, n=n, seed=seed, rank=rank, nranks=G, window=window, graph_batch=gb,
                     pricing=pricing) as ctx:
        h = ctx.mbox_export()
        tmp = os.path.join(d, f"h{rank}.tmp")
        with open(tmp, "wb") as f:
            f.write(h)
        os.replace(tmp, os.path.join(d, f"h{rank}"))
        deadline = time.time() + 60
        paths = [os.path.join(d, f"h{g}") for g in range(G)]
        while not all(os.path.exists(p) for p in paths):
            if time.time() > deadline:
                raise SystemExit("mailbox handles of the other ranks never arrived")
            time.sleep(0.01)
        handles = [open(p, "rb").read() for p in paths]
        ctx.mbox_attach(handles)
        st, piv = ctx.iterate(k)
        s = ctx.state(binv=True)
        defer = ctx.config()["defer_tail"]
        fused = ctx.config()["mbox_fused"]
        if solve:
            r = ctx.solve()
            z, pivots, status = r.z, r.pivots, int(r.status)
        else:
            z, pivots, status = ctx.objective(), piv, int(st)
        np.savez(os.path.join(d, f"r{rank}.npz"), piv=piv, b_ixs=s["b_ixs"], x_b=s["x_b"], y=s["y"],
                 binv=s["binv"], z=z, pivots=pivots, status=status, defer_tail=defer, mbox_fused=fused)


if __name__ == "__main__":
    main()

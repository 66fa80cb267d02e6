"""Golden fixtures for the two largest BASELINE configs — run in the build
container (62 GB of RAM; C5's A is 8.6 GB and the oracle's B^-1 2.1 GB).

For C4 (m=4096, n=131072) and C5 (m=16384, n=65536), seed 0, the oracle
(oracle/simplex_oracle.c, the restatement of v4_cub_reduction.cu:268-368)
runs K = 130 pivots from the slack basis (two 63-pivot eta windows and their
folds on the GPU's default path) and records:
  - the (p, q) of every pivot (trace_p / trace_q),
  - the basis order b_ixs, x_b and y after K pivots,
  - z = c_B . x_b.
Data only, written to ``tests/golden/oracle_c{4,5}_k130.npz``.

C3SE: the headline config (m=4096, n=16384, seed 0) with exact steepest-edge
pricing (the oracle's se_choose, Goldfarb-Reid recurrence; README.md:16-17),
the same K = 130 pivots, plus the pricing weights gamma_j after them ->
``tests/golden/oracle_c3se_k130.npz``.

    python tests/golden/make_golden_c45.py [C4|C5|C3SE ...]
"""
from __future__ import annotations

import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import oracle  # noqa: E402

CONFIGS = {"C4": (4096, 131072, 0), "C5": (16384, 65536, 0), "C3SE": (4096, 16384, 0)}
PRICING = {"C3SE": 2}  # oracle.solve(pricing=...): 2 = steepest edge
K = 130


def make(name: str) -> str:
    m, n, seed = CONFIGS[name]
    t0 = time.time()
    A, b, c = oracle.generate(m, n, seed)
    t1 = time.time()
    pricing = PRICING.get(name, 0)
    r = oracle.solve(A, b, c, max_iter=K, eps=1e-7, trace_cap=K, want_state=True, pricing=pricing)
    t2 = time.time()
    assert r.status == oracle.MAX_ITER and r.pivots == K, (r.status, r.pivots)
    out = os.path.join(HERE, f"oracle_{name.lower()}_k{K}.npz")
    np.savez(out, m=m, n=n, seed=seed, k=K, eps=1e-7, z=r.z,
             trace_p=r.trace_p.astype(np.int64), trace_q=r.trace_q.astype(np.int64),
             b_ixs=r.b_ixs.astype(np.int64), x_b=r.x_b, y=r.y, pricing=pricing,
             **({"weights": r.weights} if pricing else {}))
    print(f"{name}: m={m} n={n} K={K} z={r.z:.15g} generate {t1 - t0:.1f} s, "
          f"oracle {t2 - t1:.1f} s -> {os.path.basename(out)}", flush=True)
    del A, r
    return out


if __name__ == "__main__":
    for nm in (sys.argv[1:] or list(CONFIGS)):
        make(nm)

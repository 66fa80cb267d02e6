"""Golden fixture for the headline config C3 (m=4096, n=16384, seed 0) — run in
the build container (about 150 s of HiGHS plus a few minutes of the oracle).

Writes ``tests/golden/highs_c3.json``: the optimum and basic set from scipy
HiGHS dual simplex (the independent solver standing in for GLPK,
solver_glpk.cpp:23; libglpk is absent in this image), and the oracle's full
solve of the same LP (oracle/simplex_oracle.c, the restatement of
v4_cub_reduction.cu:268-368): objective, pivot count and the whole (p, q)
pivot sequence.  Data only.

    python tests/golden/make_golden_c3.py [m n seed]
"""
from __future__ import annotations

import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import oracle  # noqa: E402
from make_golden import highs_optimum  # noqa: E402


def main():
    m, n, seed = (int(v) for v in sys.argv[1:4]) if len(sys.argv) >= 4 else (4096, 16384, 0)
    A, b, c = oracle.generate(m, n, seed)
    t0 = time.time()
    z, basis, _ = highs_optimum(A, b, c)
    t1 = time.time()
    print(f"highs z={z:.15g} ({t1 - t0:.1f} s)", flush=True)
    r = oracle.solve(A, b, c, eps=1e-7, trace_cap=1 << 20)
    t2 = time.time()
    assert r.status == oracle.OPTIMUM_FOUND, r.status
    obasis = sorted(int(j) for j in r.b_ixs)
    rel = abs(r.z - z) / abs(z)
    print(f"oracle z={r.z:.15g} pivots={r.pivots} rel={rel:.2e} basis_equal={obasis == basis} "
          f"({t2 - t1:.1f} s)", flush=True)
    out = {"generator": "SURVEY.md §8(d) splitmix64; A=[U|I], b=(n-m)/4*U(1,2), c=U(0,1)|0",
           "solver": "scipy %s linprog(method='highs-ds')" % __import__("scipy").__version__,
           "eps": 1e-7, "m": m, "n": n, "seed": seed,
           "highs_z": z, "highs_basis": basis, "highs_seconds": t1 - t0,
           "oracle_z": r.z, "oracle_pivots": r.pivots, "oracle_seconds": t2 - t1,
           "oracle_basis_equal": obasis == basis, "oracle_rel_gap": rel,
           "oracle_trace_p": [int(v) for v in r.trace_p],
           "oracle_trace_q": [int(v) for v in r.trace_q]}
    name = "highs_c3.json" if (m, n, seed) == (4096, 16384, 0) else f"highs_{m}x{n}_{seed}.json"
    with open(os.path.join(HERE, name), "w") as f:
        json.dump(out, f)


if __name__ == "__main__":
    main()

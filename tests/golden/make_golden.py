"""Generate the golden fixtures under tests/golden/ (run in the build container).

Fixtures are data only: generator spec (m, n, seed), the optimum found by an
independent solver (scipy HiGHS dual simplex, ``method="highs-ds"``), the set of
basic variables at that optimum, and — as a regression record of the oracle —
the first pivots of the fp64 CPU restatement (oracle/simplex_oracle.c).

HiGHS stands in for the reference's GLPK driver (solver_glpk.cpp:23, default
``glp_simplex``) because libglpk is not installed in this image.
For the dense random LPs of SURVEY.md §8(d) the optimum is unique and
non-degenerate with probability one, so objective and basic set are
solver-independent.

    python tests/golden/make_golden.py
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np
from scipy.optimize import linprog

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import oracle  # noqa: E402

CASES = [
    (4, 8, 0), (8, 16, 1), (16, 48, 2), (32, 64, 3), (33, 97, 4),
    (64, 256, 0), (100, 300, 1), (128, 512, 0), (256, 1024, 0), (257, 771, 2),
    (512, 2048, 0), (1024, 4096, 0),
]
TRACE = 64


def highs_optimum(A_cols, b, c):
    n, m = A_cols.shape
    A = A_cols.T  # (m, n)
    res = linprog(-c, A_eq=A, b_eq=b, bounds=(0, None), method="highs-ds",
                  options={"primal_feasibility_tolerance": 1e-10,
                           "dual_feasibility_tolerance": 1e-10})
    assert res.status == 0, res.message
    x = res.x
    basis = sorted(int(j) for j in np.argsort(-x)[:m])
    return float(-res.fun), basis, x


def main():
    out = {"generator": "SURVEY.md §8(d) splitmix64; A=[U|I], b=(n-m)/4*U(1,2), c=U(0,1)|0",
           "solver": "scipy %s linprog(method='highs-ds')" % __import__("scipy").__version__,
           "eps": 1e-7, "cases": []}
    for (m, n, seed) in CASES:
        A, b, c = oracle.generate_np(m, n, seed)
        t0 = time.time()
        z, basis, x = highs_optimum(A, b, c)
        t1 = time.time()
        r = oracle.solve(A, b, c, eps=1e-7, trace_cap=TRACE)
        t2 = time.time()
        assert r.status == oracle.OPTIMUM_FOUND
        obasis = sorted(int(j) for j in r.b_ixs)
        rel = abs(r.z - z) / abs(z)
        print(f"m={m} n={n} seed={seed}: highs z={z:.12g} ({t1 - t0:.2f}s) "
              f"oracle z={r.z:.12g} pivots={r.pivots} rel={rel:.2e} "
              f"basis_equal={obasis == basis} ({t2 - t1:.2f}s)")
        out["cases"].append({
            "m": m, "n": n, "seed": seed,
            "highs_z": z, "highs_basis": basis,
            "oracle_z": r.z, "oracle_pivots": r.pivots,
            "oracle_trace_p": [int(v) for v in r.trace_p],
            "oracle_trace_q": [int(v) for v in r.trace_q],
        })
    with open(os.path.join(HERE, "highs_optima.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()

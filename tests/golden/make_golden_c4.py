"""Independent optimum for BASELINE config C4 (m=4096, n=131072, seed 0), run in
the build container: scipy HiGHS dual simplex (the solver standing in for
GLPK, solver_glpk.cpp:23; libglpk is absent in this image) on the seeded LP of
SURVEY.md §8(d).  Writes ``tests/golden/highs_c4.json`` (the optimum, the
basic set, HiGHS's wall time and the process's peak resident memory).  Data
only; the GPU tests solve C4 to optimality and compare with it
(tests/test_gpu_c4_optimum.py).

    python tests/golden/make_golden_c4.py [m n seed]
    (committed: 4096 65536 0 -> highs_4096x65536_0.json; 16384 20480 0 ->
    highs_16384x20480_0.json, C5's height, tests/test_gpu_c5_optimum.py;
    8192 24576 0 -> highs_8192x24576_0.json, tests/test_gpu_m8192_optimum.py)

The basis is read from x as make_golden.highs_optimum does (the m largest
entries); the LP is the same as there.
"""
from __future__ import annotations

import json
import os
import resource
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import numpy as np  # noqa: E402
import scipy.sparse as sp  # noqa: E402
from scipy.optimize import linprog  # noqa: E402

import oracle  # noqa: E402


def main():
    m, n, seed = (int(v) for v in sys.argv[1:4]) if len(sys.argv) >= 4 else (4096, 131072, 0)
    A, b, c = oracle.generate(m, n, seed)
    # A = [U | I] handed over as CSC (the structural columns dense, the slack
    # columns unit), built without a dense transpose: the dense path ran out
    # of the container's memory inside HiGHS (std::bad_alloc at 52 GB)
    ns = n - m
    data = np.empty(ns * m + m)
    data[: ns * m] = A[:ns].reshape(-1)
    data[ns * m:] = 1.0
    del A
    indices = np.empty(ns * m + m, dtype=np.int32)
    indices[: ns * m].reshape(ns, m)[:] = np.arange(m, dtype=np.int32)
    indices[ns * m:] = np.arange(m, dtype=np.int32)
    indptr = np.concatenate([np.arange(ns + 1, dtype=np.int64) * m, ns * m + 1 + np.arange(m, dtype=np.int64)])
    Acsc = sp.csc_array((data, indices, indptr), shape=(m, n))
    del data, indices
    t0 = time.time()
    res = linprog(-c, A_eq=Acsc, b_eq=b, bounds=(0, None), method="highs-ds",
                  options={"primal_feasibility_tolerance": 1e-10, "dual_feasibility_tolerance": 1e-10,
                           "presolve": False})  # (presolve copies the LP: no room for it here)
    assert res.status == 0, res.message
    z = float(-res.fun)
    basis = sorted(int(j) for j in np.argsort(-res.x)[:m])
    t1 = time.time()
    rss_gb = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 2**20
    print(f"highs z={z:.15g} ({t1 - t0:.1f} s, peak RSS {rss_gb:.1f} GB)", flush=True)
    out = {"generator": "SURVEY.md §8(d) splitmix64; A=[U|I], b=(n-m)/4*U(1,2), c=U(0,1)|0",
           "solver": "scipy %s linprog(method='highs-ds')" % __import__("scipy").__version__,
           "m": m, "n": n, "seed": seed, "highs_z": z, "highs_basis": basis,
           "highs_seconds": t1 - t0, "peak_rss_gb": rss_gb}
    name = "highs_c4.json" if (m, n, seed) == (4096, 131072, 0) else f"highs_{m}x{n}_{seed}.json"
    with open(os.path.join(HERE, name), "w") as f:
        json.dump(out, f)


if __name__ == "__main__":
    main()

"""Small LP generators for the robustness tests.

degenerate_lp: A = [U | I] with small-integer U (exact ties in both argmins)
and b with zeros (a degenerate slack basis); every structural column has a
positive entry, so with U >= 0 the LP is bounded.  Returns (A_cols (n, m), b, c).
"""
import numpy as np


def degenerate_lp(m: int, n: int, seed: int, density: float = 0.05, zero_frac: float = 0.1):
    rng = np.random.default_rng(seed)
    ns = n - m
    U = rng.integers(1, 4, size=(m, ns)).astype(np.float64) * (rng.random((m, ns)) < density)
    U[rng.integers(0, m, size=ns), np.arange(ns)] = rng.integers(1, 4, size=ns)
    A = np.hstack([U, np.eye(m)])
    b = rng.integers(1, 4, size=m).astype(np.float64) * (rng.random(m) >= zero_frac)
    c = np.concatenate([rng.integers(1, 5, size=ns).astype(np.float64), np.zeros(m)])
    return np.ascontiguousarray(A.T), b, c


def highs_opt(A_cols, b, c):
    """Optimum of max c.x s.t. A x <= b (slack columns dropped), x >= 0, by
    scipy HiGHS (an independent solver standing in for GLPK)."""
    from scipy.optimize import linprog

    n, m = A_cols.shape
    ns = n - m
    r = linprog(-c[:ns], A_ub=A_cols[:ns].T, b_ub=b, bounds=(0, None), method="highs-ds")
    assert r.status == 0, r.message
    return -r.fun

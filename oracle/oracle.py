"""CPU oracle for the revised-simplex hot loop — TEST INFRASTRUCTURE ONLY.

ctypes front end to ``oracle/_build/liboracle.so`` (the fp64 C restatement of
``src/v4_cub_reduction.cu:219-380``, see ``simplex_oracle.c``) plus a numpy
restatement of the seeded generator of SURVEY.md §8(d).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module, and only as the checker/baseline — never as the
thing measured or shipped.

Parity pinning: ``input/sample.txt:15-16`` (z = 9, x0 = 1, x1 = 3) and golden
optima from an independent solver (scipy HiGHS, ``tests/golden/make_golden.py``)
standing in for GLPK (``solver_glpk.cpp:23``, library absent in this image).
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")

# SolveStatus of the reference (v4_cub_reduction.cu:49-54)
MAX_ITER, OPTIMUM_FOUND, UNBOUNDED, THETA_OVERFLOW = 0, 1, 2, 3

_lib = None

# leaving-row rules (include/simplex.h SPX_RATIO_*)
RATIO_REFERENCE, RATIO_GUARDED, RATIO_HARRIS = 0, 1, 2
# entering-column rules (include/simplex.h SPX_PRICING_*)
PRICING_DANTZIG, PRICING_DEVEX, PRICING_STEEPEST = 0, 1, 2


class OrcOpts(ctypes.Structure):
    _fields_ = [("max_iter", ctypes.c_int64), ("eps", ctypes.c_double), ("threads", ctypes.c_int),
                ("ratio", ctypes.c_int), ("piv_tol", ctypes.c_double), ("feas_tol", ctypes.c_double),
                ("refactor_every", ctypes.c_int64), ("pricing", ctypes.c_int), ("w_out", ctypes.c_void_p)]


def build() -> str:
    import subprocess

    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        d, i64, u64, p = ctypes.c_double, ctypes.c_int64, ctypes.c_uint64, ctypes.c_void_p
        L.orc_splitmix64.argtypes = [u64]
        L.orc_splitmix64.restype = u64
        L.orc_uniform.argtypes = [u64, u64, u64]
        L.orc_uniform.restype = d
        L.orc_generate.argtypes = [i64, i64, u64, p, p, p]
        L.orc_generate.restype = None
        L.orc_solve.argtypes = [i64, i64, p, p, p, i64, d, ctypes.c_int,
                                p, p, p, p, p, p, i64, p, p]
        L.orc_solve.restype = ctypes.c_int
        L.orc_time_iterations.argtypes = [i64, i64, p, p, p, i64, ctypes.c_int, p]
        L.orc_time_iterations.restype = d
        L.orc_price.argtypes = [i64, i64, p, p, p, p, ctypes.c_int]
        L.orc_price.restype = None
        L.orc_solve_ex.argtypes = [i64, i64, p, p, p, ctypes.POINTER(OrcOpts),
                                   p, p, p, p, p, p, i64, p, p]
        L.orc_solve_ex.restype = ctypes.c_int
        L.orc_default_opts.argtypes = [ctypes.POINTER(OrcOpts)]
        L.orc_default_opts.restype = None
        L.orc_reinvert.argtypes = [i64, i64, p, p, p, p, ctypes.c_int, p, p, p]
        L.orc_reinvert.restype = ctypes.c_int
        L.orc_max_threads.argtypes = []
        L.orc_max_threads.restype = ctypes.c_int
        _lib = L
    return _lib


def _ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


# ---------------------------------------------------------------- generator
_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64_np(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = x.astype(np.uint64) + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def uniform_np(seed: int, stream: int, idx: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        key = (np.uint64(seed) * np.uint64(0x9E3779B97F4A7C15)) ^ (np.uint64(stream) << np.uint64(56))
        u = splitmix64_np(key ^ idx.astype(np.uint64)) >> np.uint64(11)
    return u.astype(np.float64) * (2.0 ** -53)


def generate_np(m: int, n: int, seed: int):
    """numpy restatement of orc_generate; A column-major as (n, m)."""
    ns = n - m
    A = np.zeros((n, m), dtype=np.float64)  # row j of this array = column j of A
    if ns > 0:
        idx = (np.arange(m, dtype=np.uint64)[None, :]
               + np.arange(ns, dtype=np.uint64)[:, None] * np.uint64(m))
        A[:ns] = uniform_np(seed, 1, idx)
    A[ns + np.arange(m), np.arange(m)] = 1.0
    b = (ns / 4.0) * (1.0 + uniform_np(seed, 2, np.arange(m, dtype=np.uint64)))
    c = np.zeros(n)
    c[:ns] = uniform_np(seed, 3, np.arange(ns, dtype=np.uint64))
    return A, b, c


def column_np(m: int, n: int, seed: int, j: int) -> np.ndarray:
    """Column j of the generated A (for spot checks at sizes too big to build)."""
    if j >= n - m:
        e = np.zeros(m)
        e[j - (n - m)] = 1.0
        return e
    idx = np.arange(m, dtype=np.uint64) + np.uint64(j) * np.uint64(m)
    return uniform_np(seed, 1, idx)


def generate(m: int, n: int, seed: int):
    """C generator; returns (A_cols (n, m) C-contiguous == column-major m x n, b, c)."""
    A = np.empty((n, m), dtype=np.float64)
    b = np.empty(m)
    c = np.empty(n)
    lib().orc_generate(m, n, seed, _ptr(A), _ptr(b), _ptr(c))
    return A, b, c


# ---------------------------------------------------------------- LP text I/O
def read_lp_text(path: str):
    """Restates main()'s reader (v4:401-419, load_matrix v4:94-104): ``m n``,
    then A row-major (m x n), b (m), c (n); trailing text is ignored.
    Returns (m, n, A_cols (n, m), b, c)."""
    with open(path) as f:
        toks = f.read().split()
    m, n = int(toks[0]), int(toks[1])
    if m > n:
        raise ValueError("Either failed to read m and n, or m > n.")
    need = m * n + m + n
    vals = np.array([float(t) for t in toks[2:2 + need]], dtype=np.float64)
    if vals.size < need:
        raise ValueError("truncated LP file")
    A_rows = vals[: m * n].reshape(m, n)
    b = vals[m * n: m * n + m].copy()
    c = vals[m * n + m: need].copy()
    return m, n, np.ascontiguousarray(A_rows.T), b, c


# ---------------------------------------------------------------- solve
@dataclass
class OracleResult:
    status: int
    z: float
    x_b: np.ndarray
    b_ixs: np.ndarray
    pivots: int
    trace_p: np.ndarray
    trace_q: np.ndarray
    y: np.ndarray | None = None
    binv: np.ndarray | None = None
    weights: np.ndarray | None = None  # Devex / steepest-edge weights (want_state)


def solve(A_cols: np.ndarray, b: np.ndarray, c: np.ndarray, max_iter: int = 1 << 40,
          eps: float = 1e-7, threads: int = 0, trace_cap: int = 0,
          want_state: bool = False, ratio: int = RATIO_REFERENCE, piv_tol: float = 1e-9,
          feas_tol: float = 1e-9, refactor_every: int = 0, pricing: int = 0) -> OracleResult:
    n, m = A_cols.shape
    A_cols = np.ascontiguousarray(A_cols, dtype=np.float64)
    b = np.ascontiguousarray(b, dtype=np.float64)
    c = np.ascontiguousarray(c, dtype=np.float64)
    z = ctypes.c_double(0.0)
    piv = ctypes.c_int64(0)
    x_b = np.zeros(m)
    b_ixs = np.zeros(m, dtype=np.int64)
    tp = np.full(max(trace_cap, 1), -1, dtype=np.int64)
    tq = np.full(max(trace_cap, 1), -1, dtype=np.int64)
    y = np.zeros(m) if want_state else None
    binv = np.zeros((m, m)) if want_state else None
    o = OrcOpts()
    lib().orc_default_opts(ctypes.byref(o))
    o.max_iter, o.eps, o.threads = max_iter, eps, threads
    o.ratio, o.piv_tol, o.feas_tol, o.refactor_every = ratio, piv_tol, feas_tol, refactor_every
    o.pricing = pricing
    w = np.zeros(n) if (want_state and pricing) else None
    o.w_out = None if w is None else w.ctypes.data
    st = lib().orc_solve_ex(m, n, _ptr(A_cols), _ptr(b), _ptr(c), ctypes.byref(o),
                            ctypes.byref(z), _ptr(x_b), _ptr(b_ixs), ctypes.byref(piv),
                            _ptr(tp), _ptr(tq), trace_cap, _ptr(y), _ptr(binv))
    if st < 0:
        raise ValueError(f"orc_solve failed ({st})")
    k = min(piv.value, trace_cap)
    return OracleResult(st, z.value, x_b, b_ixs, piv.value, tp[:k], tq[:k], y, binv, w)


def reinvert(A_cols, b, c, basis, threads: int = 0):
    """Pivot-in reinversion of the basis (orc_reinvert): (B^-1 row-major, x_b, y)
    in the given basis order.  Raises ValueError on a bad or singular basis."""
    n, m = A_cols.shape
    basis = np.ascontiguousarray(basis, dtype=np.int64)
    binv = np.zeros((m, m))
    x_b = np.zeros(m)
    y = np.zeros(m)
    rc = lib().orc_reinvert(m, n, _ptr(np.ascontiguousarray(A_cols, dtype=np.float64)),
                            _ptr(np.ascontiguousarray(b, dtype=np.float64)),
                            _ptr(np.ascontiguousarray(c, dtype=np.float64)), _ptr(basis), threads,
                            _ptr(binv), _ptr(x_b), _ptr(y))
    if rc != 0:
        raise ValueError(f"orc_reinvert failed ({rc}: {'singular basis' if rc == -7 else 'bad basis'})")
    return binv, x_b, y


def price(A_cols, c, y, threads: int = 0) -> np.ndarray:
    n, m = A_cols.shape
    e = np.empty(n)
    lib().orc_price(m, n, _ptr(np.ascontiguousarray(A_cols)), _ptr(np.ascontiguousarray(c)),
                    _ptr(np.ascontiguousarray(y)), _ptr(e), threads)
    return e


def time_iterations(A_cols, b, c, iters: int, threads: int = 0):
    n, m = A_cols.shape
    done = ctypes.c_int64(0)
    sec = lib().orc_time_iterations(m, n, _ptr(A_cols), _ptr(b), _ptr(c), iters, threads,
                                    ctypes.byref(done))
    return sec, done.value


def max_threads() -> int:
    return lib().orc_max_threads()

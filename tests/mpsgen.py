"""Random MPS problems for the MPS-path tests and their
HiGHS optimum (scipy.optimize.linprog, an independent solver standing in for
the reference's GLPK driver, solver_glpk.cpp:23 — libglpk is not installed).

random_mps(seed, nv, nr) mixes every row type (L, G, E, ranged L/G/E, an
extra free N row), every bound type (default, LO, UP, LO+UP, FX, FR, MI, BV,
negative UP), an objective constant and OBJSENSE MAX/MIN.  Feasibility comes
from a planted point x0; boundedness from cost signs matched to each
variable's finite bound (free variables get two single-entry rows).
"""
import numpy as np

INF = float("inf")


def random_mps(seed: int, nv: int = 12, nr: int = 9, maximize: bool | None = None):
    rng = np.random.default_rng(seed)
    if maximize is None:
        maximize = bool(rng.integers(0, 2))
    kinds = rng.choice(["def", "lo", "up", "both", "fx", "fr", "mi", "bv", "negup"], size=nv)
    lo = np.zeros(nv)
    up = np.full(nv, INF)
    x0 = np.zeros(nv)
    bounds = []  # (type, j, value or None)
    for j, k in enumerate(kinds):
        if k == "def":
            x0[j] = rng.uniform(0, 3)
        elif k == "lo":
            lo[j] = rng.integers(-3, 3)
            bounds.append(("LO", j, lo[j]))
            x0[j] = lo[j] + rng.uniform(0, 3)
        elif k == "up":
            up[j] = rng.integers(1, 5)
            bounds.append(("UP", j, up[j]))
            x0[j] = rng.uniform(0, up[j])
        elif k == "both":
            lo[j], up[j] = -2.0, 3.0
            bounds += [("LO", j, lo[j]), ("UP", j, up[j])]
            x0[j] = rng.uniform(lo[j], up[j])
        elif k == "fx":
            lo[j] = up[j] = rng.integers(-2, 3)
            bounds.append(("FX", j, lo[j]))
            x0[j] = lo[j]
        elif k == "fr":
            lo[j] = -INF
            bounds.append(("FR", j, None))
            x0[j] = rng.uniform(-3, 3)
        elif k == "mi":
            lo[j] = -INF
            up[j] = 2.0
            bounds += [("MI", j, None), ("UP", j, up[j])]
            x0[j] = rng.uniform(-3, 2)
        elif k == "bv":
            up[j] = 1.0
            bounds.append(("BV", j, None))
            x0[j] = rng.uniform(0, 1)
        else:  # negative UP with no lower bound: lower bound becomes -inf
            lo[j] = -INF
            up[j] = -1.0
            bounds.append(("UP", j, up[j]))
            x0[j] = rng.uniform(-4, -1)
    # costs with signs that keep min (or max) bounded
    c = rng.uniform(0.5, 3.0, size=nv)
    for j in range(nv):
        toward_lo = np.isfinite(lo[j])
        toward_up = np.isfinite(up[j])
        if toward_lo and toward_up:
            c[j] *= rng.choice([-1.0, 1.0])
        elif toward_up:
            c[j] = -c[j]  # min prefers large x; capped by up
    if maximize:
        c = -c
    A = np.round(rng.uniform(-3, 3, size=(nr, nv)) * (rng.random((nr, nv)) < 0.5), 3)
    rtypes, rl, ru, rhs, rng_v = [], [], [], [], []
    ax = A @ x0
    for i in range(nr):
        t = rng.choice(["L", "G", "E", "RL", "RG", "RE"])
        if t == "L":
            rtypes.append("L"); r = ax[i] + rng.uniform(0, 2); rl.append(-INF); ru.append(r); rhs.append(r); rng_v.append(None)
        elif t == "G":
            rtypes.append("G"); r = ax[i] - rng.uniform(0, 2); rl.append(r); ru.append(INF); rhs.append(r); rng_v.append(None)
        elif t == "E":
            rtypes.append("E"); r = ax[i]; rl.append(r); ru.append(r); rhs.append(r); rng_v.append(None)
        elif t == "RL":
            rtypes.append("L"); r = ax[i] + 0.5; R = 2.0; rl.append(r - R); ru.append(r); rhs.append(r); rng_v.append(R)
        elif t == "RG":
            rtypes.append("G"); r = ax[i] - 0.5; R = 2.0; rl.append(r); ru.append(r + R); rhs.append(r); rng_v.append(R)
        else:
            rtypes.append("E"); R = float(rng.choice([-1.5, 1.5])); r = ax[i] - R / 2
            rl.append(min(r, r + R)); ru.append(max(r, r + R)); rhs.append(r); rng_v.append(R)
    # free variables: keep them bounded through single-entry rows
    extra = []
    for j in range(nv):
        if not np.isfinite(lo[j]) and not np.isfinite(up[j]):
            extra.append((j, "L", 6.0))
            extra.append((j, "G", -6.0))
        elif not np.isfinite(lo[j]):
            extra.append((j, "G", -8.0))
    for j, t, r in extra:
        row = np.zeros(nv)
        row[j] = 1.0
        A = np.vstack([A, row])
        rtypes.append(t); rhs.append(r); rng_v.append(None)
        rl.append(r if t == "G" else -INF); ru.append(r if t == "L" else INF)
    const = float(np.round(rng.uniform(-5, 5), 3))
    lines = [f"NAME          RAND{seed}"]
    if maximize:
        lines += ["OBJSENSE", "    MAX"]
    lines.append("ROWS")
    lines.append(" N  COST")
    lines.append(" N  SPARE")  # a second free row: ignored
    for i, t in enumerate(rtypes):
        lines.append(f" {t}  R{i}")
    lines.append("COLUMNS")
    for j in range(nv):
        ent = [("COST", c[j])] + [(f"R{i}", A[i, j]) for i in range(A.shape[0]) if A[i, j] != 0.0]
        ent.append(("SPARE", 1.0))
        for k in range(0, len(ent), 2):
            chunk = ent[k:k + 2]
            lines.append(f"    X{j}  " + "  ".join(f"{r}  {float(v)!r}" for r, v in chunk))
    lines.append("RHS")
    rl_items = [(f"R{i}", rhs[i]) for i in range(len(rhs)) if rhs[i] != 0.0] + [("COST", -const)]
    for r, v in rl_items:
        lines.append(f"    RHS  {r}  {float(v)!r}")
    if any(v is not None for v in rng_v):
        lines.append("RANGES")
        for i, v in enumerate(rng_v):
            if v is not None:
                lines.append(f"    RNG  R{i}  {float(v)!r}")
    if bounds:
        lines.append("BOUNDS")
        for t, j, v in bounds:
            lines.append(f" {t} BND  X{j}" + (f"  {float(v)!r}" if v is not None else ""))
    lines.append("ENDATA")
    spec = dict(c=c, A=A, rl=np.array(rl), ru=np.array(ru), lo=lo, up=up, maximize=maximize, const=const)
    return "\n".join(lines) + "\n", spec


def highs_solve(spec):
    """(status, z, x) of the original problem by scipy HiGHS."""
    from scipy.optimize import linprog

    c, A, rl, ru = spec["c"], spec["A"], spec["rl"], spec["ru"]
    sgn = -1.0 if spec["maximize"] else 1.0
    A_ub, b_ub, A_eq, b_eq = [], [], [], []
    for i in range(A.shape[0]):
        if rl[i] == ru[i]:
            A_eq.append(A[i]); b_eq.append(ru[i])
            continue
        if np.isfinite(ru[i]):
            A_ub.append(A[i]); b_ub.append(ru[i])
        if np.isfinite(rl[i]):
            A_ub.append(-A[i]); b_ub.append(-rl[i])
    bnds = [(None if not np.isfinite(l) else l, None if not np.isfinite(u) else u)
            for l, u in zip(spec["lo"], spec["up"])]
    r = linprog(sgn * c, A_ub=np.array(A_ub) if A_ub else None, b_ub=b_ub or None,
                A_eq=np.array(A_eq) if A_eq else None, b_eq=b_eq or None, bounds=bnds, method="highs")
    z = None if r.status != 0 else sgn * r.fun + spec["const"]
    return r.status, z, r.x

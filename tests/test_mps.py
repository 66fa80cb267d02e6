"""MPS input: the ./solver --mps path (csrc/mps_io.cpp)
and the GLPK-driver counterpart (csrc/glpk_driver.cpp), replacing the
reference's GLPK MPS reader (solver_glpk.cpp:15) and its broken converter
(glpk_interface.cpp:46-52,80-98).

Parity: tests/mpsgen.py builds random problems with every row and bound type;
their optimum comes from scipy HiGHS on the ORIGINAL problem (not through the
MPS file), standing in for GLPK, which is not installed ("parity unpinned"
against GLPK itself).  CPU: the converted text LP solved by the oracle
(guarded ratio rule) and mapped back gives the HiGHS objective within 1e-9
(relative to max(1, |z|)).  GPU: ./solver --mps gives it directly, with the
recovered x feasible within 1e-7.
"""
import json
import os
import subprocess

import numpy as np
import pytest

from mpsgen import highs_solve, random_mps

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SOLVER = os.path.join(ROOT, "solver")
GLPK = os.path.join(ROOT, "solver_glpk")
SEEDS = list(range(16))


def run(*args, exe=SOLVER):
    return subprocess.run([exe, *map(str, args)], capture_output=True, text=True, timeout=120)


def read_map(path):
    """The trailing '# ...' block of a converted LP (mps::map_block)."""
    lines = [ln.split()[1:] for ln in open(path) if ln.startswith("#")]
    const = float(lines[1][3])
    vars_ = [(int(e[3]), int(e[4]), int(e[5]), float(e[6]), float(e[7])) for e in lines if e[0] == "var"]
    art = [int(v) for v in next(e for e in lines if e[0] == "artificial")[1:]]
    return const, vars_, art


def recover(vars_, xc):
    x = []
    for kind, plus, minus, shift, _ in vars_:
        x.append([shift + (xc[plus] if plus >= 0 else 0), shift - (xc[plus] if plus >= 0 else 0),
                  (xc[plus] - xc[minus]) if plus >= 0 else 0.0, shift][kind])
    return np.array(x)


def check_feasible(spec, x, tol=1e-7):
    A, rl, ru, lo, up = spec["A"], spec["rl"], spec["ru"], spec["lo"], spec["up"]
    ax = A @ x
    assert np.all(ax >= rl - tol * (1 + np.abs(rl))), (ax, rl)
    assert np.all(ax <= ru + tol * (1 + np.abs(ru))), (ax, ru)
    assert np.all(x >= lo - tol) and np.all(x <= up + tol)


@pytest.mark.parametrize("seed", SEEDS)
def test_converted_lp_solves_to_highs_optimum(tmp_path, oracle, seed):
    txt, spec = random_mps(seed)
    mps = tmp_path / "p.mps"
    mps.write_text(txt)
    out = tmp_path / "p.txt"
    r = run("--mps", mps, "--write-text", out, "--no-solve")
    assert r.returncode == 0, r.stderr
    st, z_star, _ = highs_solve(spec)
    assert st == 0
    m, n, A, b, c = oracle.read_lp_text(str(out))
    assert np.all(b >= 0.0) and np.array_equal(A[n - m:], np.eye(m))  # slack identity, b >= 0 (v4:272-277)
    res = oracle.solve(A, b, c, ratio=oracle.RATIO_GUARDED)
    assert res.status == oracle.OPTIMUM_FOUND
    const, vars_, art = read_map(str(out))
    xc = np.zeros(n)
    xc[res.b_ixs] = res.x_b
    assert max([xc[a] for a in art], default=0.0) <= 1e-9
    x = recover(vars_, xc)
    check_feasible(spec, x)
    z = float(spec["c"] @ x) + spec["const"]
    assert abs(z - z_star) <= 1e-9 * max(1.0, abs(z_star)), (z, z_star)


def test_mps_errors(tmp_path):
    p = tmp_path / "bad.mps"
    p.write_text("NAME X\nROWS\n N COST\n L R1\nCOLUMNS\n    X1 COST 1 R9 2\nRHS\n    RHS R1 1\nENDATA\n")
    r = run("--mps", p)
    assert r.returncode != 0 and "bad.mps:6: unknown row R9" in r.stderr
    p.write_text("NAME X\nROWS\n N COST\n L R1\nCOLUMNS\n    X1 COST 1 R1 2\n")
    r = run("--mps", p)
    assert r.returncode != 0 and "missing ENDATA" in r.stderr
    p.write_text("NAME X\nROWS\n N COST\n L R1\nCOLUMNS\n    X1 COST 1 R1 two\nENDATA\n")
    r = run("--mps", p)
    assert r.returncode != 0 and "bad number two" in r.stderr


def test_glpk_counterpart_reports_absence(tmp_path):
    """No libglpk in this image: the driver says so and exits 3 instead of
    substituting another solver."""
    txt, _ = random_mps(0)
    p = tmp_path / "p.mps"
    p.write_text(txt)
    r = run(p, exe=GLPK)
    if r.returncode == 3:
        assert "GLPK unavailable" in r.stderr
    else:  # a box with libglpk: the reference's output format
        assert r.returncode == 0 and ("Optimal objective:" in r.stdout or "Problem status:" in r.stdout)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", SEEDS)
def test_mps_solve_on_gpu(tmp_path, seed):
    txt, spec = random_mps(seed)
    p = tmp_path / "p.mps"
    p.write_text(txt)
    r = run("--mps", p, "--json")
    assert r.returncode == 0, r.stderr
    st, z_star, _ = highs_solve(spec)
    lines = r.stdout.strip().splitlines()
    res = json.loads(lines[-1])
    assert res["glp_status"] == 5 and res["status"] == 1
    assert "Optimal objective:" in r.stdout and lines[0].startswith("x[1] = ")
    x = np.array(res["x"])
    check_feasible(spec, x)
    assert abs(res["z"] - z_star) <= 1e-9 * max(1.0, abs(z_star)), (res["z"], z_star)


@pytest.mark.gpu
def test_mps_infeasible_and_unbounded(tmp_path):
    p = tmp_path / "inf.mps"
    p.write_text("NAME INF\nROWS\n N COST\n L R1\n G R2\nCOLUMNS\n    X1 COST 1 R1 1\n    X1 R2 1\n"
                 "RHS\n    RHS R1 1 R2 3\nENDATA\n")  # x1 <= 1 and x1 >= 3
    r = run("--mps", p)
    assert r.returncode == 0 and r.stdout.strip().splitlines()[0] == "Problem status: 4"  # GLP_NOFEAS
    p = tmp_path / "unb.mps"
    p.write_text("NAME UNB\nOBJSENSE\n    MAX\nROWS\n N COST\n G R1\nCOLUMNS\n    X1 COST 1 R1 1\n"
                 "    X2 COST 1 R1 -1\nRHS\n    RHS R1 1\nENDATA\n")  # max x1 + x2, x1 - x2 >= 1
    r = run("--mps", p)
    assert r.returncode == 0 and r.stdout.strip().splitlines()[0] == "Problem status: 6"  # GLP_UNBND

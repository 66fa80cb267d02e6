"""The ./solver CLI: same argv, errors and stdout as the reference's
bin/solverN.out (main() at src/v4_cub_reduction.cu:384-473)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SOLVER = os.path.join(ROOT, "solver")
SAMPLE = os.path.join(ROOT, "tests", "golden", "sample.txt")


def run(*args):
    return subprocess.run([SOLVER, *args], capture_output=True, text=True, timeout=120)


def test_no_argument():
    r = run()
    assert r.returncode == 1 and r.stderr == "Please, specify an input file.\n"  # v4:387-390


def test_missing_file():
    r = run("/nonexistent/lp.txt")
    assert r.returncode == 1 and r.stderr == "Could not open /nonexistent/lp.txt.\n"  # v4:396-399


def test_m_greater_than_n(tmp_path):
    p = tmp_path / "bad.txt"
    p.write_text("3 2\n")
    r = run(str(p))
    assert r.returncode == 1 and r.stderr == "Either failed to read m and n, or m > n.\n"  # v4:402-405


def test_truncated_matrix(tmp_path):
    p = tmp_path / "trunc.txt"
    p.write_text("2 4\n1 1 1 0\n2 1\n")
    r = run(str(p))
    assert r.returncode != 0 and "Failed to read (1,2) for A" in r.stderr  # v4:98-101


@pytest.mark.gpu
def test_sample_stdout_matches_reference():
    r = run("--compat", SAMPLE)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.splitlines()
    # expected reference stdout: 3 passes, optimum 9, basis order
    assert lines[:7] == ["# Iteration 1", "# Iteration 2", "# Iteration 3", "Optimum found: 9",
                         "\tx_1 = 3", "\tx_0 = 1", ""]
    labels = [ln.split(":")[0].strip() for ln in lines[7:] if ln.strip()]
    assert labels == ["Total", "y", "p", "B_inv", "x_b", "Alloc", "Init", "Dealloc", "Host alloc",
                      "Read file", "Solve call", "Print result", "Host free"]


@pytest.mark.gpu
def test_generated_solve_json():
    r = run("--no-iter-lines", "--json", "--gen", "64", "256", "0")
    assert r.returncode == 0, r.stderr
    import json

    js = json.loads(r.stdout.strip().splitlines()[-1])
    assert js["status"] == 1 and abs(js["z"] - 115.9505237149796) < 1e-9 * 116

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


@pytest.mark.gpu
def test_generated_solve_tableau_json():
    """--tableau (SPX_FLAG_TABLEAU): the same optimum and pivot count as the default run."""
    import json

    outs = []
    for extra in ((), ("--tableau",)):
        r = run("--no-iter-lines", "--json", *extra, "--gen", "300", "1200", "7")
        assert r.returncode == 0, r.stderr
        outs.append(json.loads(r.stdout.strip().splitlines()[-1]))
    assert outs[1]["status"] == outs[0]["status"] == 1
    assert abs(outs[1]["z"] - outs[0]["z"]) <= 1e-9 * abs(outs[0]["z"])


# --- LP file formats (simplex_method_gpu_amd/csrc/lp_io.h) ---

def _numbers(path):
    return [float(t) for t in open(path).read().split()]


def test_bad_token_messages(tmp_path):
    """Parallel parser reports the first unreadable entry like the reference's
    sequential reader (v4:94-104): A by (i,j), b by (i,0), c by (0,j)."""
    for text, msg in [("2 3\n1 2 3\n4 x 6\n1 1\n1 1 1\n", "Failed to read (1,1) for A"),
                      ("2 3\n1 2 3\n4 5 6\n7 8\n", "Failed to read (0,0) for c"),
                      ("2 3\n1 2 3\n4 5 6\n7\n", "Failed to read (1,0) for b"),
                      ("2 3\n1 2 3\n4 5 6\n7 8\n1 2 z\n", "Failed to read (0,2) for c"),
                      ("two 3\n", "Either failed to read m and n, or m > n.")]:
        p = tmp_path / "lp.txt"
        p.write_text(text)
        r = run("--no-solve", str(p))
        assert r.returncode == 1 and r.stderr == msg + "\n", (text, r.stderr)


def test_text_binary_round_trip(tmp_path):
    """text -> .spxlp -> text keeps every number (%.17g) and ignores trailing prose."""
    src = tmp_path / "src.txt"
    src.write_text(open(SAMPLE).read() + "\nthis trailing comment is ignored 1 2 3\n")
    b1, t1 = tmp_path / "a.spxlp", tmp_path / "a.txt"
    assert run("--no-solve", "--write-bin", str(b1), str(src)).returncode == 0
    assert open(b1, "rb").read(8) == b"SPXLP001"
    assert run("--no-solve", "--write-text", str(t1), str(b1)).returncode == 0
    want = _numbers(SAMPLE)
    assert _numbers(t1) == want[:2 + 2 * 4 + 2 + 4]


def test_generated_export_matches_oracle(tmp_path, oracle):
    """--gen ... --write-text exports the seeded LP bit for bit (host copy of k_generate)."""
    import numpy as np

    m, n, seed = 37, 150, 5
    t = tmp_path / "g.txt"
    assert run("--no-solve", "--write-text", str(t), "--gen", str(m), str(n), str(seed)).returncode == 0
    v = np.array(_numbers(t))
    A, b, c = oracle.generate(m, n, seed)
    assert v[:2].tolist() == [m, n]
    assert np.array_equal(v[2:2 + m * n].reshape(m, n), A.T)
    assert np.array_equal(v[2 + m * n:2 + m * n + m], b) and np.array_equal(v[2 + m * n + m:], c)


def test_parallel_parse_matches_single_thread(tmp_path):
    """A multi-MiB file parsed by 1 and by 7 threads gives the same binary."""
    t = tmp_path / "big.txt"
    assert run("--no-solve", "--write-text", str(t), "--gen", "300", "2000", "9").returncode == 0
    assert os.path.getsize(t) > 8 << 20
    outs = []
    for th in ("1", "7"):
        o = tmp_path / f"big{th}.spxlp"
        assert run("--no-solve", "--threads", th, "--write-bin", str(o), str(t)).returncode == 0
        outs.append(open(o, "rb").read())
    assert outs[0] == outs[1] and len(outs[0]) == 24 + 8 * (300 * 2000 + 300 + 2000)


def test_truncated_binary(tmp_path):
    b1 = tmp_path / "a.spxlp"
    assert run("--no-solve", "--write-bin", str(b1), SAMPLE).returncode == 0
    data = open(b1, "rb").read()
    (tmp_path / "cut.spxlp").write_bytes(data[:-8])
    r = run("--no-solve", str(tmp_path / "cut.spxlp"))
    assert r.returncode == 1 and "truncated" in r.stderr


@pytest.mark.gpu
def test_binary_solve_matches_text(tmp_path):
    """Solving the .spxlp export gives the same stdout result block as the text file."""
    t, b1 = tmp_path / "g.txt", tmp_path / "g.spxlp"
    assert run("--no-solve", "--write-text", str(t), "--write-bin", str(b1), "--gen", "64", "256", "0").returncode == 0
    outs = []
    for f in (t, b1, None):
        args = ["--no-iter-lines", "--json"] + ([str(f)] if f else ["--gen", "64", "256", "0"])
        r = run(*args)
        assert r.returncode == 0, r.stderr
        lines = r.stdout.splitlines()
        outs.append(lines[:lines.index("")])
    assert outs[0] == outs[1] == outs[2] and outs[0][0].startswith("Optimum found: ")

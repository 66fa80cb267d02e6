"""bench.py's multi-rank watchdog, on the CPU with gloo at
world size 2: a rank stalled inside a watched phase, and its peer blocked in a
barrier, both report (rank, phase, pivots, dispatch stats) and exit 3 within
the bound instead of hanging; phases that end in time never fire."""
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HELPER = os.path.join(ROOT, "tests", "watchdog_rank.py")


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _launch(mode):
    port = _port()
    procs = []
    for r in range(2):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r), WORLD_SIZE="2",
                   LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, HELPER, mode], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    out = []
    for p in procs:
        try:
            o, e = p.communicate(timeout=45)
        except subprocess.TimeoutExpired:
            p.kill()
            o, e = p.communicate()
            raise AssertionError(f"rank hung past the watchdog: {e[-500:]}")
        out.append((p.returncode, o, e))
    return out


def test_watchdog_fires_on_stalled_rank():
    t0 = time.time()
    res = _launch("stall")
    assert time.time() - t0 < 40
    for rank, (rc, o, e) in enumerate(res):
        assert rc == 3, (rc, e[-800:])
        assert "unreachable" not in o
        line = [ln for ln in e.splitlines() if ln.startswith("bench.py: {")][-1]
        rep = json.loads(line[len("bench.py: "):])
        assert rep["rank"] == rank
        assert rep["phase"] == ("timed window" if rank == 1 else "next window 1")
        assert rep["pivots_at_last_readback"] == 1234
        assert rep["dispatch_stats"]["graph_launches"] == 7


def test_watchdog_quiet_when_phases_end():
    for rc, o, e in _launch("ok"):
        assert rc == 0, e[-800:]
        assert "done" in o and "bound exceeded" not in e

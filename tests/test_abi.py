"""CPU: the C-ABI library loads, exports every symbol include/simplex.h declares,
its struct layout matches the Python binding, and the host-only helpers (shard
ranges, MINLOC merge) behave.  No compute call needs a GPU here."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "simplex.h")


def declared_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(spx_[a-z_]+)\s*\(", txt)))


def test_header_functions_exported(spx):
    lib = spx._lib.load()
    names = declared_functions()
    assert len(names) >= 20
    for name in names:
        assert hasattr(lib, name), name


def test_binding_covers_header(spx):
    assert set(declared_functions()) == set(spx._lib.SIGNATURES)


def test_opts_layout_matches_header(spx, tmp_path):
    src = tmp_path / "layout.c"
    src.write_text(
        '#include <stdio.h>\n#include <stddef.h>\n#include "simplex.h"\n'
        "int main(void){printf(\"%zu %zu %zu %zu\\n\", sizeof(spx_opts), offsetof(spx_opts, device),"
        " offsetof(spx_opts, flags), offsetof(spx_opts, trace_cap));return 0;}\n")
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()
    S = spx._lib.SpxOpts
    assert [int(v) for v in out] == [ctypes.sizeof(S), S.device.offset, S.flags.offset, S.trace_cap.offset]


def test_default_opts(spx):
    o = spx._lib.SpxOpts()
    spx._lib.load().spx_default_opts(ctypes.byref(o))
    assert o.eps == 1e-7 and o.device == -1 and o.rank == 0 and o.nranks == 1


def test_status_strings(spx):
    L = spx._lib.load()
    assert L.spx_status_string(0) == b"MAX_ITER exceeded."
    assert L.spx_status_string(2) == b"Problem unbounded."
    assert L.spx_abi_version() == 8


def _has_gpu():
    return os.path.exists("/dev/kfd")


@pytest.mark.skipif(_has_gpu(), reason="checks the no-device error path")
def test_no_device_fails_loudly(spx):
    with pytest.raises(spx.SimplexError) as ei:
        spx.Context(m=4, n=8, seed=0)
    assert ei.value.code == -6  # SPX_ERR_NO_DEVICE: no silent CPU fallback


def test_argument_errors(spx):
    L = spx._lib.load()
    h = ctypes.c_void_p()
    A = np.zeros(6)
    rc = L.spx_create(ctypes.byref(h), 3, 2, A.ctypes.data, A.ctypes.data, A.ctypes.data, None)
    assert rc == -1  # m > n rejected (v4:402-405)
    assert b"m > n" in L.spx_last_error()
    assert L.spx_solve(None, 1, None, None, None, None, None) == -1


@pytest.mark.parametrize("m,n,G", [(4096, 16384, 1), (4096, 16384, 8), (7, 20, 3), (5, 5, 4), (1000, 1001, 8)])
def test_shard_ranges_partition_columns(spx, m, n, G):
    owner = np.full(n, -1)
    for r in range(G):
        s_lo, s_hi, k_lo, k_hi = spx.shard_range(m, n, r, G)
        assert 0 <= s_lo <= s_hi <= n - m <= k_lo <= k_hi <= n
        for j in list(range(s_lo, s_hi)) + list(range(k_lo, k_hi)):
            assert owner[j] == -1
            owner[j] = r
    assert np.all(owner >= 0)  # every column owned exactly once


def test_minloc_merge_rule(spx):
    # smallest value first, then smallest global index (CUB ArgMin, v4:294)
    assert spx.minloc_merge([-1.0, -3.0, -3.0, 0.0], [5, 9, 2, 1]) == (-3.0, 2)
    assert spx.minloc_merge([np.inf], [2**63 - 1]) == (np.inf, 2**63 - 1)
    assert spx.minloc_merge([], []) == (np.inf, 2**63 - 1)
    assert spx.minloc_merge([np.nan, 1.0], [0, 4]) == (1.0, 4)


def test_read_lp_matches_oracle_reader(spx, oracle):
    p = os.path.join(ROOT, "tests", "golden", "sample.txt")
    a = spx.read_lp(p)
    b = oracle.read_lp_text(p)
    assert a[0] == b[0] and a[1] == b[1]
    for x, y in zip(a[2:], b[2:]):
        assert np.array_equal(x, y)


def test_read_lp_ignores_trailing_text(spx, tmp_path):
    p = tmp_path / "t.txt"
    p.write_text("2 4\n1 1 1 0\n2 1 0 1\n4 5\n3 2 0 0\n\nExplanation: prose here\nOptimum: 9\n")
    m, n, A, b, c = spx.read_lp(str(p))
    assert (m, n) == (2, 4) and list(c) == [3, 2, 0, 0] and A.shape == (4, 2) and list(A[0]) == [1, 2]


def _info(r, G, bus, rccl=True):
    return {"rccl_nranks": G if rccl else -1, "rccl_rank": r if rccl else -1, "rccl_device": r, "device": r,
            "graph": True, "graph_fallback": False, "nranks": G, "rank": r, "bus_id": bus}


def test_check_ranks_rules(spx):
    """bench.py's multi-GPU evidence check (spx.check_ranks over the ranks'
    all-gathered spx_comm_info): RCCL must report the job's world size and
    each rank's own rank, and no two ranks may sit on one PCI bus id."""
    G = 8
    good = [_info(r, G, f"0000:{0x11 + r:02x}:00.0") for r in range(G)]
    spx.check_ranks(good, G)
    with pytest.raises(RuntimeError, match="RCCL communicator reports"):
        spx.check_ranks([dict(i, rccl_nranks=1) for i in good], G)
    with pytest.raises(RuntimeError, match="RCCL communicator reports"):
        spx.check_ranks(good[:1] + [dict(good[1], rccl_rank=0)] + good[2:], G)
    with pytest.raises(RuntimeError, match="share a GPU"):
        spx.check_ranks(good[:7] + [dict(good[7], bus_id=good[0]["bus_id"])], G)
    with pytest.raises(RuntimeError, match="rank records"):
        spx.check_ranks(good[:4], G)
    with pytest.raises(RuntimeError, match="created as rank"):
        spx.check_ranks([dict(i, nranks=4) for i in good], G)
    mbox = [_info(r, 2, "0000:11:00.0", rccl=False) for r in range(2)]  # --share-gpu rehearsal
    spx.check_ranks(mbox, 2, exchange="mbox", distinct_gpus=False)
    with pytest.raises(RuntimeError, match="share a GPU"):
        spx.check_ranks(mbox, 2, exchange="mbox")

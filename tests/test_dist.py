"""CPU, world_size 2 over gloo: the column-shard + MINLOC exchange design.

Each rank prices only its shard (spx_shard_range, the same host function the
device path uses) with the oracle, all-gathers its 16-byte (value, index)
candidate, and merges with spx_minloc_merge (the device's rule).  The merged
entering column must equal the single-process Dantzig choice at every pivot
of an oracle trajectory.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, root, out):
    import sys

    sys.path.insert(0, root)
    sys.path.insert(0, os.path.join(root, "oracle"))
    import torch
    import torch.distributed as dist

    import oracle
    import simplex_method_gpu_amd as spx

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    m, n, seed = 40, 160, 5
    A, b, c = oracle.generate(m, n, seed)
    ref = oracle.solve(A, b, c, trace_cap=100)
    s_lo, s_hi, k_lo, k_hi = spx.shard_range(m, n, rank, world)
    owned = np.zeros(n, dtype=bool)
    owned[s_lo:s_hi] = True
    owned[k_lo:k_hi] = True
    bad = 0
    for k in range(ref.pivots):
        st = oracle.solve(A, b, c, max_iter=k, want_state=True)
        e = oracle.price(A, c, st.y)
        nonbasic = np.ones(n, dtype=bool)
        nonbasic[st.b_ixs] = False
        cand = np.where(owned & nonbasic)[0]
        if len(cand):
            j = int(cand[np.argmin(e[cand])])  # first index among ties
            mine = torch.tensor([e[j], float(j)], dtype=torch.float64)
        else:
            mine = torch.tensor([np.inf, float(2**62)], dtype=torch.float64)
        gathered = [torch.zeros(2, dtype=torch.float64) for _ in range(world)]
        dist.all_gather(gathered, mine)
        vals = [float(t[0]) for t in gathered]
        idx = [int(t[1]) for t in gathered]
        _, p = spx.minloc_merge(vals, idx)
        bad += int(p != ref.trace_p[k])
    out[rank] = bad
    dist.destroy_process_group()


def test_two_rank_minloc_reproduces_dantzig():
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    world = 2
    mgr = mp.get_context("spawn").Manager()
    out = mgr.dict()
    mp.start_processes(_worker, args=(world, _free_port(), root, out), nprocs=world, join=True,
                       start_method="spawn")
    assert dict(out) == {0: 0, 1: 0}

"""Workload for rocprofv3 PMC passes: C3 (or --m/--n) with eager launches.
    rocprofv3 --pmc FETCH_SIZE --output-format csv -d DIR -o pmc -- python3 tools/pmc_run.py
--k 110 covers a fold (every 63 pivots); --tableau runs the window tableau with
two-kernel passes (no cooperative launch: a process that made one segfaults at
exit under rocprofv3, tools/gpu_profile.sh), so k_tab_fold is counted too.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import simplex_method_gpu_amd as spx  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--m", type=int, default=4096)
ap.add_argument("--n", type=int, default=16384)
ap.add_argument("--warmup", type=int, default=20)
ap.add_argument("--k", type=int, default=30)
ap.add_argument("--tableau", action="store_true")
a = ap.parse_args()
kw = {"tableau": True, "persist": False} if a.tableau else {}
with spx.Context(m=a.m, n=a.n, seed=0, device=0, graph_batch=-1, **kw) as ctx:
    ctx.iterate(a.warmup)
    st, piv = ctx.iterate(a.k)
    info = ctx.info()
print(f"pmc_run m={a.m} n={a.n} pivots={piv} local_nonbasic={info['local_nonbasic']}")

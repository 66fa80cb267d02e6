"""Rehearsal of the column-sharded pricing on ONE GPU: the
pricing kernel of one rank of G prices (n - m) / G non-basic columns, so its
time is measured here on a one-rank LP with the same m and n' = m + (n - m) / G
(the same kernel, column count and bytes; different random columns).  The
RCCL all-gather MINLOC is measured with a one-rank communicator (the
torch.distributed path of bench.py --comm1, passed in as --minloc-us); its
latency across G ranks over xGMI is NOT measured here.  Prints one JSON line:
per-G shard pricing time and the aggregate pricing throughput it implies,
all ranks' algorithmic bytes / (shard pricing + MINLOC).  A rehearsal, not a
hardware claim.
    python tools/shard_rehearsal.py [--m 4096 --n 131072] [--minloc-us 6.5]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import simplex_method_gpu_amd as spx  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--m", type=int, default=4096)
ap.add_argument("--n", type=int, default=131072)
ap.add_argument("--k", type=int, default=40)
ap.add_argument("--warm", type=int, default=20)
ap.add_argument("--minloc-us", type=float, default=6.5)
ap.add_argument("--window", type=int, default=64)
ap.add_argument("--gs", default="1,2,4,8", help="shard counts G")
ap.add_argument("--price-grid", default="0", help="k_price workgroups to try per G (comma list; 0 = the library's)")
a = ap.parse_args()
rows = []
for G in [int(g) for g in a.gs.split(",")]:
  for pg in [int(g) for g in a.price_grid.split(",")]:
    ns = (a.n - a.m) // G
    with spx.Context(m=a.m, n=a.m + ns, seed=0, device=0, timing=True, window=a.window, price_grid=pg) as ctx:
        ctx.iterate(a.warm)
        ctx.pass_times()
        ctx.iterate(a.k)
        pt = ctx.pass_times()
        grid = ctx.config()["price_grid"]
    price_us = 1e3 * pt["price_ms"] / max(pt["passes"], 1)
    shard_bytes = 8.0 * (a.m + 1) * ns
    rows.append({"G": G, "price_grid": grid, "shard_columns": ns, "shard_price_us": round(price_us, 2),
                 "shard_GBps": round(shard_bytes / (price_us * 1e-6) / 1e9, 1),
                 "aggregate_pricing_GBps": round(G * shard_bytes / ((price_us + a.minloc_us) * 1e-6) / 1e9, 1)})
base = max(r["aggregate_pricing_GBps"] for r in rows if r["G"] == rows[0]["G"])
for r in rows:
    r["pricing_speedup_vs_1"] = round(r["aggregate_pricing_GBps"] / base, 2)
print(json.dumps({"m": a.m, "n": a.n, "window": a.window, "minloc_us_assumed": a.minloc_us,
                  "note": "one GPU; shard LP n' = m + (n-m)/G; MINLOC latency over G ranks not measured",
                  "rows": rows}), flush=True)

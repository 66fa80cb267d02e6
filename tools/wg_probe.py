"""Per-workgroup clock of two consecutive compact window passes (stamps=True,
spx_wg_times), all on one clock (s_memrealtime, 100 MHz): pricing start /
deferred ratio-test tail reduced / staging in LDS / end, FTRAN entry / p
known / A_p in LDS / partial published, and the next pricing pass's start.
Samples after several iterate() calls on the default (graph) dispatch;
medians over samples, microseconds.
    python tools/wg_probe.py [--m 4096 --n 16384 --samples 12 --step 7]"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import simplex_method_gpu_amd as spx  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--m", type=int, default=4096)
ap.add_argument("--n", type=int, default=16384)
ap.add_argument("--samples", type=int, default=12)
ap.add_argument("--step", type=int, default=7)
ap.add_argument("--warm", type=int, default=70)
ap.add_argument("--eager", action="store_true", help="one launch pair per iterate() call")
ap.add_argument("--pricing", type=int, default=0, help="0 Dantzig, 1 Devex, 2 steepest edge")
a = ap.parse_args()
kw = dict(graph_batch=-1) if a.eager else {}
kw["pricing"] = a.pricing
S = {}


def put(k, v):
    S.setdefault(k, []).append(float(v) * 0.01)  # ticks -> us


ends = []
with spx.Context(m=a.m, n=a.n, seed=0, device=0, stamps=True, **kw) as ctx:
    ctx.iterate(a.warm)
    for _ in range(a.samples):
        ctx.iterate(a.step)
        w = ctx.wg_times()
        # the earlier pass: the one whose pricing started first
        lo, hi = (0, 1) if w[0]["price"][:, 0].min() < w[1]["price"][:, 0].min() else (1, 0)
        A, B = w[lo], w[hi]
        pa, fa, pb = (A["price"].astype(np.int64), A["ftran"].astype(np.int64), B["price"].astype(np.int64))
        fa = fa[fa[:, 0] > 0]  # (SPX_FTRAN_RPW > 1: fewer workgroups than partial slots)
        p0 = pa[:, 0].min()
        f0 = fa[:, 0].min()
        put("price_entry_spread", pa[:, 0].max() - p0)
        put("price_entry_to_tail_reduced", np.median(pa[:, 2] - pa[:, 0]))
        put("price_tail_reduced_to_staged", np.median(pa[:, 3] - pa[:, 2]))
        put("price_span", pa[:, 1].max() - p0)
        put("price_end_spread", pa[:, 1].max() - pa[:, 1].min())
        put("wg0_end_minus_p50_end", pa[0, 1] - np.median(pa[:, 1]))
        put("price_end_to_ftran_entry", f0 - pa[:, 1].max())
        if A["book"] > 0:  # workgroup 0's deferred bookkeeping, after its columns
            put("wg0_bookkeeping_issued_minus_last_end", int(A["book"]) - pa[:, 1].max())
            put("wg0_end_to_bookkeeping_issued", int(A["book"]) - pa[0, 1])
        put("ftran_entry_spread", fa[:, 0].max() - f0)
        put("ftran_entry_to_p", np.median(fa[:, 1] - fa[:, 0]))
        put("ftran_p_to_ap_lds", np.median(fa[:, 2] - fa[:, 1]))
        put("ftran_ap_to_publish_p50", np.median(fa[:, 3] - fa[:, 2]))
        put("ftran_publish_max", fa[:, 3].max() - f0)
        if A["tail"] > fa[:, 3].max():  # the FTRAN pass ran the tail itself
            put("publish_max_to_tail", int(A["tail"]) - fa[:, 3].max())
        put("ftran_publish_max_to_next_price", pb[:, 0].min() - fa[:, 3].max())
        put("pass_total", pb[:, 0].min() - p0)
        ends.append((pa[:, 1] - p0) * 0.01)
out = {k: {"p50": round(float(np.median(v)), 2), "min": round(float(np.min(v)), 2),
           "max": round(float(np.max(v)), 2)} for k, v in S.items()}
E = np.stack(ends)  # samples x price grid: each workgroup's end, from the pass's first start
g = np.arange(E.shape[1])
out["price_end_by_xcd"] = [round(float(E[:, g % 8 == x].mean()), 2) for x in range(8)]
out["price_end_by_wg_rank_corr"] = round(float(np.corrcoef(E[: len(E) // 2].mean(0), E[len(E) // 2:].mean(0))[0, 1]), 3)
out["price_end_p10_p50_p90_max"] = [round(float(np.percentile(E, q)), 2) for q in (10, 50, 90, 100)]
me = E.mean(0)
out["price_slowest_wg"] = [[int(b), round(float(me[b]), 2), round(float(E[:, b].std()), 2)] for b in np.argsort(-me)[:12]]
out["price_last_wg_counts"] = {int(k): int(v) for k, v in zip(*np.unique(E.argmax(1), return_counts=True))}
out["config"] = {"m": a.m, "n": a.n, "eager": a.eager, "samples": a.samples, "pricing": a.pricing,
                 "defer_tail": os.environ.get("SPX_DEFER_TAIL", "1") != "0"}
print(json.dumps(out, indent=1))

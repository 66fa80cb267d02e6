"""Per-workgroup clock of the compact FTRAN pass (k_ftran_bc, stamps=True):
when each workgroup starts, knows p, has A_p on the column list in LDS and
publishes its partial, relative to the earliest start, over several eager
passes.
    python tools/wg_probe.py [--m 4096 --n 16384 --passes 6]"""
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
ap.add_argument("--passes", type=int, default=6)
ap.add_argument("--warm", type=int, default=70)
a = ap.parse_args()
rows, prow = [], []
with spx.Context(m=a.m, n=a.n, seed=0, device=0, stamps=True, graph_batch=-1) as ctx:
    ctx.iterate(a.warm)
    for _ in range(a.passes):
        ctx.iterate(1)
        t = ctx.wg_times().astype(np.int64)
        t = (t - t[:, 0].min()) * 0.01  # us
        rows.append(t)
        pt = ctx.price_wg_times().astype(np.int64)
        prow.append((pt - pt[:, 0].min()) * 0.01)
T = np.stack(rows)  # passes x grid x 4
names = ["entry", "p_known", "ap_in_lds", "publish"]
out = {}
for k, nm in enumerate(names):
    v = T[:, :, k]
    out[nm] = {"p50": round(float(np.median(v)), 2), "p90": round(float(np.percentile(v, 90)), 2),
               "max": round(float(v.max()), 2)}
late = T[:, :, 3].mean(axis=0)
order = np.argsort(-late)[:12]
out["slowest_wg"] = [{"wg": int(g), "xcd": int(g % 8), "publish_us": round(float(late[g]), 2),
                      "entry_us": round(float(T[:, g, 0].mean()), 2), "p_us": round(float(T[:, g, 1].mean()), 2),
                      "ap_lds_us": round(float(T[:, g, 2].mean()), 2)} for g in order]
xcd = [round(float(late[np.arange(len(late)) % 8 == x].mean()), 2) for x in range(8)]
out["publish_mean_by_xcd"] = xcd
half = len(late) // 2
out["publish_mean_first_half_vs_second"] = [round(float(late[:half].mean()), 2), round(float(late[half:].mean()), 2)]
PT = np.stack(prow)  # passes x price grid x 2
pe = PT[:, :, 1]
out["price_wg_end"] = {"p10": round(float(np.percentile(pe, 10)), 2), "p50": round(float(np.median(pe)), 2),
                       "p90": round(float(np.percentile(pe, 90)), 2), "max": round(float(pe.max()), 2),
                       "start_max": round(float(PT[:, :, 0].max()), 2)}
out["price_wg_end_by_xcd"] = [round(float(pe.mean(axis=0)[np.arange(pe.shape[1]) % 8 == x].mean()), 2)
                              for x in range(8)]
print(json.dumps(out, indent=1))

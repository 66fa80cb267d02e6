"""Per-workgroup clock of the compact fold (k_cfold, stamps=True,
spx_fold_times) after two windows at C3 (or --m/--n): medians over the
working workgroups, microseconds from each workgroup's entry (xw_done:
the xw wave's end, y_done: the y wave's, yr == 0 workgroups only).
    python tools/cfold_probe.py [--m 4096 --n 16384]"""
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
a = ap.parse_args()
with spx.Context(m=a.m, n=a.n, seed=0, device=0, stamps=True) as ctx:
    ctx.iterate(130)
    f = ctx.fold_times().astype(np.int64)
    cfg = ctx.config()
w = f[f[:, 0] > 0]
e = w[:, 0]
out = {"workgroups": int(len(w)), "compact_fold": cfg["compact_fold"], "ftran_cols": None}
names = ["staged", "R_in_lds", "tiles_done", "vectors_done", "arrived", "xw_done", "y_done"]
for k, nm in enumerate(names, start=1):
    if nm is None:
        continue
    v = (w[:, k] - e) * 0.01
    ok = w[:, k] > 0
    out[nm] = {"p50": round(float(np.median(v[ok])), 2) if ok.any() else None,
               "max": round(float(np.max(v[ok])), 2) if ok.any() else None}
out["span_us"] = round(float((w[:, 5].max() - e.min()) * 0.01), 2)
out["entry_spread_us"] = round(float((e.max() - e.min()) * 0.01), 2)
print(json.dumps(out, indent=1))

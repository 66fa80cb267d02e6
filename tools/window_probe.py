"""Why does bench.py's first timed window differ from the windows after it?

For each config, builds the bench's context (spx_prepare'd), runs bench.py's
warm-up (W pivots, lead to the window boundary, one untimed whole window),
then times NW consecutive windows one by one (each between device syncs, as
bench.py's timed region and its next_windows are).  Variants:
  shift=1     one more untimed window first (the same pivot range as the base
              run's second window becomes the first timed one: data vs position)
  sleep=S     S seconds of host idle before every window
  prime=1     one eager pass + sync right before every window
Prints one JSON line per (config, variant) with the per-window it/s.

    python tools/window_probe.py [--configs C2,C3] [--nw 6] [--reps 2]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CONFIGS = {"C2": (1024, 4096, 100), "C3": (4096, 16384, 20), "C4": (4096, 131072, 20), "C5": (16384, 65536, 20)}


def run(spx, torch, m, n, steps_req, warmup, nw, shift=0, sleep=0.0, prime=0, stamps=False):
    ctx = spx.Context(m=m, n=n, seed=0, device=0, stamps=stamps)
    ctx.prepare()
    cfg = ctx.config()
    kw = cfg["window"]
    per = kw - 1 if kw else max(cfg["graph_batch"], 1)
    steps = per * max(1, -(-steps_req // per))
    ctx.iterate(warmup)
    lead = 0
    if kw:
        ds = ctx.dispatch_stats()
        lead = (kw - ds["window_pos"]) if ds["window_pos"] < kw else 0
    ctx.info()
    ctx.iterate(lead)
    _, piv = ctx.iterate(per * (1 + shift))
    ctx.dispatch_stats()
    out = []
    for _ in range(nw):
        if sleep:
            time.sleep(sleep)
        if prime:
            _, piv = ctx.iterate(prime)
        d0 = ctx.dispatch_stats()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        st, p1 = ctx.iterate(steps)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        d1 = ctx.dispatch_stats()
        inf = ctx.info()
        out.append({"it_s": round((p1 - piv) / dt, 1), "piv0": piv, "S": ctx.ftran_cols(),
                    "price_MB": round(inf["bytes_price"] / 1e6, 2),
                    "graphs": d1["graph_launches"] - d0["graph_launches"],
                    "eager": d1["eager_passes"] - d0["eager_passes"], "folds": d1["folds"] - d0["folds"]})
        piv = p1
        if st != 0:
            break
    ctx.close()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="C2,C3")
    ap.add_argument("--nw", type=int, default=6)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--variants", default="base,shift=1,sleep=0.05,prime=1")
    a = ap.parse_args()
    import torch
    import simplex_method_gpu_amd as spx
    torch.cuda.set_device(0)
    for rep in range(a.reps):
        for c in a.configs.split(","):
            m, n, steps = CONFIGS[c]
            for v in a.variants.split(","):
                kw = {}
                if "=" in v:
                    k, val = v.split("=")
                    kw[k] = float(val) if k == "sleep" else int(val)
                res = run(spx, torch, m, n, steps, 5, a.nw, **kw)
                print(json.dumps({"rep": rep, "config": c, "variant": v,
                                  "it_s": [r["it_s"] for r in res], "piv0": [r["piv0"] for r in res],
                                  "S": [r["S"] for r in res],
                                  "dispatch": [(r["graphs"], r["eager"], r["folds"]) for r in res]}), flush=True)


if __name__ == "__main__":
    main()

"""Fresh-process view of bench.py's timed windows (tools/window_probe.py runs
every variant in one process): each call is one process that builds the C3
context as bench.py's main run does and times NW windows one by one, after
an optional dummy context (created, iterated, closed) or host idle.

    python tools/window_fresh.py [--config C3] [--nw 10] [--pre none|ctx|idle]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--nw", type=int, default=10)
    ap.add_argument("--pre", default="none")
    ap.add_argument("--shift", type=int, default=0, help="untimed whole windows before the first timed one")
    a = ap.parse_args()
    import torch
    import simplex_method_gpu_amd as spx
    from window_probe import CONFIGS, run
    torch.cuda.set_device(0)
    m, n, steps = CONFIGS[a.config]
    t0 = time.time()
    if a.pre == "ctx":
        with spx.Context(m=m, n=n, seed=0, device=0) as c:
            c.iterate(200)
    elif a.pre == "idle":
        time.sleep(2.0)
    res = run(spx, torch, m, n, steps, 5, a.nw, shift=a.shift)
    print(json.dumps({"config": a.config, "pre": a.pre, "shift": a.shift, "it_s": [r["it_s"] for r in res],
                      "price_MB_end": [r["price_MB"] for r in res],
                      "piv0": [r["piv0"] for r in res], "S": [r["S"] for r in res],
                      "wall_s": round(time.time() - t0, 2)}), flush=True)


if __name__ == "__main__":
    main()

"""Tuning sweep on one GPU: per-kernel event times and in-kernel phase split for
a set of launch geometries.  python tools/sweep.py [--m 4096 --n 16384]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import simplex_method_gpu_amd as spx  # noqa: E402


def run(m, n, k, warm, **kw):
    with spx.Context(m=m, n=n, seed=0, device=0, timing=True, stamps=True, **kw) as ctx:
        ctx.iterate(warm)
        ctx.kernel_times()
        ctx.phase_times()
        t0 = time.perf_counter()
        st, piv0 = ctx.iterate(0)
        st, piv = ctx.iterate(k)
        dt = time.perf_counter() - t0
        kt = ctx.kernel_times()
        ph = ctx.phase_times()
        info = ctx.info()
    nl = max(kt["price_launches"], 1)
    return {
        "cfg": kw, "ms_per_iter": 1e3 * dt / max(piv - piv0, 1),
        "price_us": 1e3 * kt["price_ms"] / nl, "update_us": 1e3 * kt["update_ms"] / nl,
        "price_body_us": ph["price_body_us"] / nl, "price_tail_us": ph["price_tail_us"] / nl,
        "update_body_us": ph["update_body_us"] / nl, "update_tail_us": ph["update_tail_us"] / nl,
        **{k: v / nl for k, v in ph.items() if k.startswith("tail_") or "prologue" in k or "drain" in k},
        "update_GBps": 16.0 * m * m / (kt["update_ms"] / nl * 1e-3) / 1e9,
        "price_GBps": 8.0 * (m + 1) * info["local_nonbasic"] / (kt["price_ms"] / nl * 1e-3) / 1e9,
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=4096)
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--warm", type=int, default=10)
    ap.add_argument("--configs", default=None, help="JSON list of kwargs dicts")
    a = ap.parse_args()
    cfgs = json.loads(a.configs) if a.configs else [
        {"update_rows": 1}, {"update_rows": 2}, {"update_rows": 4}, {"update_rows": 8},
        {"price_block": 256}, {"price_block": 512}, {"price_block": 1024},
    ]
    for kw in cfgs:
        r = run(a.m, a.n, a.k, a.warm, **kw)
        print(json.dumps({k: (round(v, 2) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)


if __name__ == "__main__":
    main()

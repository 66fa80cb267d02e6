"""Persistent loop kernel phase split (timing mode): per-pass microseconds of
pricing / FTRAN / tail as seen by workgroup 0, plus graph-free ms/iteration.
    python tools/loop_probe.py [--m 4096 --n 16384 --k 189] [--kw '{"loop_block":512}']"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import simplex_method_gpu_amd as spx  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--m", type=int, default=4096)
ap.add_argument("--n", type=int, default=16384)
ap.add_argument("--k", type=int, default=189)
ap.add_argument("--kw", default="{}")
a = ap.parse_args()
kw = json.loads(a.kw)
with spx.Context(m=a.m, n=a.n, seed=0, device=0, timing=True, **kw) as ctx:
    cfg = ctx.config()
    ctx.iterate(63)
    ctx.loop_times()
    t0 = time.perf_counter()
    st, p0 = ctx.iterate(0)
    st, p1 = ctx.iterate(a.k)
    dt = time.perf_counter() - t0
    lt = ctx.loop_times()
n = max(lt["clock_passes"], 1)
print(json.dumps({"kw": kw, "persistent": cfg["persistent"], "loop_block": cfg["loop_block"],
                  "ms_per_iter_timed": round(1e3 * dt / max(p1 - p0, 1), 4),
                  "loop_us_per_pass": round(1e3 * lt["loop_ms"] / max(lt["loop_passes"], 1), 2),
                  "price_us": round(lt["price_us"] / n, 2), "ftran_us": round(lt["ftran_us"] / n, 2),
                  "tail_us": round(lt["tail_us"] / max(n - 1, 1), 2)}), flush=True)

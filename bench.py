"""Benchmark: dense revised-simplex iterations/s on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--m 4096 --n 16384]

A *step* is one simplex iteration (pricing over the non-basic columns, entering
MINLOC, fused B^-1 rank-1 update + FTRAN, ratio test, x_b / y update) on the
seeded dense random LP of SURVEY.md §8(d) (default C3: m=4096, n=16384, fp64),
with A, b, c generated directly in HBM.  W untimed iterations, then exactly K
timed ones between barriers + device syncs; rank 0 prints one JSON line.

Multi-GPU (torchrun, one process per GPU): pricing columns are sharded over the
ranks with an RCCL all-gather MINLOC per iteration, B^-1 is replicated, so the
whole job still does one iteration per step (strong scaling on a fixed LP).

roofline: the pricing kernel (dominant: 60 % of algorithmic bytes at C3),
algorithmic bytes = 8*(m+1)*(non-basic columns priced) per launch, duration
from hipEvents recorded by the kernel dispatch itself (hipExtLaunchKernel) on
the library's stream over the timed region.  cpu_baseline: the oracle
(oracle/simplex_oracle.c, OpenMP) on a bounded sample of the same workload.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--m", type=int, default=4096)
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="budget of the CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_r01.json"),
                    help="PMC-derived HBM bytes per launch (written by tools/pmc_traffic.py)")
    ap.add_argument("--update-rows", type=int, default=0)
    ap.add_argument("--price-block", type=int, default=0)
    ap.add_argument("--graph-batch", type=int, default=0)
    return ap.parse_args()


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("--gpus N > 1 must be launched with torch.distributed.run (one process per GPU)")
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    import simplex_method_gpu_amd as spx

    m, n = args.m, args.n

    def make(timing):
        ctx = spx.Context(m=m, n=n, seed=args.seed, device=local, rank=rank, nranks=world, timing=timing,
                          update_rows=args.update_rows, price_block=args.price_block,
                          graph_batch=args.graph_batch)
        if world > 1:
            obj = [spx.comm_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(obj, src=0)
            ctx.attach_comm(obj[0])
        return ctx

    def barrier():
        if world > 1:
            dist.barrier()

    def max_over_ranks(v):
        if world == 1:
            return v
        t = torch.tensor([v], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def timed_window(ctx):
        ctx.iterate(args.warmup)
        if ctx.info()["local_nonbasic"] < 0:
            raise RuntimeError("bad state")
        _, piv0 = ctx.iterate(0)
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        st, piv1 = ctx.iterate(args.steps)
        torch.cuda.synchronize()
        barrier()
        dt = max_over_ranks(time.perf_counter() - t0)
        return dt, piv1 - piv0, st

    # --- timed region with per-kernel hipEvents (eager dispatch)
    ctx = make(timing=True)
    info = ctx.info()
    ctx.iterate(args.warmup)
    ctx.kernel_times()  # reset the event pools after warmup
    _, piv0 = ctx.iterate(0)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    st, piv1 = ctx.iterate(args.steps)
    torch.cuda.synchronize()
    barrier()
    dt = max_over_ranks(time.perf_counter() - t0)
    kt = ctx.kernel_times()
    info_end = ctx.info()
    ctx.close()
    pivots = piv1 - piv0

    # --- the same window replayed from captured hipGraphs (no events)
    ctx = make(timing=False)
    dt_g, pivots_g, st_g = timed_window(ctx)
    ctx.close()

    # use the faster dispatch mode for `value`; the event-timed run gives the roofline
    if pivots_g > 0 and dt_g / pivots_g < dt / max(pivots, 1):
        best_dt, best_piv, mode = dt_g, pivots_g, "hipGraph replay"
    else:
        best_dt, best_piv, mode = dt, pivots, "eager + hipExtLaunchKernel events"
    value = best_piv / best_dt if best_dt > 0 else 0.0

    # algorithmic bytes; non-basic count is constant per rank
    # on average — use the mean of window start/end for this rank's pricing
    nb_local = 0.5 * (info["local_nonbasic"] + info_end["local_nonbasic"])
    price_bytes = 8.0 * (m + 1) * nb_local
    update_bytes = 16.0 * m * m
    price_ms = kt["price_ms"] / max(kt["price_launches"], 1)
    update_ms = kt["update_ms"] / max(kt["update_launches"], 1)
    price_gbs = price_bytes / (price_ms * 1e-3) / 1e9 if price_ms > 0 else 0.0
    update_gbs = update_bytes / (update_ms * 1e-3) / 1e9 if update_ms > 0 else 0.0
    b_alg = 8.0 * ((m + 1) * (n - m) + 2.0 * m * m)  # whole-iteration, all ranks

    traffic = None
    if os.path.exists(args.traffic_json):
        try:
            with open(args.traffic_json) as f:
                tj = json.load(f)
            if tj.get("m") == m and tj.get("n") == n:
                traffic = tj.get("price_hbm_bytes_per_launch")
        except Exception:
            traffic = None

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(m, n, args.seed, args.cpu_seconds)

    if rank == 0:
        out = {
            "metric": "simplex iterations/sec on dense m=4096 n=16384 fp64; achieved HBM GB/s",
            "value": value,
            "unit": "iterations/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * best_dt / max(best_piv, 1),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded generator of SURVEY.md §8(d), generated in HBM)",
            "config": {
                "workload": f"dense random LP m={m} n={n} seed={args.seed}, Dantzig revised simplex, "
                            f"explicit B^-1",
                "m": m, "n": n, "seed": args.seed,
                "parallelism": (f"pricing column-sharded x{world} (RCCL all-gather MINLOC), "
                                "B^-1 replicated") if world > 1 else "single GPU",
                "dispatch": mode,
            },
            "roofline": {
                "bound": "hbm",
                "kernel": "k_price (pricing GEMV + entering argmin)",
                "achieved": price_gbs,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": price_gbs / HBM_PEAK_GBS,
                "traffic": traffic,
                "algorithmic_bytes_per_launch": price_bytes,
                "avg_launch_ms": price_ms,
            },
            "kernels": {
                "k_update": {"avg_launch_ms": update_ms, "algorithmic_bytes_per_launch": update_bytes,
                             "achieved_GBps": update_gbs, "frac": update_gbs / HBM_PEAK_GBS},
                "iteration": {"algorithmic_bytes": b_alg,
                              "achieved_GBps": b_alg * value / 1e9,
                              "frac": b_alg * value / 1e9 / HBM_PEAK_GBS,
                              "event_timed_ms_per_step": 1e3 * dt / max(pivots, 1),
                              "graph_ms_per_step": 1e3 * dt_g / max(pivots_g, 1)},
            },
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline(m, n, seed, budget_s):
    """The oracle (fp64 C restatement, OpenMP) on a bounded sample: K iterations
    from the slack basis of the same LP, K sized to ~budget_s of CPU time."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle

    threads = oracle.max_threads()
    A, b, c = oracle.generate(m, n, seed)
    t1, d1 = oracle.time_iterations(A, b, c, 2, threads)
    per = t1 / max(d1, 1)
    k = int(max(3, min(500, budget_s / max(per, 1e-6))))
    sec, done = oracle.time_iterations(A, b, c, k, threads)
    return {"value": done / sec, "unit": "iterations/s", "cores": threads, "kind": "port",
            "sample": f"{done} iterations from the slack basis of the same m={m} n={n} LP "
                      f"(oracle/simplex_oracle.c, {threads} OpenMP threads, {sec:.1f} s)"}


if __name__ == "__main__":
    main()

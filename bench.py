"""Benchmark: dense revised-simplex iterations/s on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C3|C2|C4|C5 | --m M --n N]

A *step* is one simplex iteration (pricing over the non-basic columns, entering
MINLOC, FTRAN, ratio test, B^-1 update, x_b / y update) on the seeded dense
random LP of SURVEY.md §8(d) (default C3: m=4096, n=16384, fp64), with A, b, c
generated directly in HBM.

B^-1 is kept in the representation the library picks for (m, n) — the eta
window of 64 (B_w + U R) at m >= 2048 (C3, C4, C5), the explicit
inverse at C2 — at every N.  The window's rank-63 fold runs every 63 pivots, so
the timed region is aligned to whole windows — W untimed warm-up pivots, then untimed pivots up to the next window
boundary, then K rounded up to a multiple of 63 timed pivots -- at least
MIN_SPAN = 252 (four windows, about 19 ms at C3), so no single window's
transient sets the rate -- which therefore hold exactly K/63 folds (`timed_region` reports the pivots, folds and hipGraph
replays the library enqueued there, and `config.dispatch` is derived from
those counts).  `explicit` times the reference's own representation (explicit
B^-1 rewritten by a rank-1 update every pivot, v4:331-333) on the same LP with
the same clock.

Multi-GPU (torch.distributed.run, one process per GPU): the north-star
partitioning — pricing columns sharded over the ranks with an RCCL all-gather
MINLOC per iteration, B^-1 replicated, so N=1 runs the same representation as
N>1.  `--row-shard` instead row-shards an explicit B^-1
(SURVEY.md §8f row 1).  The job does one iteration per step on a fixed LP
("strong" scaling); `pricing` reports the aggregate pricing throughput (all
ranks' algorithmic pricing bytes / max-over-ranks of pricing kernel + MINLOC
time); `pricing_c4` measures the same on the north-star pricing-scaling config
(C4, m=4096 n=131072) at every N, so the SCALE lines give its 1 -> N speedup.

roofline: the pricing kernel (dominant: 60 % of the algorithmic bytes at C3),
algorithmic bytes = 8*(m+1)*(non-basic columns priced on this rank) per launch,
duration from hipEvents recorded by the kernel dispatch itself
(hipExtLaunchKernel) on the library's stream over an event-timed copy of the
same window; traffic = rocprofv3 PMC bytes per launch (profiles/traffic_rNN.json).
cpu_baseline: the oracle (oracle/simplex_oracle.c, OpenMP) on a bounded sample
of the same workload (rank 0, N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

class Watchdog:
    """Multi-rank bench guard (one per rank): each phase of the run (a timed
    window, the next windows, one spx_iterate call of the whole solve, ...)
    is armed with a bound; if the phase has not ended by then -- a lost peer,
    a hung all-gather or mailbox poll -- this rank prints its rank, the phase,
    the host's pivot count and spx_dispatch_stats to stderr and exits with
    status 3 from a watcher thread (os._exit: no re-exec, nothing else runs on
    the GPU).  Off (seconds <= 0) on one rank unless asked for."""

    EXIT = 3

    def __init__(self, seconds, rank, out=None):
        import threading

        self.seconds = float(seconds)
        self.rank = rank
        self.out = out or sys.stderr
        self._cv = threading.Condition()
        self._phase = None
        self._deadline = None
        self._ctx = None
        self._gen = 0
        if self.seconds > 0:
            threading.Thread(target=self._watch, name="bench-watchdog", daemon=True).start()

    def arm(self, phase, ctx=None, seconds=None):
        with self._cv:
            self._phase, self._ctx = phase, ctx
            self._deadline = time.monotonic() + (self.seconds if seconds is None else float(seconds))
            self._gen += 1
            self._cv.notify()

    def disarm(self):
        with self._cv:
            self._phase = self._deadline = self._ctx = None
            self._gen += 1
            self._cv.notify()

    def phase(self, name, ctx=None, seconds=None):
        wd = self

        class _P:
            def __enter__(self_):
                wd.arm(name, ctx, seconds)
                return wd

            def __exit__(self_, *exc):
                wd.disarm()
        return _P()

    def _report(self, phase, ctx):
        msg = {"watchdog": "bound exceeded", "rank": self.rank, "phase": phase, "bound_s": self.seconds}
        if ctx is not None:
            try:
                msg["dispatch_stats"] = ctx.dispatch_stats()
                msg["pivots_at_last_readback"] = getattr(ctx, "last_pivots", None)
            except Exception as e:  # the report must not hang or raise
                msg["dispatch_stats"] = f"unavailable: {e}"
        print("bench.py: " + json.dumps(msg), file=self.out, flush=True)

    def _watch(self):
        while True:
            with self._cv:
                while self._deadline is None:
                    self._cv.wait()
                gen, left = self._gen, self._deadline - time.monotonic()
                if left > 0:
                    self._cv.wait(left)
                    continue
                if gen != self._gen:
                    continue
                phase, ctx = self._phase, self._ctx
            self._report(phase, ctx)
            os._exit(self.EXIT)


HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
# The shortest timed span, in pivots (rounded up to whole windows / batches).
# One 63-pivot window measured 0.4-1.6 % below the windows after it in bench
# runs (tools/window_probe.py, window_fresh.py: the first window after the
# warm-up streams slightly more pricing bytes -- fewer slack columns have left
# the basis -- and is the first replay timed); four windows make the rate
# representative of the sustained one (timed_region.next_windows_it_per_s).
MIN_SPAN = 252


def span(k, per):
    """K pivots rounded up to whole units of `per`, at least MIN_SPAN."""
    return per * max(-(-k // per), -(-MIN_SPAN // per), 1)
CONFIGS = {"C2": (1024, 4096), "C3": (4096, 16384), "C4": (4096, 131072), "C5": (16384, 65536)}
METRIC = "simplex iterations/sec on dense m={m} n={n} fp64; achieved HBM GB/s"  # BASELINE.json at C3


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", choices=sorted(CONFIGS), default=None)
    ap.add_argument("--m", type=int, default=None)
    ap.add_argument("--n", type=int, default=None)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="budget of the CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_r06.json"),
                    help="PMC-derived HBM bytes per launch (tools/pmc_traffic.py)")
    ap.add_argument("--update-rows", type=int, default=0)
    ap.add_argument("--update-block", type=int, default=0)
    ap.add_argument("--price-block", type=int, default=0)
    ap.add_argument("--graph-batch", type=int, default=0)
    ap.add_argument("--window", type=int, default=0,
                    help="B^-1 representation: 0 = the library's choice (eta window 64 at m >= 2048, "
                         "explicit below and with --row-shard), "
                         "-1 explicit rank-1 update, 8/16/32/64 eta window")
    ap.add_argument("--row-shard", action="store_true",
                    help="N > 1: row-shard an explicit B^-1 over the ranks (SURVEY.md §8f row 1) "
                         "instead of replicating the eta window")
    ap.add_argument("--persist", choices=["auto", "on", "off"], default="auto",
                    help="persistent loop kernel (k_loop): the library's choice, forced on, or two-kernel passes")
    ap.add_argument("--no-explicit", action="store_true", help="skip the explicit-B^-1 block")
    ap.add_argument("--no-sharded-pricing", action="store_true",
                    help="skip the C4 column-sharded pricing block (pricing_c4)")
    ap.add_argument("--no-tableau", action="store_true",
                    help="skip the window-tableau measurement (the `tableau` block, one GPU only)")
    ap.add_argument("--no-solve-to-optimum", action="store_true",
                    help="skip the whole-solve block (the same LP from the slack basis to optimality)")
    ap.add_argument("--no-steepest", action="store_true",
                    help="skip the steepest-edge block (one GPU, eta window)")
    ap.add_argument("--comm1", action="store_true",
                    help="rehearsal on one GPU: run the multi-rank path (torch.distributed + RCCL "
                         "MINLOC) with a one-rank communicator")
    ap.add_argument("--minloc", choices=["rccl", "mbox"], default="rccl",
                    help="N > 1: the pricing MINLOC exchange as an RCCL all-gather (default) or as direct "
                         "stores into the peers' mailboxes (spx_mbox_attach, one small kernel per pass)")
    ap.add_argument("--watchdog", type=float, default=None,
                    help="seconds a phase (a timed window, one iterate call of the whole solve, ...) may take "
                         "before this rank reports where it is and exits 3 (default: 120 with N > 1, off on one rank)")
    ap.add_argument("--share-gpu", action="store_true",
                    help="rehearsal of --gpus N on a one-GPU box: every rank on GPU 0 (gloo process group, "
                         "mailbox MINLOC; RCCL refuses two ranks on one device). Exercises the multi-rank "
                         "bench path; its timings are not a scaling measurement")
    a = ap.parse_args()
    m, n = CONFIGS[a.config or "C3"]
    a.m = a.m or m
    a.n = a.n or n
    if a.window == 0:
        a.window = -1 if a.row_shard else 0
    return a


def describe_dispatch(d):
    """What the library enqueued in the timed region (spx_dispatch_stats deltas)."""
    parts = []
    if d["graph_launches"]:
        parts.append(f"{d['graph_launches']} hipGraph replays x {d['graph_passes'] // d['graph_launches']} passes")
    if d["persistent_launches"]:
        parts.append(f"{d['persistent_launches']} persistent k_loop launches ({d['persistent_passes']} passes)")
    if d["eager_passes"]:
        parts.append(f"{d['eager_passes']} eager passes")
    return " + ".join(parts) + f"; {d['folds']} folds" if parts else "nothing enqueued"


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world == 1 and args.gpus > 1:
        raise SystemExit("--gpus N > 1 must be launched with torch.distributed.run (one process per GPU)")
    if args.share_gpu:  # rehearsal: every rank on GPU 0, gloo process group, mailbox MINLOC
        local = 0
        args.minloc = "mbox"
    torch.cuda.set_device(local)
    multi = world > 1 or args.comm1  # the multi-rank code path (RCCL exchange)
    if multi:
        if args.share_gpu:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    import simplex_method_gpu_amd as spx

    wd = Watchdog(args.watchdog if args.watchdog is not None else (120.0 if multi else 0.0), rank)
    m, n = args.m, args.n
    row_shard = multi and args.row_shard

    def make(timing, window, mm=None, nn=None):
        ctx = spx.Context(m=mm or m, n=nn or n, seed=args.seed, device=local, rank=rank, nranks=world, timing=timing,
                          update_rows=args.update_rows, update_block=args.update_block,
                          price_block=args.price_block, graph_batch=args.graph_batch,
                          row_shard=row_shard and window < 0, window=window,
                          comm1=(args.comm1 and world == 1),
                          persist={"auto": None, "on": True, "off": False}[args.persist])
        if multi and (args.minloc == "rccl" or (row_shard and window < 0)):
            obj = [spx.comm_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(obj, src=0)
            ctx.attach_comm(obj[0])
        if multi and args.minloc == "mbox":  # MINLOC by k_exchange through the peer mailboxes
            hs = [None] * world
            dist.all_gather_object(hs, ctx.mbox_export())
            ctx.mbox_attach(hs)
        # the batch hipGraph is captured, instantiated and uploaded here (one
        # rank: already by spx_create; with RCCL or mailboxes only now that
        # they are attached), never inside a timed region
        ctx.prepare()
        return ctx

    def barrier():
        if multi:
            dist.barrier()

    def reduce_max(vals):
        if not multi:
            return list(vals)
        t = torch.tensor(list(vals), dtype=torch.float64, device="cpu" if args.share_gpu else "cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return t.tolist()

    def reduce_sum(vals):
        if not multi:
            return list(vals)
        t = torch.tensor(list(vals), dtype=torch.float64, device="cpu" if args.share_gpu else "cuda")
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return t.tolist()

    def timed_window(window, events, spread=False):
        """W warm-up pivots, untimed pivots to the next window boundary, one
        more untimed whole window (so the timed passes are not the batch
        graph's first replay), then K (rounded up to whole windows) timed
        pivots between barriers and device syncs.  Returns the max-over-ranks
        time and what ran; with `spread`, also the max-over-ranks times of the
        next three windows, each timed on its own."""
        with wd.phase("context + warm-up" + (" (event-timed)" if events else "")):
            ctx = make(events, window)
        wd.arm("warm-up" + (" (event-timed)" if events else ""), ctx)
        cfg = ctx.config()
        kw = cfg["window"]
        # whole windows (eta window), or whole captured batches of passes
        # (explicit B^-1: the timed region replays graphs, as the window's does)
        per = kw - 1 if kw else max(cfg["graph_batch"], 1)
        warm = per
        steps = span(args.steps, per)
        ctx.iterate(args.warmup)
        lead = 0
        if kw:
            ds = ctx.dispatch_stats()
            lead = (kw - ds["window_pos"]) if ds["window_pos"] < kw else 0
        info0 = ctx.info()  # (readbacks first: the lead passes run right before the timed region)
        ctx.iterate(lead)  # the next pass starts with a fold
        _, piv0 = ctx.iterate(warm)  # one whole untimed window / batch: a graph replay where the library captures
        if events:
            ctx.pass_times()  # drop the warm-up's and the lead's events
            ctx.loop_times()
        d0 = ctx.dispatch_stats()
        wd.arm("timed window" + (" (event-timed)" if events else ""), ctx)
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        st, piv1 = ctx.iterate(steps)
        torch.cuda.synchronize()
        # this rank's span ends at its device sync; the closing barrier only
        # re-aligns the ranks (with NCCL it is an all-reduce of its own,
        # 1-3 % of a C3 span when it was inside the clock); the job's time
        # is the max over ranks of the spans, which all began after one barrier
        t_end = time.perf_counter()
        barrier()
        dt = reduce_max([t_end - t0])[0]
        d1 = ctx.dispatch_stats()
        # the averages behind the roofline cover the timed region, not the
        # windows timed after it
        info1 = ctx.info()
        cols = ctx.ftran_cols()
        delta = {k: d1[k] - d0[k] for k in ("eager_passes", "graph_launches", "graph_passes",
                                            "persistent_launches", "persistent_passes", "folds", "graph_builds")}
        windows = None
        if spread and st == 0:
            ts, pv = [], piv1
            for k in range(3):
                wd.arm(f"next window {k + 1}", ctx)
                barrier()
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                _, p2 = ctx.iterate(steps)
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t1)
                ts[-1] = ts[-1] / max(p2 - pv, 1)
                pv = p2
            windows = reduce_max(ts)
        pt = lt = None
        if events:
            lt = ctx.loop_times()  # fold events (and the persistent loop's phases)
            pt = ctx.pass_times()
            if cfg["persistent"]:
                # persistent loop kernel (k_loop): phases timed in-kernel by
                # workgroup 0 (pricing to grid barrier 1, FTRAN to barrier 2)
                np_ = max(lt["clock_passes"], 1)
                pt = {"passes": np_, "price_ms": 1e-3 * lt["price_us"],
                      "price_minloc_ms": 1e-3 * lt["price_us"], "update_ms": 1e-3 * lt["ftran_us"],
                      "loop_ms_per_pass": lt["loop_ms"] / max(lt["loop_passes"], 1)}
        wd.arm("readback", ctx)
        comm = ctx.comm_info()
        ctx.close()
        wd.disarm()
        return {"cfg": cfg, "dt": dt, "pivots": piv1 - piv0, "steps": steps, "lead": lead + warm, "dispatch": delta,
                "windows_s_per_pivot": windows,
                "pt": pt, "lt": lt, "nb": 0.5 * (info0["local_nonbasic"] + info1["local_nonbasic"]),
                "price_bytes": 0.5 * (info0["bytes_price"] + info1["bytes_price"]), "ftran_cols": cols,
                "status": int(st), "comm": comm}

    def kernel_split(run, window):
        """Per-kernel averages of an event-timed run, with algorithmic bytes."""
        pt, lt = run["pt"], run["lt"]
        passes = max(pt["passes"], 1)
        price_ms = pt["price_ms"] / passes
        minloc_ms = pt["price_minloc_ms"] / passes
        update_ms = pt["update_ms"] / passes
        # this rank's launch: the streamed non-basic columns
        # (non-basic slacks are priced without their column, spx_info)
        price_bytes = run["price_bytes"]
        # B^-1 bytes of the update launch: read + write (explicit rank-1
        # update), or the read-only FTRAN stream of the eta window: its
        # non-unit columns with the compact operand (spx_ftran_cols, as of the
        # window's last fold: an upper bound over the window)
        update_bytes = 8.0 * m * run["ftran_cols"] if window > 0 else 16.0 * m * m
        fold_ms = lt["fold_ms"] / lt["folds"] if lt and lt["folds"] else 0.0
        return {"price_ms": price_ms, "minloc_ms": minloc_ms, "update_ms": update_ms,
                "price_bytes": price_bytes, "update_bytes": update_bytes, "fold_ms": fold_ms,
                "folds": int(lt["folds"]) if lt else 0}

    win = args.window
    # (1) the measured run: undisturbed (no events), graph replay where the
    #     library captures, timed over whole windows
    main_run = timed_window(win, False, spread=True)
    cfg = main_run["cfg"]
    win = cfg["window"]
    value = main_run["pivots"] / main_run["dt"] if main_run["dt"] > 0 else 0.0
    # evidence of what joined the job: every rank's own RCCL communicator
    # size / rank, HIP device and PCI bus id, and graph capture, all-gathered
    # and checked (rc != 0 on a mismatch: the line would not be a N-GPU run)
    infos = [main_run["comm"]]
    if multi:
        infos = [None] * world
        dist.all_gather_object(infos, main_run["comm"])
    exchange = ("rccl" if args.minloc == "rccl" else "mbox") if multi else "none"
    try:
        spx.check_ranks(infos, world, exchange=exchange, distinct_gpus=not args.share_gpu)
    except RuntimeError as e:
        if multi:
            dist.destroy_process_group()
        raise SystemExit(f"bench.py: rank evidence check failed: {e}")
    # (2) the same window with per-dispatch hipEvents (eager): kernel split
    ev_run = timed_window(args.window, True)
    ks = kernel_split(ev_run, win)
    price_ms_max, minloc_ms_max, update_ms_max = reduce_max([ks["price_ms"], ks["minloc_ms"], ks["update_ms"]])
    price_bytes_all = reduce_sum([ks["price_bytes"]])[0]
    price_gbs = ks["price_bytes"] / (ks["price_ms"] * 1e-3) / 1e9 if ks["price_ms"] > 0 else 0.0
    update_gbs = ks["update_bytes"] / (ks["update_ms"] * 1e-3) / 1e9 if ks["update_ms"] > 0 else 0.0
    # fold: dense -- B_w read + written, U / Qrows read once
    # per window; compact (k_cfold) -- the operand's S columns read, written
    # and scattered into the dense B_w, U read once
    S_end = ev_run["ftran_cols"]
    if win and cfg.get("compact_fold"):
        fold_bytes = 8.0 * m * (3.0 * S_end + win)
    else:
        fold_bytes = 16.0 * m * m + 8.0 * win * 2 * m if win else 0.0
    b_upd = 8.0 * m * S_end + fold_bytes / (win - 1) if win else 16.0 * m * m
    b_moved = price_bytes_all + b_upd                       # this representation, per pivot
    b_alg = 8.0 * (m + 1) * (n - m) + 16.0 * m * m         # SURVEY.md §8(d) B_alg, per pivot

    traffic = None
    if os.path.exists(args.traffic_json):
        try:
            with open(args.traffic_json) as f:
                tj = json.load(f)
            if tj.get("m") == m and tj.get("n") == n and world == 1:
                traffic = tj.get("price_hbm_bytes_per_launch")
        except (OSError, ValueError):
            traffic = None

    explicit = None
    if not args.no_explicit and win > 0 and not row_shard:
        explicit = explicit_block(timed_window, kernel_split, reduce_max, m, n)

    sharded = None
    if not args.no_sharded_pricing and (m, n) != CONFIGS["C4"]:
        with wd.phase("pricing_c4 (C4 sharded pricing window)"):
            sharded = sharded_pricing_block(make, reduce_max, reduce_sum, world, args)

    to_opt = None
    if not args.no_solve_to_optimum:
        to_opt = solve_to_optimum_block(make, barrier, reduce_max, torch, args.window, main_run, value, wd)

    steep = None
    if world == 1 and not multi and not args.no_steepest and win > 0:
        steep = steepest_block(spx, torch, m, n, args, local)

    tab = None
    if world == 1 and not multi and not args.no_tableau:
        tab = tableau_block(spx, torch, m, n, args, local)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(m, n, args.seed, args.cpu_seconds)
        cpu["glpk"] = glpk_status()

    if rank == 0:
        fc = ev_run["ftran_cols"]
        rep = (("eta window %d: B_w + U R, FTRAN stream read-only, rank-%d fold every %d pivots" % (win, win - 1, win - 1)
                + ("; B_w's non-unit columns only (compact FTRAN operand, %d of %d columns at the window's end)"
                   % (fc, m) if fc < m else ""))
               if win else "explicit B^-1, rank-1 update in place every pivot (v4:331-333)")
        out = {
            "metric": METRIC.format(m=m, n=n),
            "value": value,
            "unit": "iterations/s",
            "n_gpus": world,
            "steps": main_run["pivots"],
            "steps_requested": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * main_run["dt"] / max(main_run["pivots"], 1),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded generator of SURVEY.md §8(d), generated in HBM)",
            "config": {
                "workload": f"dense random LP m={m} n={n} seed={args.seed}, Dantzig revised simplex, "
                            f"one step = one pivot; {rep}",
                "b_inverse": rep,
                "geometry": cfg,
                "m": m, "n": n, "seed": args.seed,
                "parallelism": ((f"pricing column-sharded x{world} " +
                                 ("(RCCL all-gather MINLOC), " if args.minloc == "rccl" else
                                  "(MINLOC through peer mailboxes, k_exchange), ") +
                                 ("explicit B^-1 row-sharded (pivot row in a 2nd all-gather)" if row_shard else
                                  "B^-1 replicated"))
                                if multi else "single GPU"),
                "dispatch": describe_dispatch(main_run["dispatch"]),
            },
            "ranks": {
                "world_size": world,
                "exchange": exchange,
                "rccl_nranks": infos[0]["rccl_nranks"],
                "per_rank": [{"rank": i["rank"], "rccl_rank": i["rccl_rank"], "device": i["device"],
                              "rccl_device": i["rccl_device"], "bus_id": i["bus_id"],
                              "graph_captured": i["graph"], "graph_fallback": i["graph_fallback"]}
                             for i in infos],
                "checked": "spx.check_ranks: RCCL reports world_size ranks and each rank's own rank"
                           + ("; distinct PCI bus ids" if not args.share_gpu else
                              " (bus ids shared on purpose: --share-gpu rehearsal)"),
            },
            "timed_region": {
                "pivots": main_run["pivots"],
                "steps_rounding": ((f"K rounded up to whole windows of {win - 1} pivots" if win else
                                    f"K rounded up to whole captured batches of {cfg['graph_batch']} passes")
                                   + f", at least {MIN_SPAN} pivots (one window's transient does not set the rate)"
                                   if cfg["graph_batch"] > 0 else "none"),
                "clock": "barrier + device sync, then t0; the K pivots; device sync, then t1 on each rank; "
                         "barrier; value uses the max over ranks of t1 - t0",
                "untimed_pivots_before": args.warmup + main_run["lead"],
                "folds": main_run["dispatch"]["folds"],
                "graph_launches": main_run["dispatch"]["graph_launches"],
                "graph_passes": main_run["dispatch"]["graph_passes"],
                "eager_passes": main_run["dispatch"]["eager_passes"],
                "persistent_launches": main_run["dispatch"]["persistent_launches"],
                "graph_builds": main_run["dispatch"]["graph_builds"],
                "warm_up": "W pivots, then untimed pivots to the window boundary and one more untimed whole "
                           "window (a graph replay); the batch graph was built before any of them (spx_prepare)",
                "next_windows_it_per_s": ([1.0 / t for t in main_run["windows_s_per_pivot"]]
                                          if main_run["windows_s_per_pivot"] else None),
                "next_windows_spread": ((max(main_run["windows_s_per_pivot"]) / min(main_run["windows_s_per_pivot"])
                                         - 1.0) if main_run["windows_s_per_pivot"] else None),
            },
            "roofline": {
                "bound": "hbm",
                "kernel": ("k_loop pricing phase (in-kernel clock, workgroup 0), rank 0" if cfg.get("persistent")
                           else "k_price (pricing GEMV + entering argmin"
                           + (", prologue: the previous pivot's deferred ratio-test reduction" if cfg.get("defer_tail")
                              else "") + "), rank 0"),
                "achieved": price_gbs,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": price_gbs / HBM_PEAK_GBS,
                "traffic": traffic,
                "algorithmic_bytes_per_launch": ks["price_bytes"],
                "avg_launch_ms": ks["price_ms"],
            },
            "kernels": {
                "k_update": {"what": ("rank-1 update (RMW) + FTRAN" if not win else
                                      "FTRAN (B_w read-only) + ratio-test partials; the leaving argmin and the "
                                      "bookkeeping run in the next k_price (deferred tail)" if cfg.get("defer_tail")
                                      else "FTRAN (B_w read-only) + ratio test"),
                             "avg_launch_ms": ks["update_ms"], "algorithmic_bytes_per_launch": ks["update_bytes"],
                             "achieved_GBps": update_gbs, "frac": update_gbs / HBM_PEAK_GBS},
                "k_fold": ({"kernels": ("k_bc_list + k_cfold (the listed columns of B_w only)"
                                        if cfg.get("compact_fold") else "k_fold + k_bc_list + k_bc_gather"),
                            "avg_launch_ms": ks["fold_ms"], "launches_timed": ks["folds"],
                            "per_pivot_ms": ks["fold_ms"] / (win - 1),
                            "algorithmic_bytes_per_launch": fold_bytes,
                            "achieved_GBps": fold_bytes / (ks["fold_ms"] * 1e-3) / 1e9 if ks["fold_ms"] > 0 else 0.0}
                           if win else None),
                # whole-iteration roofline of this representation: the bytes
                # it moves per pivot (pricing stream, FTRAN operand, fold / 63)
                # over the pivot time.  SURVEY.md §8(d)'s B_alg counts the
                # explicit representation's per-pivot B^-1 rewrite, which the
                # window never does, so B_alg / time is only an equivalent
                # rate, not a fraction of peak (the explicit block's
                # iteration.frac is that representation's own roofline)
                "iteration": {"algorithmic_bytes": b_moved,
                              "achieved_GBps": b_moved * value / 1e9,
                              "frac": b_moved * value / 1e9 / HBM_PEAK_GBS,
                              "bytes_survey_B_alg": b_alg,
                              "equivalent_GBps_survey": b_alg * value / 1e9,
                              "explicit_iteration_frac": explicit["iteration"]["frac"] if explicit else None,
                              "event_timed_ms_per_step": 1e3 * ev_run["dt"] / max(ev_run["pivots"], 1),
                              "event_timed_dispatch": describe_dispatch(ev_run["dispatch"])},
            },
            "pricing": {
                "bytes_all_ranks": price_bytes_all,
                "max_rank_price_ms": price_ms_max,
                "max_rank_price_plus_minloc_ms": minloc_ms_max,
                "throughput_GBps": price_bytes_all / (minloc_ms_max * 1e-3) / 1e9 if minloc_ms_max > 0 else 0.0,
                "max_rank_update_ms": update_ms_max,
            },
            "solve_to_optimum": to_opt,
            "steepest": steep,
            "explicit": explicit,
            "pricing_c4": sharded,
            "tableau": tab,
            "cpu_baseline": cpu,
        }
        if args.share_gpu:
            out["rehearsal"] = (f"{world} ranks share one GPU (--share-gpu: gloo process group, mailbox MINLOC); "
                                "checks the multi-rank path, not a scaling number")
        print(json.dumps(out), flush=True)
    if multi:
        dist.destroy_process_group()


SOLVE_CHUNKS = "16, 32, ..., 2048, then 2048 per call"


def run_to_exit(ctx, arm=None):
    """Iterate from the current basis until the solve terminates, in
    spx_solve's chunks (spx_api.cpp, `spx_solve`: 16 pivots, doubling to 2,048
    per spx_iterate call; the status is read back after each call). A call
    enqueues all its passes, so the passes after the optimum inside the last
    call price nothing (the larger the chunk, the more of them).
    Returns (status, pivots, calls)."""
    st, piv = ctx.iterate(0)
    chunk, calls = 16, 0
    while st == 0:  # SolveStatus.MaxIter: not terminated yet
        if arm is not None:
            arm(chunk, piv)  # one call's bound
        st, piv = ctx.iterate(chunk)
        calls += 1
        chunk = min(2 * chunk, 2048)
    return st, piv, calls


def calls_passes(calls):
    """Passes enqueued by `calls` spx_iterate calls of run_to_exit's schedule."""
    tot, chunk = 0, 16
    for _ in range(calls):
        tot += chunk
        chunk = min(2 * chunk, 2048)
    return tot


def solve_to_optimum_block(make, barrier, reduce_max, torch, window, main_run, value, wd):
    """The whole solve of the headline LP: the default path from the slack
    basis to optimality on the same clock as `value` (barrier + device sync on
    both sides, max over ranks), dispatched as the library does it (captured
    hipGraphs of whole windows plus a few eager passes at the ends of each
    spx_iterate call; spx_solve's chunk schedule, `run_to_exit`).  `value` samples an early window, where the compact
    FTRAN operand is narrow (S columns of B_w that are not unit); S grows over
    the solve, and so does the FTRAN pass."""
    with wd.phase("solve_to_optimum: context"):
        ctx = make(False, window)
    try:
        cols0 = ctx.ftran_cols()
        wd.arm("solve_to_optimum: start", ctx)
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        st, piv, calls = run_to_exit(ctx, lambda k, p: wd.arm(f"solve_to_optimum: iterate({k}) from pivot {p}", ctx))
        wd.arm("solve_to_optimum: end", ctx)
        torch.cuda.synchronize()
        t_end = time.perf_counter()  # (the closing barrier outside the clock, as in timed_window)
        barrier()
        dt = reduce_max([t_end - t0])[0]
        cols1 = ctx.ftran_cols()
        z = ctx.objective()
        ds = ctx.dispatch_stats()
    finally:
        ctx.close()
        wd.disarm()
    rate = piv / dt if dt > 0 else 0.0
    return {"status": ["MaxIter", "OptimumFound", "Unbounded", "ThetaOverflow"][int(st)], "pivots": int(piv),
            "seconds": dt, "iterations_per_s": rate, "z": z,
            "ftran_cols_start": cols0, "ftran_cols_end": cols1,
            "vs_value": rate / value if value > 0 else None,
            "dispatch": f"{ds['graph_launches']} hipGraph replays ({ds['graph_passes']} passes) + "
                        f"{ds['eager_passes']} eager passes; {ds['folds']} folds; {calls} spx_iterate calls "
                        f"({SOLVE_CHUNKS}), {calls_passes(calls) - piv} passes after the optimum",
            "note": "time to optimum from the slack basis (the v4:286-359 loop run to its exit, as the "
                    "reference CLI times it at v4:456-471); `value` times one early window "
                    f"(ftran_cols {main_run['ftran_cols']} there)"}


def steepest_block(spx, torch, m, n, args, device):
    """Exact steepest-edge pricing (SPX_PRICING_STEEPEST, Goldfarb-Reid
    recurrence; README.md:16-17) on the same LP, one GPU: the per-pivot rate
    over whole windows after the same warm-up (event-timed copy for the
    pricing kernel with its third dot), and the whole solve from the slack
    basis against Dantzig's pivot count."""
    def ctx_():
        return spx.Context(m=m, n=n, seed=args.seed, device=device, pricing=spx.PRICING_STEEPEST)

    def window_run(timing):
        with spx.Context(m=m, n=n, seed=args.seed, device=device, pricing=spx.PRICING_STEEPEST,
                         timing=timing) as ctx:
            cfg = ctx.config()
            per = max(cfg["window"] - 1, 1)
            steps = span(args.steps, per)
            ctx.iterate(args.warmup)
            ds = ctx.dispatch_stats()
            if ds["window"] and ds["window_pos"] < ds["window"]:
                ctx.iterate(ds["window"] - ds["window_pos"])
            if timing:
                ctx.pass_times()
                ctx.loop_times()
            _, p0 = ctx.iterate(0)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            _, p1 = ctx.iterate(steps)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            pt = ctx.pass_times() if timing else None
            info = ctx.info()
        return cfg, dt, p1 - p0, pt, info

    cfg, dt, piv, _, info = window_run(False)
    _, dt_e, piv_e, pt, _ = window_run(True)
    passes = max(pt["passes"], 1)
    price_ms = pt["price_ms"] / passes
    with ctx_() as ctx:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        st, tot, calls = run_to_exit(ctx)
        torch.cuda.synchronize()
        sdt = time.perf_counter() - t0
        z = ctx.objective()
    return {"value": piv / dt if dt > 0 else 0.0, "unit": "iterations/s",
            "ms_per_step": 1e3 * dt / max(piv, 1), "steps": piv,
            "k_price_ms": price_ms, "k_price_bytes": info["bytes_price"],
            "k_price_GBps": info["bytes_price"] / (price_ms * 1e-3) / 1e9 if price_ms > 0 else 0.0,
            "k_update_ms": pt["update_ms"] / passes,
            "event_timed_ms_per_step": 1e3 * dt_e / max(piv_e, 1),
            "solve": {"status": ["MaxIter", "OptimumFound", "Unbounded", "ThetaOverflow"][int(st)],
                      "pivots": int(tot), "seconds": sdt, "z": z, "iterate_calls": calls,
                      "passes_after_optimum": calls_passes(calls) - int(tot)},
            "representation": f"eta window {cfg['window']}, two-kernel passes; k_price carries a third "
                              "dot on the A stream (B_w^T alpha beside y_w and the base row)"}


def sharded_pricing_block(make, reduce_max, reduce_sum, world, args):
    """The north-star pricing-scaling config (BASELINE.json configs[3], C4:
    m=4096, n=131072, columns sharded over the ranks, RCCL all-gather MINLOC):
    each rank's pricing kernel and pricing + MINLOC exchange event-timed over
    one whole window of pivots; aggregate pricing throughput = all ranks'
    algorithmic pricing bytes / the max over ranks of pricing + MINLOC.  Run
    at every N, so SCALE's lines give the 1 -> N pricing speedup directly."""
    m4, n4 = CONFIGS["C4"]
    ctx = make(True, 0, m4, n4)
    try:
        cfg = ctx.config()
        per = max(cfg["window"] - 1, 1)
        ctx.iterate(args.warmup)
        ds = ctx.dispatch_stats()
        if cfg["window"] and ds["window_pos"] < cfg["window"]:
            ctx.iterate(cfg["window"] - ds["window_pos"])
        ctx.pass_times()
        info0 = ctx.info()
        ctx.iterate(per)
        pt = ctx.pass_times()
        info1 = ctx.info()
    finally:
        ctx.close()
    passes = max(pt["passes"], 1)
    price_ms = pt["price_ms"] / passes
    pm_ms = pt["price_minloc_ms"] / passes
    bytes_rank = 0.5 * (info0["bytes_price"] + info1["bytes_price"])  # streamed columns (spx_info)
    price_max, pm_max = reduce_max([price_ms, pm_ms])
    bytes_all = reduce_sum([bytes_rank])[0]
    return {"config": f"C4 m={m4} n={n4}, pricing columns sharded over {world} rank(s)",
            "passes_timed": int(pt["passes"]), "bytes_all_ranks": bytes_all,
            "max_rank_price_ms": price_max, "max_rank_price_plus_minloc_ms": pm_max,
            "throughput_GBps": bytes_all / (pm_max * 1e-3) / 1e9 if pm_max > 0 else 0.0,
            "price_kernel_GBps_per_rank": bytes_rank / (price_ms * 1e-3) / 1e9 if price_ms > 0 else 0.0}


def explicit_block(timed_window, kernel_split, reduce_max, m, n):
    """The reference's representation on the same LP and clock: explicit B^-1
    rewritten in place by the rank-1 update every pivot (Sger, v4:331-333),
    fused with the next FTRAN (v4:306-308): 16 m^2 bytes per k_update."""
    run = timed_window(-1, False)
    ev = timed_window(-1, True)
    ks = kernel_split(ev, -1)
    upd_max = reduce_max([ks["update_ms"]])[0]
    value = run["pivots"] / run["dt"] if run["dt"] > 0 else 0.0
    b_alg = 8.0 * (m + 1) * (n - m) + 16.0 * m * m
    return {
        "value": value, "unit": "iterations/s", "ms_per_step": 1e3 * run["dt"] / max(run["pivots"], 1),
        "steps": run["pivots"], "dispatch": describe_dispatch(run["dispatch"]),
        "k_update": {"what": "rank-1 update B += E r^T in place (read + write) fused with FTRAN",
                     "avg_launch_ms": ks["update_ms"], "max_rank_avg_launch_ms": upd_max,
                     "algorithmic_bytes_per_launch": ks["update_bytes"],
                     "achieved_GBps": ks["update_bytes"] / (ks["update_ms"] * 1e-3) / 1e9 if ks["update_ms"] else 0.0,
                     "frac": ks["update_bytes"] / (ks["update_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS
                     if ks["update_ms"] else 0.0},
        "k_price": {"avg_launch_ms": ks["price_ms"], "algorithmic_bytes_per_launch": ks["price_bytes"],
                    "achieved_GBps": ks["price_bytes"] / (ks["price_ms"] * 1e-3) / 1e9 if ks["price_ms"] else 0.0},
        "iteration": {"algorithmic_bytes": b_alg, "achieved_GBps": b_alg * value / 1e9,
                      "frac": b_alg * value / 1e9 / HBM_PEAK_GBS},
    }


def tableau_block(spx, torch, m, n, args, device):
    """The same LP and pivot rule on the window tableau (SPX_FLAG_TABLEAU,
    DESIGN.md §4d): T_w = B_w A and dw = y_w A - c are kept in HBM and folded
    every 63 pivots by an fp64-MFMA rank-63 update, so a pivot reads neither
    A nor B_w; the passes run in the persistent loop kernel (k_tab_loop).  Not
    the north-star loop (no per-pivot A / B^-1 stream): reported beside it.
    Timed like the headline (W warmup pivots, then K rounded up to whole
    windows of KW - 1 pivots, so the timed run holds exactly K / (KW - 1) folds
    — at C5 the fold is most of a pivot's cost and a partial window would
    under-count it), plus an event-timed run for the loop / fold split and the
    fold kernel's roofline."""
    def run(timing):
        with spx.Context(m=m, n=n, seed=args.seed, device=device, timing=timing, tableau=True) as ctx:
            cfg = ctx.config()
            per = max(cfg["window"] - 1, 1)
            steps = span(args.steps, per)
            ctx.iterate(args.warmup)
            ds = ctx.dispatch_stats()
            if ds["window"] and ds["window_pos"] < ds["window"]:
                ctx.iterate(ds["window"] - ds["window_pos"])  # the timed run starts with a fold
            if timing:
                ctx.loop_times()
                ctx.pass_times()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            _, p0 = ctx.iterate(0)
            _, p1 = ctx.iterate(steps)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            lt = ctx.loop_times() if timing else None  # fold events (and the persistent loop's)
            pt = ctx.pass_times() if timing else None  # two-kernel passes
            info = ctx.info()
        return cfg, dt, p1 - p0, (lt, pt), info
    cfg, dt, piv, _, info = run(False)
    _, dt_e, piv_e, (lt, pt), _ = run(True)
    L = info["ld"]
    win = cfg["window"]
    # the tableau fold touches the active columns only (k_tab_active): the
    # non-basic ones and at most KW - 1 that entered during the window
    n_act = min(n, n - m + win - 1)
    fold_bytes = 16.0 * L * n_act + 16.0 * m * L        # T_w (active) and B_w read + written once per fold
    fold_flops = 2.0 * m * (n_act + L) * (win - 1)      # rank-(KW-1) updates of T_w and B_w
    folds = max(lt["folds"], 1)
    fold_ms = lt["fold_ms"] / folds if lt["folds"] else 0.0
    passes = max(lt["clock_passes"], 1)
    out = {
        "value": piv / dt if dt > 0 else 0.0,
        "unit": "iterations/s",
        "ms_per_step": 1e3 * dt / max(piv, 1),
        "steps": piv,
        "representation": f"window tableau {win}: T_w = B_w A, dw = y_w A - c in HBM, fp64-MFMA fold every "
                          f"{win - 1} pivots; persistent loop kernel k_tab_loop ({cfg['loop_grid']} workgroups)"
                          if cfg.get("persistent") else f"window tableau {win}, two-kernel passes",
        "persistent": cfg.get("persistent", 0),
        "loop": ({"us_per_pass": 1e3 * lt["loop_ms"] / max(lt["loop_passes"], 1),
                  "phase_us": {"pricing_to_barrier1": lt["price_us"] / passes,
                               "ftran_ratio_to_barrier2": lt["ftran_us"] / passes,
                               "leaving_row_bookkeeping": lt["tail_us"] / max(passes - 1, 1)}}
                 if cfg.get("persistent") else
                 {"kernels": "k_price WM 3 + k_tab_update",
                  "price_us": 1e3 * pt["price_ms"] / max(pt["passes"], 1),
                  "update_us": 1e3 * pt["update_ms"] / max(pt["passes"], 1)}),
        "fold": {"kernels": "k_tab_active + k_tab_fold + k_fold", "avg_ms": fold_ms,
                 "per_pivot_us": 1e3 * fold_ms / (win - 1), "active_columns": n_act,
                 "algorithmic_bytes": fold_bytes, "flops": fold_flops,
                 "achieved_GBps": fold_bytes / (fold_ms * 1e-3) / 1e9 if fold_ms > 0 else 0.0,
                 "frac_hbm": fold_bytes / (fold_ms * 1e-3) / 1e9 / HBM_PEAK_GBS if fold_ms > 0 else 0.0,
                 "achieved_TFLOPs": fold_flops / (fold_ms * 1e-3) / 1e12 if fold_ms > 0 else 0.0},
        "event_timed_ms_per_step": 1e3 * dt_e / max(piv_e, 1),
    }
    return out


def glpk_status():
    """The reference's CPU baseline is GLPK (solver_glpk.cpp).  Its counterpart
    ./solver_glpk binds libglpk at run time and exits 3 when it is absent; the
    oracle then stands in (kind "port") and this says why."""
    import subprocess

    exe = os.path.join(ROOT, "solver_glpk")
    if not os.path.exists(exe):
        return "solver_glpk not built"
    try:
        r = subprocess.run([exe, "--text", os.path.join(ROOT, "tests", "golden", "sample.txt")],
                           capture_output=True, text=True, timeout=60)
    except (OSError, subprocess.SubprocessError) as e:
        return f"solver_glpk failed: {e}"
    if r.returncode == 3:
        return "unavailable: libglpk not loadable on this host (solver_glpk exit 3)"
    return "available" if r.returncode == 0 else f"solver_glpk exit {r.returncode}"


def cpu_baseline(m, n, seed, budget_s):
    """The oracle (fp64 C restatement, OpenMP) on a bounded sample: K iterations
    from the slack basis of the same LP, K sized to ~budget_s of CPU time."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle

    threads = oracle.max_threads()
    A, b, c = oracle.generate(m, n, seed)
    t1, d1 = oracle.time_iterations(A, b, c, 2, threads)
    per = t1 / max(d1, 1)
    k = int(max(3, min(2000, budget_s / max(per, 1e-6))))
    sec, done = oracle.time_iterations(A, b, c, k, threads)
    return {"value": done / sec, "unit": "iterations/s", "cores": threads, "kind": "port",
            "sample": f"{done} iterations from the slack basis of the same m={m} n={n} LP "
                      f"(oracle/simplex_oracle.c, {threads} OpenMP threads, {sec:.1f} s)"}


if __name__ == "__main__":
    main()

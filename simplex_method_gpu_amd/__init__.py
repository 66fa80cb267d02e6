"""simplex_method_gpu_amd — MI355X-native dense revised-simplex hot loop.

Python mirror of the reference's host interface (Girjoaba/simplex_method_gpu,
``src/v4_cub_reduction.cu``):

* :func:`read_lp`   <- main()'s LP text reader (v4:395-419, load_matrix v4:94-104)
* :func:`solve`     <- ``solve(A, b, c, x_b, b_ixs, m, n, t)`` (v4:219-380)
* :class:`SolveStatus` <- ``enum class SolveStatus`` (v4:49-54)
* :class:`Context`  step-wise / benchmark access to the same device loop
  (``price`` = v4:288-302, ``pivot`` = v4:306-357).

Everything computes through ``libsimplex.so`` (hand-written gfx950 HIP
kernels behind the C-ABI in ``include/simplex.h``); there is no CPU path.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from enum import IntEnum

import numpy as np

from ._lib import SimplexError, SpxOpts, check, load

__all__ = ["SolveStatus", "SolveResult", "Context", "solve", "read_lp", "comm_unique_id",
           "shard_range", "minloc_merge", "group_iterate", "group_sync", "check_ranks",
           "SimplexError", "FLAG_TIMING", "RATIO_REFERENCE", "RATIO_GUARDED", "RATIO_HARRIS",
           "PRICING_DANTZIG", "PRICING_DEVEX", "PRICING_STEEPEST"]

FLAG_TIMING = 1
FLAG_STAMPS = 2
FLAG_GLOBAL_Y = 4
FLAG_ROW_SHARD = 8
FLAG_SPLIT_TAIL = 16
FLAG_NO_PERSIST = 32
FLAG_PERSIST = 64  # force the persistent loop kernel where it applies (default: auto)
FLAG_COMM1 = 128  # one rank through the RCCL path (tests)
MBOX_HANDLE_BYTES = 64  # SPX_MBOX_HANDLE_BYTES
FLAG_TABLEAU = 256  # window tableau: T_w = B_w A and dw kept beside the eta window
FLAG_COUNTED_TAIL = 512  # ratio-test hand-off by drained stores + last-arrival count (default: tagged poll)
FLAG_PRICE_TAIL = 1024  # k_price's last workgroup merges the entering candidates (default: deferred into k_update)

# leaving-row rules (include/simplex.h SPX_RATIO_*)
RATIO_REFERENCE, RATIO_GUARDED, RATIO_HARRIS = 0, 1, 2
# entering-column rules (include/simplex.h SPX_PRICING_*)
PRICING_DANTZIG, PRICING_DEVEX, PRICING_STEEPEST = 0, 1, 2


class SolveStatus(IntEnum):
    MaxIter = 0
    OptimumFound = 1
    Unbounded = 2
    ThetaOverflow = 3


@dataclass
class SolveResult:
    z: float
    status: SolveStatus
    x_b: np.ndarray
    b_ixs: np.ndarray
    pivots: int


def _ptr(a: np.ndarray | None):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def read_lp(path: str):
    """LP text format of the reference: ``m n``, A (m x n, row-major), b (m),
    c (n); anything after c is ignored (input/sample.txt).  Returns
    ``(m, n, A_cols, b, c)`` with ``A_cols`` shaped (n, m) — i.e. A stored
    column-major, the layout the reference keeps on the device (R2C, v4:59-60)."""
    with open(path) as f:
        toks = f.read().split()
    try:
        m, n = int(toks[0]), int(toks[1])
    except (IndexError, ValueError):
        raise ValueError("Either failed to read m and n, or m > n.")
    if m > n:
        raise ValueError("Either failed to read m and n, or m > n.")
    need = m * n + m + n
    if len(toks) - 2 < need:
        raise ValueError("truncated LP file")
    vals = np.array(toks[2:2 + need], dtype=np.float64)
    A_cols = np.ascontiguousarray(vals[: m * n].reshape(m, n).T)
    return m, n, A_cols, vals[m * n: m * n + m].copy(), vals[m * n + m:].copy()


def shard_range(m: int, n: int, rank: int, nranks: int):
    """(s_lo, s_hi, k_lo, k_hi): this rank's structural and slack column blocks."""
    out = (ctypes.c_int64 * 4)()
    check(load().spx_shard_range(m, n, rank, nranks, out))
    return tuple(out)


def minloc_merge(vals, idx):
    """Cross-rank MINLOC rule: smallest value, then smallest global index."""
    v = np.ascontiguousarray(vals, dtype=np.float64)
    i = np.ascontiguousarray(idx, dtype=np.int64)
    bv, bi = ctypes.c_double(), ctypes.c_int64()
    check(load().spx_minloc_merge(_ptr(v), _ptr(i), len(v), ctypes.byref(bv), ctypes.byref(bi)))
    return bv.value, bi.value


def group_iterate(ctxs, k: int):
    """Lockstep k iterations of an in-process shard group (see spx_group_iterate)."""
    arr = (ctypes.c_void_p * len(ctxs))(*[c._h.value for c in ctxs])
    st, piv = ctypes.c_int32(), ctypes.c_int64()
    check(load().spx_group_iterate(arr, len(ctxs), k, ctypes.byref(st), ctypes.byref(piv)))
    return SolveStatus(st.value), piv.value


def group_sync(ctxs):
    """Row-sharded groups: flush every member and exchange x_b rows (spx_group_sync)."""
    arr = (ctypes.c_void_p * len(ctxs))(*[c._h.value for c in ctxs])
    check(load().spx_group_sync(arr, len(ctxs)))


def check_ranks(infos, world: int, exchange: str = "rccl", distinct_gpus: bool = True):
    """Validate the all-gathered :meth:`Context.comm_info` of every rank of a
    job of ``world`` processes; raises ``RuntimeError`` naming the mismatch.
    RCCL exchange: every communicator reports ``world`` ranks and rank r is
    RCCL's rank r.  Always: rank r was created as rank r of ``world``; and,
    unless ``distinct_gpus`` is off (the one-GPU --share-gpu rehearsal), no two
    ranks share a PCI bus id (one process per GPU)."""
    if len(infos) != world:
        raise RuntimeError(f"{len(infos)} rank records for a world of {world}")
    for r, inf in enumerate(infos):
        if inf["nranks"] != world or inf["rank"] != r:
            raise RuntimeError(f"rank {r}: context created as rank {inf['rank']} of {inf['nranks']}")
        if exchange == "rccl" and (inf["rccl_nranks"] != world or inf["rccl_rank"] != r):
            raise RuntimeError(f"rank {r}: RCCL communicator reports rank {inf['rccl_rank']} of "
                               f"{inf['rccl_nranks']}, the job has {world}")
    buses = [inf["bus_id"] for inf in infos]
    if distinct_gpus and len(set(buses)) != len(buses):
        raise RuntimeError(f"ranks share a GPU: PCI bus ids {buses}")


def comm_unique_id() -> bytes:
    buf = (ctypes.c_uint8 * 128)()
    check(load().spx_comm_unique_id(buf))
    return bytes(buf)


class Context:
    """One device-resident LP (``spx_ctx``).  Either pass ``A_cols`` (n, m),
    ``b``, ``c`` or ``m, n, seed`` for the seeded generator of SURVEY.md §8(d)."""

    def __init__(self, A_cols=None, b=None, c=None, *, m: int | None = None, n: int | None = None,
                 seed: int | None = None, eps: float = 1e-7, device: int = -1, rank: int = 0,
                 nranks: int = 1, graph_batch: int = 0, timing: bool = False, price_block: int = 0,
                 update_rows: int = 0, price_grid: int = 0, update_block: int = 0, stamps: bool = False,
                 global_y: bool = False, row_shard: bool = False, split_tail: bool = False, window: int = 0,
                 ratio_test: int = 0, piv_tol: float = 1e-9, feas_tol: float = 1e-9, refactor_every: int = 0,
                 pricing: int = 0, persist: bool | None = None, loop_block: int = 0, comm1: bool = False,
                 tableau: bool = False, trace: int = 0, counted_tail: bool = False,
                 price_tail: bool = False):
        L = load()
        o = SpxOpts()
        L.spx_default_opts(ctypes.byref(o))
        o.eps, o.device, o.rank, o.nranks = eps, device, rank, nranks
        o.graph_batch, o.price_block, o.update_rows, o.price_grid = graph_batch, price_block, update_rows, price_grid
        o.update_block = update_block
        o.window = window  # 0 auto, -1 explicit rank-1 B^-1 update, 8/16/32/64 eta window
        o.ratio_test, o.piv_tol, o.feas_tol = ratio_test, piv_tol, feas_tol  # RATIO_*
        o.refactor_every = refactor_every
        o.pricing = pricing  # PRICING_DANTZIG / PRICING_DEVEX / PRICING_STEEPEST
        o.loop_block = loop_block
        o.trace_cap = trace  # record the first `trace` pivots' (p, q) on the device
        o.flags = ((FLAG_TIMING if timing else 0) | (FLAG_STAMPS if stamps else 0)
                   | (FLAG_GLOBAL_Y if global_y else 0) | (FLAG_ROW_SHARD if row_shard else 0)
                   | (FLAG_SPLIT_TAIL if split_tail else 0)
                   | ({None: 0, True: FLAG_PERSIST, False: FLAG_NO_PERSIST}[persist])
                   | (FLAG_COMM1 if comm1 else 0) | (FLAG_TABLEAU if tableau else 0)
                   | (FLAG_COUNTED_TAIL if counted_tail else 0) | (FLAG_PRICE_TAIL if price_tail else 0))
        h = ctypes.c_void_p()
        if A_cols is not None:
            A_cols = np.ascontiguousarray(A_cols, dtype=np.float64)
            n_, m_ = A_cols.shape
            b = np.ascontiguousarray(b, dtype=np.float64)
            c = np.ascontiguousarray(c, dtype=np.float64)
            if b.shape != (m_,) or c.shape != (n_,):
                raise ValueError("shape mismatch: A_cols (n, m), b (m,), c (n,)")
            check(L.spx_create(ctypes.byref(h), m_, n_, _ptr(A_cols), _ptr(b), _ptr(c), ctypes.byref(o)))
            self.m, self.n = m_, n_
        else:
            if m is None or n is None or seed is None:
                raise ValueError("give A_cols, b, c or m, n, seed")
            check(L.spx_create_generated(ctypes.byref(h), m, n, seed, ctypes.byref(o)))
            self.m, self.n = m, n
        self._h = h
        self._L = L

    # -- lifecycle
    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            self._L.spx_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def attach_comm(self, uid: bytes):
        buf = (ctypes.c_uint8 * 128).from_buffer_copy(uid)
        check(self._L.spx_attach_comm(self._h, buf))

    def comm_info(self):
        """What joined the exchange (spx_comm_info): the RCCL communicator's
        own rank count, rank and device (-1 without one), this context's HIP
        device ordinal and PCI bus id, and whether loop passes replay captured
        hipGraphs (``graph``) or fell back to eager after a refused capture."""
        out = (ctypes.c_int32 * 8)()
        bus = ctypes.create_string_buffer(64)
        check(self._L.spx_comm_info(self._h, out, bus))
        return {"rccl_nranks": out[0], "rccl_rank": out[1], "rccl_device": out[2], "device": out[3],
                "graph": bool(out[4]), "graph_fallback": bool(out[5]), "nranks": out[6], "rank": out[7],
                "bus_id": bus.value.decode(errors="replace")}

    def mbox_export(self) -> bytes:
        """This rank's mailbox handle (spx_mbox_export): gather every rank's
        in rank order and pass the list to :meth:`mbox_attach`."""
        buf = (ctypes.c_uint8 * MBOX_HANDLE_BYTES)()
        check(self._L.spx_mbox_export(self._h, buf))
        return bytes(buf)

    def mbox_attach(self, handles):
        """MINLOC through the peer mailboxes from now on (spx_mbox_attach)."""
        blob = b"".join(handles)
        if len(blob) != MBOX_HANDLE_BYTES * len(handles):
            raise ValueError("mailbox handles are %d bytes each" % MBOX_HANDLE_BYTES)
        buf = (ctypes.c_uint8 * len(blob)).from_buffer_copy(blob)
        check(self._L.spx_mbox_attach(self._h, buf))

    def prepare(self):
        """Build (capture, instantiate, upload) the batch hipGraph now
        (spx_prepare), e.g. right after attach_comm / mbox_attach, so no later
        iterate() pays for it inside a timed region."""
        check(self._L.spx_prepare(self._h))

    def reset(self):
        check(self._L.spx_reset(self._h))

    def reinvert(self):
        """Rebuild B^-1 (and x_b, y) from the current basis columns (spx_reinvert)."""
        check(self._L.spx_reinvert(self._h))

    def set_basis(self, basis):
        """Warm start from ``basis`` (m distinct column indices, basis order)."""
        bs = np.ascontiguousarray(basis, dtype=np.int64)
        if bs.shape != (self.m,):
            raise ValueError(f"basis must have {self.m} entries")
        check(self._L.spx_set_basis(self._h, _ptr(bs)))

    # -- loop
    def iterate(self, k: int):
        st, piv = ctypes.c_int32(), ctypes.c_int64()
        check(self._L.spx_iterate(self._h, k, ctypes.byref(st), ctypes.byref(piv)))
        self.last_pivots = piv.value  # (host-side: read by bench.py's watchdog without a device call)
        return SolveStatus(st.value), piv.value

    def solve(self, max_iter: int = (1 << 62)) -> SolveResult:
        z, st, piv = ctypes.c_double(), ctypes.c_int32(), ctypes.c_int64()
        x_b = np.zeros(self.m)
        b_ixs = np.zeros(self.m, dtype=np.int64)
        check(self._L.spx_solve(self._h, max_iter, ctypes.byref(z), _ptr(b_ixs), _ptr(x_b),
                                ctypes.byref(st), ctypes.byref(piv)))
        return SolveResult(z.value, SolveStatus(st.value), x_b, b_ixs, piv.value)

    def weights(self):
        """Devex / steepest-edge pricing weights of every column (spx_get_weights)."""
        w = np.empty(self.n, dtype=np.float64)
        check(self._L.spx_get_weights(self._h, _ptr(w)))
        return w

    def trace(self):
        """(entering columns, leaving rows) of the pivots recorded so far
        (needs ``trace=K`` at construction; spx_get_trace)."""
        cap = self.pivots_made()
        p = np.zeros(max(cap, 1), dtype=np.int64)
        q = np.zeros(max(cap, 1), dtype=np.int64)
        k = ctypes.c_int64()
        check(self._L.spx_get_trace(self._h, _ptr(p), _ptr(q), cap, ctypes.byref(k)))
        return p[:k.value], q[:k.value]

    def pivots_made(self) -> int:
        return self.iterate(0)[1]

    def price(self):
        p, e, opt = ctypes.c_int64(), ctypes.c_double(), ctypes.c_int32()
        check(self._L.spx_price(self._h, ctypes.byref(p), ctypes.byref(e), ctypes.byref(opt)))
        return p.value, e.value, bool(opt.value)

    def pivot(self):
        q, st = ctypes.c_int64(), ctypes.c_int32()
        check(self._L.spx_pivot(self._h, ctypes.byref(q), ctypes.byref(st)))
        return q.value, SolveStatus(st.value)

    # -- readback
    def state(self, binv: bool = False):
        m = self.m
        out = {"x_b": np.zeros(m), "b_ixs": np.zeros(m, dtype=np.int64), "y": np.zeros(m),
               "c_B": np.zeros(m), "binv": np.zeros((m, m)) if binv else None}
        st, piv = ctypes.c_int32(), ctypes.c_int64()
        check(self._L.spx_get_state(self._h, _ptr(out["x_b"]), _ptr(out["b_ixs"]), _ptr(out["y"]),
                                    _ptr(out["c_B"]), _ptr(out["binv"]), ctypes.byref(st), ctypes.byref(piv)))
        out["status"] = SolveStatus(st.value)
        out["pivots"] = piv.value
        return out

    def reduced_costs(self) -> np.ndarray:
        e = np.zeros(self.n)
        check(self._L.spx_reduced_costs(self._h, _ptr(e)))
        return e

    def objective(self) -> float:
        z = ctypes.c_double()
        check(self._L.spx_objective(self._h, ctypes.byref(z)))
        return z.value

    def kernel_times(self):
        tp, tu, np_, nu = ctypes.c_double(), ctypes.c_double(), ctypes.c_int64(), ctypes.c_int64()
        check(self._L.spx_kernel_times(self._h, ctypes.byref(tp), ctypes.byref(np_), ctypes.byref(tu),
                                       ctypes.byref(nu)))
        return {"price_ms": tp.value, "price_launches": np_.value,
                "update_ms": tu.value, "update_launches": nu.value}

    def wg_times(self):
        """Per-pass clocks of the last two compact window passes (stamps=True,
        spx_wg_times), 100 MHz ticks, indexed by pass parity (iteration & 1):
        a list of two dicts {"ftran": (grid, 4) entry / p known / A_p on the
        list in LDS / partial published, "price": (price grid, 4) start / end
        of the column loop / deferred tail reduced / staging in LDS, "tail": the tick the FTRAN tail had issued the
        bookkeeping, "mark": the start of the SPX_DIAG_MARK=1 probe kernel
        launched before the FTRAN pass (0 without it), "book": the tick k_price's
        workgroup 0 had issued the deferred tail's bookkeeping}."""
        cfg = self.config()
        g, gp = cfg["update_grid"], cfg["price_grid"]
        per = 4 * min(g, 4096) + 4 * min(gp, 4096) + 3
        out = np.zeros(2 * per, dtype=np.uint64)
        cnt = ctypes.c_int64()
        check(self._L.spx_wg_times(self._h, _ptr(out), out.size, ctypes.byref(cnt)))
        res = []
        for par in range(2):
            b = out[par * per: (par + 1) * per]
            nu, npr = 4 * min(g, 4096), 4 * min(gp, 4096)
            res.append({"ftran": b[:nu].reshape(-1, 4), "price": b[nu: nu + npr].reshape(-1, 4),
                        "tail": int(b[nu + npr]), "mark": int(b[nu + npr + 1]), "book": int(b[nu + npr + 2])})
        return res

    def fold_times(self):
        """The compact fold's per-workgroup clocks of its last launch (stamps=True,
        spx_fold_times): (workgroups, 8) ticks -- entry, coefficients staged,
        R in LDS, tiles done, vectors done, arrival counted, (unused), then
        the xw wave's end and the y wave's end (row-range-0 workgroups); zero
        for workgroups past the grid."""
        out = np.zeros(8 * 1024, dtype=np.uint64)
        cnt = ctypes.c_int64()
        check(self._L.spx_fold_times(self._h, _ptr(out), out.size, ctypes.byref(cnt)))
        return out.reshape(1024, 8)

    def phase_times(self):
        """In-kernel phase split (needs stamps=True), microseconds summed."""
        out = (ctypes.c_double * 18)()
        check(self._L.spx_phase_times(self._h, out))
        return {"price_body_us": out[0], "price_tail_us": out[1],
                "update_body_us": out[2], "update_tail_us": out[3],
                "tail_partials_us": out[4], "tail_sy_us": out[5], "tail_blocksum_us": out[6],
                "tail_bookkeeping_us": out[7], "update_prologue_us": out[9], "update_drain_us": out[10],
                "price_prologue_us": out[11], "price_drain_us": out[12],
                # k_update workgroup 0, since its start: status checked, entering
                # column reduced, row scalars issued, its wave 0 stream done,
                # its partial published
                "upd_wg0_us": [round(out[13 + k], 2) for k in range(5)]}

    def loop_times(self):
        """Persistent loop kernel (timing=True): launch ms + passes (hipEvents)
        and the in-kernel phase split (microseconds summed over passes)."""
        out, n = (ctypes.c_double * 7)(), ctypes.c_int64()
        check(self._L.spx_loop_times(self._h, out, ctypes.byref(n)))
        return {"loop_ms": out[0], "loop_passes": int(out[1]), "price_us": out[2], "ftran_us": out[3],
                "tail_us": out[4], "clock_passes": n.value, "fold_ms": out[5], "folds": int(out[6])}

    def pass_times(self):
        """Event-timed sums (timing=True): pricing kernel, pricing + MINLOC
        exchange, update kernel (ms), and the number of timed passes."""
        out, n = (ctypes.c_double * 3)(), ctypes.c_int64()
        check(self._L.spx_pass_times(self._h, out, ctypes.byref(n)))
        return {"price_ms": out[0], "price_minloc_ms": out[1], "update_ms": out[2], "passes": n.value}

    def info(self):
        m, n, ld, nb = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        bp, bu = ctypes.c_double(), ctypes.c_double()
        check(self._L.spx_info(self._h, ctypes.byref(m), ctypes.byref(n), ctypes.byref(ld), ctypes.byref(nb),
                               ctypes.byref(bp), ctypes.byref(bu)))
        return {"m": m.value, "n": n.value, "ld": ld.value, "local_nonbasic": nb.value,
                "bytes_price": bp.value, "bytes_update": bu.value}


    def ftran_cols(self) -> int:
        """Columns of B^-1 per row the FTRAN stream reads (spx_ftran_cols)."""
        v = ctypes.c_int32()
        check(self._L.spx_ftran_cols(self._h, ctypes.byref(v)))
        return v.value

    def dispatch_stats(self):
        """Monotone counts of what the loop enqueued (spx_dispatch_stats)."""
        out = (ctypes.c_int64 * 10)()
        check(self._L.spx_dispatch_stats(self._h, out))
        keys = ("eager_passes", "graph_launches", "graph_passes", "persistent_launches", "persistent_passes",
                "folds", "window_pos", "window", "persist_fallbacks", "graph_builds")
        return dict(zip(keys, list(out)))

    def config(self):
        """Resolved representation and launch geometry (spx_config)."""
        out = (ctypes.c_int32 * 16)()
        check(self._L.spx_config(self._h, out))
        keys = ("window", "price_block", "price_grid", "price_lds", "update_block", "update_rows", "update_grid",
                "graph_batch", "persistent", "loop_block", "tableau", "loop_grid", "defer_tail", "compact_fold",
                "ftran_rows_per_wave", "mbox_fused")
        return dict(zip(keys, list(out)))


def solve(A_cols, b, c, max_iter: int = (1 << 62), eps: float = 1e-7, device: int = -1) -> SolveResult:
    """Mirror of the reference's ``solve()`` (v4:219-380): A column-major as
    (n, m), returns z, status, x_b and b_ixs in basis order, pivots made."""
    with Context(A_cols, b, c, eps=eps, device=device) as ctx:
        return ctx.solve(max_iter)

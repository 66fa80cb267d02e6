// spx_kernels.hip — gfx950 kernels of the dense revised-simplex hot loop.
//
// One loop pass is two launches (SURVEY.md §7 design notes):
//   k_price   stages y in LDS (applying the last pivot's y update on the fly),
//             then e_j = y.A_j - c_j over this rank's non-basic columns fused
//             with the entering argmin (v4:288-302).  One wave per column, A
//             read with 16-byte non-temporal loads, wave shuffle + LDS argmin,
//             last-workgroup-done fan-in.
//   k_update  applies the pending rank-1 update B^-1 += E r^T (v4:331-333)
//             while streaming B^-1 once, and in the same pass computes FTRAN
//             alpha = B^-1_new A_p (v4:307-308), the last pivot's x_b update
//             (v4:347-348) for the rows it owns, compute_theta and the leaving
//             argmin (v4:199-208,324); the last workgroup then finds q, the
//             y-update scalar (v4:352-355) and does the basis bookkeeping
//             (v4:339-342).
// Host synchronisation per pass: none.  Termination (optimum / unbounded /
// iteration limit) is a device-side status word every kernel checks first.
// The deferred pivot state is described in spx_device.h.
//
// Cross-workgroup hand-offs inside a launch (partials, alpha) use agent-scope
// relaxed atomic stores/loads (global_* sc1: L1 bypass) drained with
// s_waitcnt vmcnt(0) before a workgroup barrier and one agent-scope ticket
// add per workgroup (MI355X_MICROARCH.md, Valid forms, first table row), on
// sharded counters (arrive_last, spx_common.h).
// Everything is deterministic: fixed reduction orders, no float atomics, so
// results are bit-identical for any grid / block size and any shard count.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <math.h>

#include <atomic>

#include "spx_device.h"
#include "spx_common.h"
#include "spx_fold.h"
#include "spx_kernels.h"
#include "spx_tableau.h"
#include "spx_tabdev.h"

namespace spx {

// B^-1 storage: 1 = one buffer updated in place (the pivot row the stream
// needs is staged into P.rbuf by k_price); 0 = ping-pong between B0 and B1.
#ifndef SPX_INPLACE
#define SPX_INPLACE 1
#endif
#ifndef SPX_LDS_BATCH
#define SPX_LDS_BATCH 4  // eta-window pricing: y / base-row LDS reads issued together
#endif
#ifndef SPX_PRICE_CH
#define SPX_PRICE_CH 8  // chunks of a column's start prefetched (8-wave workgroups)
#endif
#ifndef SPX_PRICE_DEEP
#define SPX_PRICE_DEEP 1  // deferred tail: the first column's first 16 chunks requested before the reduction
#endif
#ifndef SPX_SE_LDS_BATCH
// steepest edge (WM 4): its LDS operand batch (0 = SPX_LDS_BATCH); 2 frees
// the registers its two-batch deep prefetch needs (248 VGPRs, no spills)
#define SPX_SE_LDS_BATCH 2
#endif
#ifndef SPX_PRICE_DEEP1
#define SPX_PRICE_DEEP1 0  // (A/B, with SPX_PRICE_DEEP=0) WM 1 with the one-batch deep prefetch
#endif
#ifndef SPX_PRICE_DEEP_SE
// steepest edge (WM 4): the first column's first 8 (1) or 16 (2, the default
// since round 6: k_price 0.711 -> 0.721 of 8 TB/s, pass 87.9 -> 86.4 us,
// profiles/r06_steepest_ab.txt) chunks requested before the deferred-tail reduction
#define SPX_PRICE_DEEP_SE 2
#endif
#ifndef SPX_PRICE_DYN_PCT
#define SPX_PRICE_DYN_PCT 85  // the share of the columns handed out statically (grid stride)
#endif
#ifndef SPX_PRICE_PIPE
#define SPX_PRICE_PIPE 1  // eta-window pricing: two 8-chunk batches of a column in flight
#endif
#ifndef SPX_WIN_APLDS
#define SPX_WIN_APLDS 0  // eta-window FTRAN: A_p from LDS (1) or through L1/L2 (0)
#endif
#ifndef SPX_WIN_U1
#define SPX_WIN_U1 8  // eta-window FTRAN stream, 1 row per wave: dbl2 loads per lane per round trip
#endif
bool kernels_inplace() { return SPX_INPLACE != 0; }
// compact FTRAN (Params::bc): dbl2 chunks of each compact row requested at
// k_update entry (256 columns), and column-list entries per thread requested
// ahead of the entering column (1,024 columns at 512 threads)
#ifndef SPX_BC_PF
#define SPX_BC_PF 1  // C3 A/B (round-2 tools/r02_abbench.sh, in git history): 1 chunk 12.45k it/s, 2 chunks 12.31-12.34k
#endif
#ifndef SPX_FTRAN_TRIM
// k_ftran_bc's entry loads: 2 = the U row only up to the window's pending
// pivots, requested after the state arrives (the default since round 6: PMC
// read per launch 5.27 -> 3.70 MB, C3 pass 74.76 -> 74.75 us, tools/ftran_ab.sh,
// profiles/r06_ftran_ab.txt); 1 = the compact row's chunks only up to S as
// well (lanes past it re-read the row's first line): 2.91 MB but 75.16 us
#define SPX_FTRAN_TRIM 2
#endif
#ifndef SPX_BC_PF2
#define SPX_BC_PF2 4
#endif
constexpr int BC_PF = SPX_BC_PF;
constexpr int BC_PF2 = SPX_BC_PF2;  // chunks requested once S is known (up to 512 columns)
constexpr int BC_APC = 8192;  // A_p gathered onto the list in LDS blocks of this many columns
constexpr int BC_RL = 2;

// Diagnostic phase stamps: slot[0] = earliest workgroup start of the current
// launch, slot[1] += (last-workgroup ticket - start), slot[2] += tail duration.
__device__ __forceinline__ void stamp_start(unsigned long long* slot) {
    if (slot && threadIdx.x == 0) atomicMin(&slot[0], rtime());
}
// Stream window per launch: slot[S+0] = earliest wave stream start, slot[S+1]
// = latest wave stream end; the tail adds prologue (earliest stream start -
// earliest workgroup start) to slot[S+2] and drain (last ticket - latest
// stream end) to slot[S+3].
__device__ __forceinline__ void stamp_stream(unsigned long long* s, bool begin) {
    if (s && threadIdx.x == 0) {  // one atomic per workgroup (wave 0 as its proxy)
        if (begin) atomicMin(&s[0], rtime());
        else atomicMax(&s[1], rtime());
    }
}
__device__ __forceinline__ void stamp_tail(unsigned long long* slot, unsigned long long t_tail,
                                           unsigned long long* win) {
    if (slot && threadIdx.x == 0) {
        const unsigned long long t_end = rtime();
        const unsigned long long t0 = __hip_atomic_load(&slot[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        atomicAdd(&slot[1], t_tail - t0);
        atomicAdd(&slot[2], t_end - t_tail);
        __hip_atomic_store(&slot[0], ~0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long b = __hip_atomic_load(&win[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long e = __hip_atomic_load(&win[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        atomicAdd(&win[2], b - t0);
        atomicAdd(&win[3], t_tail > e ? t_tail - e : 0ull);  // (tagged hand-off: the tail may start first)
        __hip_atomic_store(&win[0], ~0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&win[1], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}
// Workgroup 0 timeline of k_update (diagnostic): slot 24 + k accumulates
// the ticks from its start to mark k (thread 0 only).
__device__ __forceinline__ void wg0_mark(const Params& P, int k, unsigned long long t0) {
    if (P.stamps && blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&P.stamps[24 + k], rtime() - t0);
}
// Sub-phase marks inside the update tail: slot 8+k accumulates the ticks since
// the previous mark (thread 0 only).
__device__ __forceinline__ unsigned long long tail_mark(const Params& P, int k, unsigned long long prev) {
    if (!P.stamps || threadIdx.x != 0) return prev;
    const unsigned long long now = rtime();
    atomicAdd(&P.stamps[8 + k], now - prev);
    return now;
}

// ---------------------------------------------------------------------------
// Pieces of the deferred pivot (one definition, so every consumer — k_price,
// k_update, k_flush, k_materialize — produces the same bits)
// ---------------------------------------------------------------------------
// The workgroup's best wave partial, chosen on (val, idx) scalars and read
// back from LDS by index: selecting whole PricePartial structs in a loop put
// the running winner in scratch, and a kernel with a private segment paid
// about 4 us more at its kernel boundary
template <int WAVES>
__device__ __forceinline__ int best_wave(const PricePartial* red) {
    double bv = red[0].val;
    int64_t bi = red[0].idx;
    int bk = 0;
#pragma unroll
    for (int i = 1; i < WAVES; ++i) {
        const double v = red[i].val;
        const int64_t x = red[i].idx;
        if (argmin_better(v, x, bv, bi)) {
            bv = v;
            bi = x;
            bk = i;
        }
    }
    return bk;
}

// ---------------------------------------------------------------------------
// Pricing + entering argmin
// ---------------------------------------------------------------------------
// WM: 0 = explicit B^-1 (y updated in the LDS fill); 1 = eta window with the
// pending base row in LDS next to y; 2 = eta window, base row read from global
// (L2) when y and the row do not both fit; 3 = window tableau (P.tab): no A
// stream, each column reads T_w[q_tau, j], dw[j] and its Wt row; 4 / 5 = 1 / 2
// with steepest-edge pricing (P.steep): a third dot v.A_j per column, v =
// B_w^T alpha (P.se_v) in LDS beside y and the base row (4) or from global (5).
// Peer mailboxes (k_exchange below; the fused exchange in k_price's pricing
// tail and k_ftran_bc's entry).  A rank that polls for MBOX_TIMEOUT_TICKS
// without seeing a peer's word stops with ST_HANDOFF_TIMEOUT.
constexpr unsigned long long MBOX_TIMEOUT_TICKS = 3000000000ull;  // 30 s of s_memrealtime (100 MHz)
constexpr int MBOX_FUSED_MAX_G = 64;  // ranks the fused receiver merges (k_ftran_bc LDS)
// Fused exchange (Params::mbox_fused): a loop pass's record carries the tag
// (epoch << 24) | (iteration + 1) in every word; the epoch (DevState,
// advanced by every reset on every rank) keeps a record of an earlier solve
// from matching after the iteration count restarts.  k_exchange's seq tags
// stay below 2^24, so the two never match each other's words.
__device__ __forceinline__ uint32_t mbox_tag(uint32_t epoch, int64_t it) {
    return (epoch << 24) | ((uint32_t)(it + 1) & 0xFFFFFFu);
}
// word h of rank g's record in this rank's mailbox, polled until it carries tag
__device__ __forceinline__ bool mbox_poll(const Params& P, int64_t par, int g, int h, uint32_t tag,
                                          uint32_t* half) {
    const int64_t nh = (int64_t)P.pr_stride * 4;
    const uint64_t* q = &P.mbox[(par * P.nin + g) * nh + h];
    const unsigned long long t0 = rtime();
    for (;;) {
        const uint64_t w = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if ((uint32_t)(w >> 32) == tag) {
            *half = (uint32_t)w;
            return true;
        }
        if (rtime() - t0 > MBOX_TIMEOUT_TICKS) {
            *half = 0u;
            return false;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

template <int BLOCK, bool PLAIN = false>
__device__ UpdPartial reduce_update_partials(const Params& P, UpdPartial* red, int nparts, uint32_t tag = 0,
                                             bool* timed_out = nullptr);
template <int BLOCK, bool PLAIN>
__device__ __forceinline__ UpdPartial reduce_partial_block(const UpdPartial& w, UpdPartial* red);
template <int BLOCK>
__device__ __forceinline__ UpdPartial reduce_partial_pair(const UpdPartial& wa, const UpdPartial& wb,
                                                          UpdPartial* red);
template <bool PLAIN = false>
__device__ __forceinline__ UpdPartial upd_fetch(const Params& P, int g);
__device__ __forceinline__ UpdPartial wave_reduce_partial(const UpdPartial& w);
// the deferred ratio-test tail's bookkeeping (TailRec; defined with the tail)
__device__ __forceinline__ void apply_deferred_tail(const Params& P, DevState* st, const TailRec& R,
                                                    const UpdPartial& t);
// TK: the ticketed tail compiled in for WM 1 (a separate instantiation, so the
// static C3 pass keeps its code: carrying the disabled ticket branches cost
// it 0.5 us per pass); WM 2 always carries it
template <int BLOCK, bool LDS_Y, int WM, bool TK = false>
__global__ __launch_bounds__(BLOCK) void k_price(Params P) {
    DevState* st = P.st;
    constexpr int WAVES = BLOCK / 64;
    constexpr bool WIN = WM != 0;
    constexpr bool LDS_R = WM == 1 || WM == 4;
    constexpr bool SE = WM == 4 || WM == 5;
    constexpr bool LDS_V = WM == 4;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int idx0 = blockIdx.x * WAVES + wave;
    // speculative: this wave's first non-basic column, loaded together with the
    // status word (index clamped into the list; validated against nb_count)
    int64_t j0 = P.nb_list[idx0 < P.n ? idx0 : P.n - 1];
    const unsigned long long t_pw0 = P.stamps ? rtime() : 0ull;
    // Deferred tail: the record and this thread's partial(s) are requested at
    // entry beside the column and the state -- unconditionally (clamped
    // slot), so no test of the record or the state sits between them: a
    // branch there made the compiler wait for the state, then for the
    // record, before the partials were even requested (three round trips)
    // (a record of zeros when there is none: a branch around these loads
    // moved the record's uniform fields into SGPRs inside it, i.e. waited)
    // Only the compact window passes defer the tail (the explicit form and the
    // tableau never do: no record, no partials, no loads)
    constexpr bool PAIR = BLOCK == 256;  // (two partials of the 512-thread shape per thread)
    constexpr bool DT = WM != 0 && WM != 3;
    TailRec R{};
    if constexpr (DT) R = *(P.defer_tail ? P.trec : reinterpret_cast<const TailRec*>(P.zeros));
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    constexpr int SW = (int)(sizeof(DevState) / 16);
    u32x4 sw[SW];  // the state as raw words (st_snapshot's loads)
#pragma unroll
    for (int i = 0; i < SW; ++i) sw[i] = reinterpret_cast<const u32x4*>(st)[i];
    UpdPartial w0 = upd_empty(), w1 = upd_empty();
    if constexpr (DT) {
        const int tp = P.tail_parts > 0 ? P.tail_parts : 1;
        w0 = upd_fetch<true>(P, tid < tp ? tid : tp - 1);
        if constexpr (PAIR) w1 = upd_fetch<true>(P, tid + BLOCK < tp ? tid + BLOCK : tp - 1);
    }
    __builtin_amdgcn_sched_barrier(0);
    // (every state word held until here: a dead word's register, reused
    // early, made the partials' loads wait for the state)
#pragma unroll
    for (int i = 0; i < SW; ++i) asm volatile("" ::"v"(sw[i]));
    const DevState S = __builtin_bit_cast(DevState, sw);
    // the fields the pass prices with (fresh: derived from the deferred tail;
    // kept as scalars -- assigning into the snapshot put it in scratch)
    int64_t s_iter = S.iter, s_q = S.q, s_leave = S.leave;
    double s_aq = S.aq, s_sy = S.s_y, s_wp = S.wp;
    int32_t s_nb = S.nb_count, s_nw = S.nw;
    // Deferred ratio-test tail (TailRec, P.defer_tail): the previous FTRAN
    // pass left its workgroup partials and this record.  Every workgroup
    // reduces the partials itself (the same reduction as the FTRAN tail, so
    // the same bits) and prices with the state the bookkeeping produces;
    // workgroup 0 applies that bookkeeping meanwhile.  No workgroup reads a
    // state word workgroup 0 writes: the list is read through the two slots
    // the pivot changes (nbl), SY[tau] is the derived s_y.
    bool fresh = false;
    int32_t pk_a = -1, pk_b = -1;
    int64_t pv_a = 0, pv_b = 0;
    constexpr int CH = (BLOCK <= 512 && WM != 3) ? SPX_PRICE_CH : 8;
    constexpr int LB = (WM == 4 && SPX_SE_LDS_BATCH > 0) ? SPX_SE_LDS_BATCH : SPX_LDS_BATCH;  // LDS operand batch
    // SPX_PRICE_DEEP (deferred tail): the first column's first 2 CH chunks are
    // requested as soon as the tail's record says which column this slot
    // holds after the pivot's list edit -- before the partials are reduced
    // and the base row staged -- so HBM streams during the prologue instead
    // of idling (only the end-of-list slot depends on q; it is left out)
    // Only with y_w and the base row both staged in LDS (WM 1, the C3 / C4
    // shape): with the base row read from L2 (WM 2, C5) it measured 4.6 %
    // slower per pass (1,071 against 1,022 us, tools/pass_ab.py).
    // (only run_pipe consumes vd0 / vd1, so DEEP needs the pipelined loop)
    // (steepest edge, WM 4: both batches with its LDS operand batch at 2,
    // SPX_SE_LDS_BATCH; at the default batch the second one spilled)
    constexpr bool DEEP2 = SPX_PRICE_DEEP && SPX_PRICE_PIPE && BLOCK <= 512 && CH == 8 &&
                           (WM == 1 || (SPX_PRICE_DEEP_SE == 2 && WM == 4));
    constexpr bool DEEP = DEEP2 || (SPX_PRICE_DEEP_SE && SPX_PRICE_PIPE && WM == 4 && BLOCK <= 512 && CH == 8) ||
                          (SPX_PRICE_DEEP1 && SPX_PRICE_PIPE && WM == 1 && BLOCK <= 512 && CH == 8);
    dbl2 vd0[DEEP ? CH : 1], vd1[DEEP2 ? CH : 1];
    int64_t jdeep = -1;  // the column the deep prefetch holds (-1: none)
    // the bookkeeping's inputs for workgroup 0's thread 0, which applies them
    // after its columns (issued first, its stores would hold up the waits for
    // its own staging loads: vmcnt retires in order)
    __shared__ TailRec s_rec;
    __shared__ UpdPartial s_tp;
    if (DT && P.defer_tail) {
        fresh = R.fresh != 0;
        if constexpr (DEEP) {
            // slots below cnt0 hold the same column before and after the
            // list edit, except p's slot R.kp, which takes the last entry.
            // The loads are unconditional buffer loads: behind a branch, the
            // compiler's waits for the partials below covered these loads too
            // (the wait counts of the two paths merge).  Their range is the
            // prefetched chunks when the record is fresh and the slot prices
            // a column, else 0 bytes: out-of-range lanes read 0 and send no
            // request, so a pass after the optimum (the rest of an iterate()
            // call; it prices nothing) no longer streams 16-32 KB per wave
            const int64_t L2d = P.L >> 1;
            const int32_t cnt0 = R.kp >= 0 ? R.cnt - 1 : R.cnt;
            const bool dv = fresh && idx0 < cnt0 && (L2d & 511) == 0 && L2d >= 2 * CH * 64;
            int64_t jd = (R.kp >= 0 && idx0 == R.kp) ? (int64_t)R.last : j0;
            jd = (uint64_t)jd < (uint64_t)P.n ? jd : 0;
            constexpr int NB = (DEEP2 ? 2 : 1) * CH * 64 * (int)sizeof(dbl2);
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                const_cast<double*>(P.A + jd * P.L), 0, dv ? NB : 0, SPX_BUF_DW3);
#pragma unroll
            for (int u = 0; u < CH; ++u)
                vd0[u] = ldbuf2<SPX_NT_A>(rs, (lane + u * 64) * (int)sizeof(dbl2));
            if constexpr (DEEP2) {
#pragma unroll
                for (int u = 0; u < CH; ++u)
                    vd1[u] = ldbuf2<SPX_NT_A>(rs, (CH * 64 + lane + u * 64) * (int)sizeof(dbl2));
            }
            jdeep = dv ? jd : -1;
        }
        // slots past the FTRAN pass's partials: empty (after the deep loads'
        // issue: the selects wait for the partials)
        if (tid >= P.tail_parts) w0 = upd_empty();
        if constexpr (PAIR) {
            if (tid + BLOCK >= P.tail_parts) w1 = upd_empty();
        }
        if (fresh) {
            __shared__ UpdPartial s_ured[(PAIR ? 2 * WAVES : WAVES) + 1];
            UpdPartial t;
            if constexpr (PAIR) {
                for (int g = tid + 2 * BLOCK; g < P.tail_parts; g += 2 * BLOCK) {
                    upd_merge(w0, upd_fetch<true>(P, g));
                    if (g + BLOCK < P.tail_parts) upd_merge(w1, upd_fetch<true>(P, g + BLOCK));
                }
                t = reduce_partial_pair<BLOCK>(w0, w1, s_ured);
            } else {
                for (int g = tid + BLOCK; g < P.tail_parts; g += BLOCK) upd_merge(w0, upd_fetch<true>(P, g));
                t = reduce_partial_block<BLOCK, true>(w0, s_ured);
            }
            const int64_t q = t.idx;
            const bool unb = t.nonpos == P.m || q < 0 || q >= P.m;
            if (blockIdx.x == 0 && tid == 0) {
                if (unb) apply_deferred_tail(P, st, R, t);
                s_rec.it = R.it;  // (field by field: a struct copy went through scratch)
                s_rec.p = R.p;
                s_rec.e_rep = R.e_rep;
                s_rec.c_p = R.c_p;
                s_rec.wp = R.wp;
                s_rec.cnt = R.cnt;
                s_rec.kp = R.kp;
                s_rec.last = R.last;
                s_rec.nw = R.nw;
                s_tp.idx = t.idx;
                s_tp.nonpos = t.nonpos;
                s_tp.T = t.T;
                s_tp.a_w = t.a_w;
                s_tp.cb_w = t.cb_w;
                s_tp.bix_w = t.bix_w;
            }
            if (unb) return;  // Unbounded (v4:319-322; workgroup 0 has recorded it)
            s_iter = R.it + 1;
            s_q = q;
            s_aq = t.a_w;
            s_sy = y_scalar(t.T, t.a_w, t.cb_w, R.c_p);
            s_nw = R.nw + 1;
            if (P.devex) {
                s_leave = t.bix_w;
                s_wp = R.wp;
            }
            // pivot_bookkeeping's list edit: p's slot takes the last entry,
            // the leaving column joins at the end
            int32_t c1 = R.cnt;
            if (R.kp >= 0) {
                --c1;
                if (R.kp != c1) {
                    pk_b = R.kp;
                    pv_b = R.last;
                }
            }
            if (owns_col(P, t.bix_w)) {
                pk_a = c1;
                pv_a = t.bix_w;
                ++c1;
            }
            s_nb = c1;
            if (idx0 == pk_a) j0 = pv_a;
            else if (idx0 == pk_b) j0 = pv_b;
        }
    }
    const unsigned long long t_pw1 = P.stamps ? rtime() : 0ull;  // the deferred tail is reduced
    auto nbl = [&](int idx) -> int64_t {
        return idx == pk_a ? pv_a : (idx == pk_b ? pv_b : (int64_t)P.nb_list[idx]);
    };
    if (S.status != ST_RUNNING || s_iter >= S.limit) {
        if (fresh && blockIdx.x == 0 && tid == 0) apply_deferred_tail(P, st, s_rec, s_tp);
        return;
    }
    unsigned long long* const slot = P.stamps;
    if (!P.defer_price) stamp_start(slot);  // (deferred passes: per-workgroup clocks only, below)
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int64_t L = P.L;
    const int64_t L2 = L >> 1;
    double* ys = reinterpret_cast<double*>(smem);
    double* rs = reinterpret_cast<double*>(smem + (LDS_Y ? L * 8 : 0));
    double* vs = reinterpret_cast<double*>(smem + (LDS_Y ? L * 8 : 0) + (LDS_R ? L * 8 : 0));
    PricePartial* red = reinterpret_cast<PricePartial*>(smem + (LDS_Y ? L * 8 : 0) + (LDS_R ? L * 8 : 0) +
                                                        (LDS_V ? L * 8 : 0));
    int* s_last = reinterpret_cast<int*>(red + WAVES);
    const int nb = s_nb;

    const int64_t it = s_iter;
    const bool wg0 = blockIdx.x == 0;
    constexpr int YB = 4;
    const dbl2* yin = reinterpret_cast<const dbl2*>(S.y_buf ? P.y1 : P.y0);
    // explicit B^-1: current y = ybuf + s_y r while the last pivot's y update is
    // pending (workgroup 0 also persists that y and, in place, stages r for
    // k_update).  Eta window: y_w is fixed between folds; the pending pivot's
    // base row B_w[q,:] is staged next to it (workgroup 0 also keeps it, and
    // U[q][s<tau], in Qrows/Urows for k_fold).  Loads are batched YB deep per
    // thread so the fill is one memory round trip, not one per element.
    const int KW = P.win;
    const int nw = WIN ? s_nw : 0;
    if (WIN && nw >= KW) {  // the host folds before this can happen
        if (wg0 && tid == 0) {
            if (fresh) apply_deferred_tail(P, st, s_rec, s_tp);
            st->status = ST_WINDOW_FULL;
        }
        return;
    }
    const bool pend = WIN ? nw > 0 : it > 0;
    const int tau = nw - 1;  // pending pivot of the window
    const int64_t qq = pend ? s_q : 0;
    const bool upd_y = !WIN && S.y_applied < it;
    const double s_y = s_sy;
    dbl2* yout = reinterpret_cast<dbl2*>(S.y_buf ? P.y0 : P.y1);
    // the pending pivot row: row q of the stored B^-1 (replicated storage), or
    // rbuf, staged by k_finalize_rs from the all-gather (row-sharded storage)
    const dbl2* rr = reinterpret_cast<const dbl2*>(
        !pend ? P.zeros
              : (P.row_shard ? P.rbuf : ((SPX_INPLACE || WIN || !(it & 1)) ? P.B0 : P.B1) + qq * L));
    const bool stage_r = WIN ? (pend && wg0) : (SPX_INPLACE && pend && wg0 && !P.row_shard);
    const bool stage = LDS_Y || LDS_R || wg0;
    const dbl2* vin = reinterpret_cast<const dbl2*>(P.se_v);  // steepest edge: B_w^T alpha
    const bool load_y = LDS_Y || (!WIN && wg0);
    const bool need_r = WIN ? (pend && (LDS_R || stage_r)) : (upd_y || stage_r);

    // Issue order (vmcnt retires in issue order): the first batch of y /
    // base-row loads, then the first CH chunks of this wave's first column,
    // which stay in flight across the LDS fill and the barrier.  Every load
    // here is unconditional with a clamped index (rr is always a valid row),
    // so the fill waits for its own loads only, not for the A prefetch.
    static_assert(CH >= 1 && CH <= 8, "the pipelined column loop consumes at most one 8-chunk batch of prefetch");
    const bool deep_hit = DEEP && jdeep >= 0 && jdeep == j0;  // (else the first column goes the usual way)
    const bool pre = WM != 3 && idx0 < nb && L2 >= CH * 64;
    dbl2 yv[YB], rv[YB], vv[YB];
    double uqrow = 0.0;  // U[q][tid] for Urows (window, workgroup 0)
    if (stage) {
#pragma unroll
        for (int u = 0; u < YB; ++u) {
            const int64_t k = (int64_t)u * BLOCK + tid;
            const int64_t kc = k < L2 ? k : L2 - 1;
            if (load_y) yv[u] = yin[kc];
            rv[u] = rr[kc];
            if constexpr (LDS_V) vv[u] = vin[kc];
        }
        if constexpr (WIN) uqrow = P.U[qq * KW + (tid < KW ? tid : KW - 1)];
    }
    __builtin_amdgcn_sched_barrier(0);  // (the scheduler would hoist the A loads)
    dbl2 v0[CH];
    if constexpr (WM != 3) {
        if (!deep_hit) {
            const dbl2* c0 = reinterpret_cast<const dbl2*>(P.A + j0 * L);
#pragma unroll
            for (int u = 0; u < CH; ++u) {
                const int64_t k = lane + u * 64;
                v0[u] = ld2<SPX_NT_A>(&c0[k < L2 ? k : L2 - 1]);
            }
        }
    }
    if (stage) {
        // the staging values are taken here, behind the A prefetch's issue
        // (otherwise the loads sink into the conditional stores below and
        // their waits cover the prefetch too)
#pragma unroll
        for (int u = 0; u < YB; ++u) {
            if (load_y) asm volatile("" ::"v"(yv[u].x), "v"(yv[u].y));
            asm volatile("" ::"v"(rv[u].x), "v"(rv[u].y));
            if constexpr (LDS_V) asm volatile("" ::"v"(vv[u].x), "v"(vv[u].y));
        }
        if constexpr (WIN) asm volatile("" ::"v"(uqrow));
        dbl2* yl = reinterpret_cast<dbl2*>(ys);
        dbl2* rl = reinterpret_cast<dbl2*>(rs);
        dbl2* vl = reinterpret_cast<dbl2*>(vs);
        dbl2* rb = reinterpret_cast<dbl2*>(WIN ? P.Qrows + (int64_t)tau * L : P.rbuf);
        for (int64_t k0 = 0; k0 < L2; k0 += (int64_t)YB * BLOCK) {
            if (k0 > 0) {  // later batches (L2 > YB * BLOCK)
#pragma unroll
                for (int u = 0; u < YB; ++u) {
                    const int64_t k = k0 + (int64_t)u * BLOCK + tid;
                    const int64_t kc = k < L2 ? k : L2 - 1;
                    if (load_y) yv[u] = yin[kc];
                    if (need_r) rv[u] = rr[kc];
                    if constexpr (LDS_V) vv[u] = vin[kc];
                }
            }
#pragma unroll
            for (int u = 0; u < YB; ++u) {
                const int64_t k = k0 + (int64_t)u * BLOCK + tid;
                if (k < L2) {
                    if constexpr (!WIN) {
                        const dbl2 v = upd_y ? y_apply(s_y, rv[u], yv[u]) : yv[u];
                        if constexpr (LDS_Y) yl[k] = v;
                        if (upd_y && wg0) yout[k] = v;  // flipped in by k_update's tail
                    } else {
                        if constexpr (LDS_Y) yl[k] = yv[u];
                        if constexpr (LDS_R) {
                            if (pend) rl[k] = rv[u];
                        }
                        if constexpr (LDS_V) {
                            if (pend) vl[k] = vv[u];
                        }
                    }
                    if (stage_r) rb[k] = rv[u];
                }
            }
        }
        if (WIN && stage_r && tid < tau) P.Urows[(int64_t)tau * KW + tid] = uqrow;
    }
    // LDS only: the A prefetch stays in flight across the barrier (the staged
    // Qrows / rbuf stores are read after the kernel boundary)
    if constexpr (LDS_Y || LDS_R) lds_barrier();
    auto Y = [&](int64_t k) -> dbl2 {
        if constexpr (LDS_Y) return reinterpret_cast<const dbl2*>(ys)[k];
        else if constexpr (WIN) return yin[k];
        else return upd_y ? y_apply(s_y, rr[k], yin[k]) : yin[k];
    };
    auto Rw = [&](int64_t k) -> dbl2 {
        if constexpr (LDS_R) return reinterpret_cast<const dbl2*>(rs)[k];
        else return rr[k];
    };
    auto Vw = [&](int64_t k) -> dbl2 {
        if constexpr (LDS_V) return reinterpret_cast<const dbl2*>(vs)[k];
        else return vin[k];
    };
    // window coefficients of this lane (lane s < tau: pivot s of the window)
    double uq = 0.0, syl = 0.0, syp = 0.0;
    double csl = 0.0, se_gp = 0.0;  // steepest edge: U[:, s] . alpha (lane s), gamma_p
    if constexpr (WIN) {
        if (pend) {
            if (lane < tau) {
                uq = P.U[qq * KW + lane];
                syl = P.SY[lane];
                if constexpr (SE) csl = P.se_cg[lane];
            }
            syp = fresh ? s_sy : P.SY[tau];  // (fresh: workgroup 0 is writing SY[tau])
            if constexpr (SE) se_gp = P.se_cg[KW];
        }
    }
    double best = INFINITY, bw = 0.0, be = 0.0;
    int64_t bj = INT64_MAX;
    const int64_t dvx_leave = s_leave;
    const double dvx_wp = s_wp, dvx_aq = s_aq;
    unsigned long long* const win = (slot && !P.defer_price) ? P.stamps + 20 : nullptr;
    stamp_stream(win, true);
    const unsigned long long t_pw2 = P.stamps ? rtime() : 0ull;  // the staging is in LDS
    const int nlist = nb;
    const int stride = gridDim.x * WAVES;
    // Dynamic tail (P.price_dyn: WM 2, C5, and WM 1 where a wave prices many
    // columns, C4): the first SPX_PRICE_DYN_PCT % of the list in grid-stride
    // rounds as before, the rest one column per ticket.  P.tk_shards
    // counters (a 128-byte line each, per pass parity): counter k hands out
    // the slots s_lim + k + SHARDS t, and a wave draws from counter
    // (wave + workgroup) mod SHARDS: workgroups b .. b + 7 all reach counter
    // b + 7, so every counter serves waves of all eight XCDs (blockIdx % 8),
    // and every counter has waves when WAVES + grid - 1 >= SHARDS (the host
    // caps the count so; a counter nobody draws from would leave its slots
    // unpriced, which the pass after this one checks on the device: every
    // counter's last value must reach the slots it hands out, else
    // DevState::uncovered is set and the host fails the call).  No address
    // takes more than 1/SHARDS of the
    // fetch-adds (one address: same-address atomics run one after another in
    // their L2 channel, ~8 ns each).  A wave takes each ticket one column
    // ahead -- the first as it starts its last static column, the next as it
    // starts a ticketed one -- so the round trip overlaps a column's stream.
    // Every column's terms and the argmin's total order are unchanged, so the
    // same bits.  Workgroup 0 writes how many tickets of each counter this
    // pass needs (word 1 of its line); at its end it checks the previous
    // pass's counters (the other parity) against theirs and zeroes them for
    // the next pass.
    constexpr bool DYN = WM == 2 || (TK && WM == 1);
    const int TKS = P.tk_shards;  // (1..16, the host's choice per pricing mode)
    int s_lim = nlist;
    uint32_t* tkc = nullptr;
    const int tk_k = (int)((wave + blockIdx.x) % TKS);
    if (DYN && P.price_dyn) {
        s_lim = stride * (int)(((int64_t)nlist * SPX_PRICE_DYN_PCT / 100) / stride);
        if (s_lim < stride) s_lim = stride;
        if (s_lim < nlist) {
            tkc = P.tickets + ((it & 1) * TKS + tk_k) * 32;
            if (wg0 && tid < TKS) {  // counter tid hands out slots s_lim + tid + TKS t < nlist
                const int rem = nlist - s_lim - tid;
                P.tickets[((it & 1) * TKS + tid) * 32 + 1] = rem > 0 ? (uint32_t)((rem + TKS - 1) / TKS) : 0u;
            }
        }
    }
    uint32_t tk_pend = 0;  // the ticket taken ahead (lane 0)
    // candidate update shared by every mode: Devex key, then the argmin
    auto consider = [&](int64_t j, double e, double wn, double dd) {
        double key = e;
        if (WIN && P.devex) {
            // Devex (include/simplex.h SPX_PRICING_DEVEX): the pending pivot's
            // row entry wn = r.A_j updates this column's reference weight.
            // Steepest edge (SPX_PRICING_STEEPEST, oracle se_choose): the
            // Goldfarb-Reid recurrence with dd = A_j . B^-T alpha
            double w = P.W[j];
            if (pend) {
                if constexpr (SE) {
                    if (j == dvx_leave) w = fmax(se_gp / (dvx_aq * dvx_aq), 1.0);
                    else {
                        const double g = wn / dvx_aq;
                        const double t = fma(g * g, se_gp, fma(-2.0 * g, dd, w));
                        w = fmax(t, fma(g, g, 1.0));
                    }
                } else {
                    if (j == dvx_leave) w = fmax(dvx_wp / (dvx_aq * dvx_aq), 1.0);
                    else {
                        const double g = wn / dvx_aq;
                        w = fmax(w, g * g * dvx_wp);
                    }
                }
                if (lane == 0) {
                    // (a group's last pricing workgroup reads the winner's weight back)
                    if (P.nin > 1) st_agent(&P.W[j], w);
                    else P.W[j] = w;
                }
            }
            key = (e < -P.eps) ? -(e * e) / w : INFINITY;
        }
        if (argmin_better(key, j, best, bj)) { best = key; bj = j; bw = wn; be = e; }
    };
    if constexpr (WM == 3) {
        // window tableau (spx_tabdev.h): one lane per non-basic column, the
        // window sums in pivot order inside the lane; a wave takes 64
        // consecutive list slots
        __shared__ double s_sy[64], s_uq[64];
        if (tid < 64) {
            s_sy[tid] = (pend && tid <= tau) ? P.SY[tid] : 0.0;
            s_uq[tid] = (pend && tid < tau) ? P.U[qq * KW + tid] : 0.0;
        }
        __syncthreads();
        for (int base = (blockIdx.x * WAVES + wave) * 64; base < nlist; base += stride * 64) {
            const int idx = base + lane;
            const bool cv = idx < nlist;
            const int64_t j = cv ? (int64_t)P.nb_list[idx] : 0;
            const double tq = (pend && cv) ? P.T[j * L + qq] : 0.0;
            const double dv = cv ? P.dw[j] : 0.0;
            double w, e;
            tab_price_column(tq, dv, cv ? tau : -1, s_sy, s_uq, [&](int s2) { return P.Wt[j * KW + s2]; }, w, e);
            if (!cv) continue;
            if (pend) P.Wt[j * KW + tau] = w;
            double key = e;
            if (P.devex) {  // include/simplex.h SPX_PRICING_DEVEX
                double wt = P.W[j];
                if (pend) {
                    if (j == dvx_leave) wt = fmax(dvx_wp / (dvx_aq * dvx_aq), 1.0);
                    else {
                        const double g = w / dvx_aq;
                        wt = fmax(wt, g * g * dvx_wp);
                    }
                    P.W[j] = wt;
                }
                key = (e < -P.eps) ? -(e * e) / wt : INFINITY;
            }
            if (argmin_better(key, j, best, bj)) { best = key; bj = j; bw = w; be = e; }
        }
        wave_price_min(best, bj, bw, be);
    } else {
    // The first CH chunks of every column are loaded before the previous
    // column's reduction (and, for the first column, before the LDS fill), so
    // a wave's A stream does not stall at column boundaries.
    // slack columns (A[:, ns:] = I, P.slack_unit): the unit vector's dot
    // products without its stream (see below)
    auto unit_col = [&](int64_t jj) { return P.slack_unit && jj >= P.ns; };
    bool have = pre && !unit_col(j0);
    int idx_next = 0;
    for (int idx = idx0; idx < nlist; idx = idx_next) {
        const bool first = idx == idx0;
        if constexpr (DYN) {
            if (tkc && idx < s_lim && idx + stride >= s_lim) {  // the last static column: the first ticket
                uint32_t t = 0;
                if (lane == 0) t = __hip_atomic_fetch_add(tkc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                tk_pend = t;
            }
        }
        const int64_t j = first ? j0 : nbl(idx);
        const dbl2* __restrict__ col = reinterpret_cast<const dbl2*>(P.A + j * L);
        double wv = 0.0;
        if (WIN && pend && lane < tau) wv = P.Wt[j * KW + lane];
        double a0 = 0.0, a1 = 0.0, b0 = 0.0, b1 = 0.0, d0 = 0.0, d1 = 0.0;
        int64_t k = lane;
        const bool unit = unit_col(j);
        // Two 8-chunk batches in flight through the column: the batch after
        // the prefetched first one is requested before that one is consumed,
        // and every later batch before its predecessor is (kb: the batch
        // base, uniform).  The fma order is the loop's below (the same bits).
        const bool pipe = SPX_PRICE_PIPE && BLOCK <= 512 && have && (L2 & 511) == 0 && L2 > CH * 64;
        auto run_pipe = [&](auto pend_t) {
            constexpr bool PD = decltype(pend_t)::value;
            auto consume = [&](const dbl2* vv, int nb8, int64_t kb) {
#pragma unroll
                for (int h = 0; h < 8; h += LB) {
                    if (h >= nb8) break;
                    dbl2 w[LB], r[LB], x[LB];
#pragma unroll
                    for (int u = 0; u < LB; ++u) {
                        w[u] = Y(kb + lane + (h + u) * 64);
                        if constexpr (PD) r[u] = Rw(kb + lane + (h + u) * 64);
                        if constexpr (PD && SE) x[u] = Vw(kb + lane + (h + u) * 64);
                    }
#pragma unroll
                    for (int u = 0; u < LB; ++u) {
                        a0 = fma(vv[h + u].x, w[u].x, a0);
                        a1 = fma(vv[h + u].y, w[u].y, a1);
                        if constexpr (PD) {
                            b0 = fma(vv[h + u].x, r[u].x, b0);
                            b1 = fma(vv[h + u].y, r[u].y, b1);
                        }
                        if constexpr (PD && SE) {
                            d0 = fma(vv[h + u].x, x[u].x, d0);
                            d1 = fma(vv[h + u].y, x[u].y, d1);
                        }
                    }
                }
            };
            int64_t kb = CH * 64;
            dbl2 vc[8];
            if (DEEP2 && first && deep_hit) {
                // the two deep-prefetched batches, the third requested first
                kb = 2 * CH * 64;
                if (kb < L2) {
#pragma unroll
                    for (int u = 0; u < 8; ++u) vc[u] = ld2<SPX_NT_A>(&col[kb + lane + u * 64]);
                }
                consume(vd0, CH, 0);
                consume(vd1, CH, CH * 64);
                if (kb >= L2) {
                    k = L2;
                    return;
                }
            } else if (DEEP && first && deep_hit) {
                // (WM 4) the one deep-prefetched batch in place of v0
#pragma unroll
                for (int u = 0; u < 8; ++u) vc[u] = ld2<SPX_NT_A>(&col[kb + lane + u * 64]);
                consume(vd0, CH, 0);
            } else {
#pragma unroll
                for (int u = 0; u < 8; ++u) vc[u] = ld2<SPX_NT_A>(&col[kb + lane + u * 64]);
                consume(v0, CH, 0);
            }
            for (; kb + 8 * 64 < L2; kb += 8 * 64) {
                dbl2 vn[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) vn[u] = ld2<SPX_NT_A>(&col[kb + 8 * 64 + lane + u * 64]);
                consume(vc, 8, kb);
#pragma unroll
                for (int u = 0; u < 8; ++u) vc[u] = vn[u];
            }
            consume(vc, 8, kb);
            k = L2;
        };
        if (unit) {
            // column ns + i is e_i: every lane partial of the dense sum stays
            // +0 except the one holding element i, which is fma(1, y_i, +0)
            // (fma with the exact zeros of the other rows adds +-0), so
            // these are the dense loop's bits without its 8L-byte stream
            const int64_t i = j - P.ns, k2 = i >> 1;
            if (lane == (int)(k2 & 63)) {
                const dbl2 w = Y(k2);
                const double v = fma(1.0, (i & 1) ? w.y : w.x, 0.0);
                if (i & 1) a1 = v;
                else a0 = v;
                if (WIN && pend) {
                    const dbl2 r = Rw(k2);
                    const double u = fma(1.0, (i & 1) ? r.y : r.x, 0.0);
                    if (i & 1) b1 = u;
                    else b0 = u;
                    if constexpr (SE) {
                        const dbl2 x = Vw(k2);
                        const double t = fma(1.0, (i & 1) ? x.y : x.x, 0.0);
                        if (i & 1) d1 = t;
                        else d0 = t;
                    }
                }
            }
        } else if (pipe && WIN && pend) {
            run_pipe(std::true_type());
        } else if (pipe) {
            run_pipe(std::false_type());
        } else {
        if (have) {  // consume the prefetched chunks (same k order as the loop)
#pragma unroll
            for (int u = 0; u < CH; ++u) {
                const dbl2 w = Y(lane + u * 64);
                a0 = fma(v0[u].x, w.x, a0);
                a1 = fma(v0[u].y, w.y, a1);
                if (WIN && pend) {
                    const dbl2 r = Rw(lane + u * 64);
                    b0 = fma(v0[u].x, r.x, b0);
                    b1 = fma(v0[u].y, r.y, b1);
                    if constexpr (SE) {
                        const dbl2 x = Vw(lane + u * 64);
                        d0 = fma(v0[u].x, x.x, d0);
                        d1 = fma(v0[u].y, x.y, d1);
                    }
                }
            }
            k += CH * 64;
        }
        if (!WIN || !pend) {
            for (; k + 7 * 64 < L2; k += 8 * 64) {
                dbl2 v[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) v[u] = ld2<SPX_NT_A>(&col[k + u * 64]);
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const dbl2 w = Y(k + u * 64);
                    a0 = fma(v[u].x, w.x, a0);
                    a1 = fma(v[u].y, w.y, a1);
                }
            }
            for (; k < L2; k += 64) {
                const dbl2 v = ld2<SPX_NT_A>(&col[k]);
                const dbl2 w = Y(k);
                a0 = fma(v.x, w.x, a0);
                a1 = fma(v.y, w.y, a1);
            }
        } else {
            for (; k + 7 * 64 < L2; k += 8 * 64) {
                dbl2 v[8], w[8], r[8], x[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) v[u] = ld2<SPX_NT_A>(&col[k + u * 64]);
                // LDS operands fetched LB elements at a time (one
                // LDS latency per batch, not one per element)
#pragma unroll
                for (int h = 0; h < 8; h += LB) {
#pragma unroll
                    for (int u = h; u < h + LB; ++u) {
                        w[u] = Y(k + u * 64);
                        r[u] = Rw(k + u * 64);
                        if constexpr (SE) x[u] = Vw(k + u * 64);
                    }
#pragma unroll
                    for (int u = h; u < h + LB; ++u) {
                        a0 = fma(v[u].x, w[u].x, a0);
                        a1 = fma(v[u].y, w[u].y, a1);
                        b0 = fma(v[u].x, r[u].x, b0);
                        b1 = fma(v[u].y, r[u].y, b1);
                        if constexpr (SE) {
                            d0 = fma(v[u].x, x[u].x, d0);
                            d1 = fma(v[u].y, x[u].y, d1);
                        }
                    }
                }
            }
            for (; k < L2; k += 64) {
                const dbl2 v = ld2<SPX_NT_A>(&col[k]);
                const dbl2 w = Y(k);
                const dbl2 r = Rw(k);
                a0 = fma(v.x, w.x, a0);
                a1 = fma(v.y, w.y, a1);
                b0 = fma(v.x, r.x, b0);
                b1 = fma(v.y, r.y, b1);
                if constexpr (SE) {
                    const dbl2 x = Vw(k);
                    d0 = fma(v.x, x.x, d0);
                    d1 = fma(v.y, x.y, d1);
                }
            }
        }
        }
        // next column's first chunks in flight during this column's reduction
        int nidx = idx + stride;
        if constexpr (DYN) {
            if (tkc && nidx >= s_lim) {  // (wave-uniform) the next column comes by the ticket taken ahead
                nidx = s_lim + tk_k + TKS * (int)__builtin_amdgcn_readfirstlane(tk_pend);
                if (nidx < nlist) {
                    uint32_t t = 0;
                    if (lane == 0) t = __hip_atomic_fetch_add(tkc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    tk_pend = t;
                }
            }
        }
        idx_next = nidx;
        const int64_t jn = nidx < nlist ? nbl(nidx) : 0;
        have = nidx < nlist && L2 >= CH * 64 && !unit_col(jn);
        if (have) {
            const dbl2* cn = reinterpret_cast<const dbl2*>(P.A + jn * L);
#pragma unroll
            for (int u = 0; u < CH; ++u) v0[u] = ld2<SPX_NT_A>(&cn[lane + u * 64]);
        }
        double e, wn = 0.0, dd = 0.0;
        if (WIN && pend) {
            // r_tau . A_j = B_w[q,:] . A_j + sum_s U[q][s] Wt[j][s]; the window
            // terms join the lane partials before the butterflies
            double sa = fma(syl, wv, a0 + a1);
            wn = fma(uq, wv, b0 + b1);
            if constexpr (SE) {
                // A_j . B^-T alpha = v . A_j + sum_{s<tau} (U[:, s] . alpha) Wt[j][s]
                dd = fma(csl, wv, d0 + d1);
                wave_sum3(sa, wn, dd);
            } else {
                wave_sum2(sa, wn);
            }
            if (lane == 0) P.Wt[j * KW + tau] = wn;
            e = fma(syp, wn, sa) - P.c[j];
        } else {
            e = wave_sum(a0 + a1) - P.c[j];
        }
        consider(j, e, wn, dd);
    }
    }

    stamp_stream(win, false);
    // workgroup argmin over waves (lane 0 of each wave holds the wave's best)
    if (lane == 0) red[wave] = PricePartial{best, bj, bw, be};
    __syncthreads();
    if constexpr (DYN) {
        // the previous pass's tickets (final: it ended at the kernel
        // boundary): every wave draws from its counter until it gets a slot
        // past the list, so a counter with waves ends above the slots it
        // hands out; one below them had slots nobody priced (a wrong entering
        // column, or a wrong optimum): stop loudly.  Then zero them.
        if (P.price_dyn && wg0 && tid < TKS) {
            uint32_t* o = P.tickets + (((it + 1) & 1) * TKS + tid) * 32;
            if (o[1] > o[0]) st->uncovered = 1u;
            o[0] = 0u;
            o[1] = 0u;
        }
    }
    if (P.stamps && tid == 0 && blockIdx.x < 4096) {  // diagnostics: this workgroup's start and end
        unsigned long long* pw = P.stamps + STAMP_PRICE + (it & 1) * 4 * 4096 + 4 * (int64_t)blockIdx.x;
        pw[0] = t_pw0;
        pw[1] = rtime();
        pw[2] = t_pw1;
        pw[3] = t_pw2;
    }
    if (P.defer_price) {  // k_update reduces the partials after the kernel boundary
        if (tid == 0) {
            P.price_partials[blockIdx.x] = red[best_wave<WAVES>(red)];
            if (fresh && blockIdx.x == 0) {
                apply_deferred_tail(P, st, s_rec, s_tp);
                if (P.stamps) P.stamps[STAMP_TAIL + 4 + (it & 1)] = rtime();  // the bookkeeping is issued
            }
        }
        return;
    }
    // multi-rank passes (the pricing tail in this launch, for the exchange):
    // workgroup 0 applies a deferred tail before it arrives; the fan-in below
    // reads no state word the bookkeeping writes
    if (fresh && blockIdx.x == 0 && tid == 0) apply_deferred_tail(P, st, s_rec, s_tp);
    if (P.price_tag) {
        // Tagged hand-off (as k_update's, upd_publish_tagged): wave 0
        // publishes the workgroup's partial as PRICE_WORDS {32-bit half, tag}
        // words with one sc1 store instruction, and the last workgroup polls
        // every slot until its words carry this pass's tag -- no drain and no
        // last-arrival count.  The winner's new Wt entry travels in the
        // partial; its earlier window entries were written by earlier kernels.
        const uint32_t tag = (uint32_t)(it + 1);
        if (wave == 0) {
            const PricePartial w = red[best_wave<WAVES>(red)];
            if (lane < PRICE_WORDS) {
                const int f = lane >> 1;
                const uint64_t u = f == 0 ? (uint64_t)__double_as_longlong(w.val)
                                 : f == 1 ? (uint64_t)w.idx
                                 : f == 2 ? (uint64_t)__double_as_longlong(w.w)
                                          : (uint64_t)__double_as_longlong(w.pad);
                const uint32_t half = (lane & 1) ? (uint32_t)(u >> 32) : (uint32_t)u;
                st_agent(&P.price_tag[(int64_t)lane * P.price_cap + blockIdx.x], ((uint64_t)tag << 32) | half);
            }
        }
        if (blockIdx.x != gridDim.x - 1) return;
        const unsigned long long t_tail = slot ? rtime() : 0;
        __shared__ bool s_to;
        if (tid == 0) s_to = false;
        lds_barrier();
        PricePartial w{INFINITY, INT64_MAX, 0.0, 0.0};
        for (int g = tid; g < (int)gridDim.x; g += BLOCK) {
            uint64_t wd[PRICE_WORDS];
            bool ok = false;
            for (uint32_t spins = 0; spins <= (1u << 20); ++spins) {
#pragma unroll
                for (int k = 0; k < PRICE_WORDS; ++k) wd[k] = ld_agent(&P.price_tag[(int64_t)k * P.price_cap + g]);
                ok = true;
#pragma unroll
                for (int k = 0; k < PRICE_WORDS; ++k) ok = ok && (uint32_t)(wd[k] >> 32) == tag;
                if (ok) break;
                __builtin_amdgcn_s_sleep(1);
            }
            if (!ok) {
                s_to = true;  // (a benign race: every writer stores true)
                break;
            }
            uint64_t f[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) f[k] = (wd[2 * k] & 0xffffffffull) | (wd[2 * k + 1] << 32);
            const PricePartial v{__longlong_as_double((long long)f[0]), (int64_t)f[1],
                                 __longlong_as_double((long long)f[2]), __longlong_as_double((long long)f[3])};
            if (argmin_better(v.val, v.idx, w.val, w.idx)) w = v;
#pragma unroll
            for (int k = 0; k < PRICE_WORDS; ++k) P.price_tag[(int64_t)k * P.price_cap + g] = 0ull;
        }
        // wave DPP argmin; the winner's payload from its lane
        double bv = w.val;
        int64_t bj = w.idx;
        lane_argmin<64>(bv, bj);
        bv = readlane_d(bv, 63);
        bj = readlane_l(bj, 63);
        const uint64_t hit = __ballot(w.val == bv && w.idx == bj);
        const int wl = hit ? (int)__builtin_ctzll(hit) : 0;
        const PricePartial o{bv, bj, readlane_d(w.w, wl), readlane_d(w.pad, wl)};
        if (lane == 0) red[wave] = o;
        lds_barrier();
        PricePartial t = red[0];
        for (int i = 1; i < WAVES; ++i)
            if (argmin_better(red[i].val, red[i].idx, t.val, t.idx)) t = red[i];
        if (s_to) {  // a partial never arrived (a fault elsewhere): stop loudly
            if (tid == 0) st->status = ST_HANDOFF_TIMEOUT;
            return;
        }
        if (tid == 0) {
            P.price_out[0] = ArgMinEntry{t.val, t.idx};
            if (WIN && P.devex) *P.dvx_e = t.pad;
            if (WIN && P.devex && P.nin > 1) {  // the reduced cost and weight travel with the record
                double* ex = reinterpret_cast<double*>(P.price_out + 1 + KW / 2);
                ex[0] = t.pad;
                ex[1] = t.idx == INT64_MAX ? 1.0 : ld_agent(&P.W[t.idx]);
            }
        }
        if (WIN && P.nin > 1) {
            double* wo = reinterpret_cast<double*>(P.price_out + 1);
            if (tid < KW)
                wo[tid] = (t.idx == INT64_MAX || tid >= nw) ? 0.0 : (tid == tau ? t.w : P.Wt[t.idx * KW + tid]);
        }
        if (WIN && P.mbox_fused) {
            // fused exchange: the record (the same words k_exchange would
            // send: the entry, the winner's window coefficients, Devex's
            // reduced cost and weight) stored into every rank's mailbox
            // straight from here, one 32-bit half per thread and word
            const int nh = P.pr_stride * 4;
            const int G = P.nin;
            const uint32_t tag = mbox_tag(S.mbox_epoch, it);
            const int64_t par = it & 1;
            for (int h = tid; h < nh; h += BLOCK) {
                const int f = h >> 1;  // the record's 8-byte field
                uint64_t u;
                if (f == 0) u = (uint64_t)__double_as_longlong(t.val);
                else if (f == 1) u = (uint64_t)t.idx;
                else if (f < 2 + KW) {
                    const int d = f - 2;
                    const double v = (t.idx == INT64_MAX || d >= nw) ? 0.0 : (d == tau ? t.w : P.Wt[t.idx * KW + d]);
                    u = (uint64_t)__double_as_longlong(v);
                } else {
                    const double v = f == 2 + KW ? t.pad : (t.idx == INT64_MAX ? 1.0 : ld_agent(&P.W[t.idx]));
                    u = (uint64_t)__double_as_longlong(v);
                }
                const uint64_t w = ((uint64_t)tag << 32) | ((h & 1) ? (uint32_t)(u >> 32) : (uint32_t)u);
                for (int g = 0; g < G; ++g)
                    __hip_atomic_store(&P.mbox_peer[g][(par * G + P.mbox_rank) * nh + h], w, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
        stamp_tail(slot, t_tail, win);
        return;
    }
    if (tid == 0) {
        PricePartial w = red[0];
        for (int i = 1; i < WAVES; ++i)
            if (argmin_better(red[i].val, red[i].idx, w.val, w.idx)) w = red[i];
        st_agent(&P.price_partials[blockIdx.x].val, w.val);
        st_agent(&P.price_partials[blockIdx.x].idx, w.idx);
        if constexpr (WIN) {
            st_agent(&P.price_partials[blockIdx.x].w, w.w);
            st_agent(&P.price_partials[blockIdx.x].pad, w.pad);
        }
        drain_vmem();
        *s_last = arrive_last(arrive_group(P.arrive, ARR_PRICE), gridDim.x, blockIdx.x);
    }
    __syncthreads();
    if (!*s_last) return;
    const unsigned long long t_tail = slot ? rtime() : 0;

    // last workgroup: reduce all partials
    PricePartial w{INFINITY, INT64_MAX, 0.0, 0.0};
    for (int g = tid; g < (int)gridDim.x; g += BLOCK) {
        const double v = ld_agent(&P.price_partials[g].val);
        const int64_t i = ld_agent(&P.price_partials[g].idx);
        if (argmin_better(v, i, w.val, w.idx))
            w = PricePartial{v, i, WIN ? ld_agent(&P.price_partials[g].w) : 0.0,
                             WIN ? ld_agent(&P.price_partials[g].pad) : 0.0};
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const double v = __shfl_xor(w.val, off, 64);
        const int64_t i = __shfl_xor(w.idx, off, 64);
        const double ww = __shfl_xor(w.w, off, 64);
        const double we = __shfl_xor(w.pad, off, 64);
        if (argmin_better(v, i, w.val, w.idx)) w = PricePartial{v, i, ww, we};
    }
    __syncthreads();
    if (lane == 0) red[wave] = w;
    __syncthreads();
    PricePartial t = red[0];
    for (int i = 1; i < WAVES; ++i)
        if (argmin_better(red[i].val, red[i].idx, t.val, t.idx)) t = red[i];
    if (tid == 0) {
        P.price_out[0] = ArgMinEntry{t.val, t.idx};
        if (WIN && P.devex) *P.dvx_e = t.pad;
        if (WIN && P.devex && P.nin > 1) {  // the reduced cost and weight travel with the record
            double* ex = reinterpret_cast<double*>(P.price_out + 1 + KW / 2);
            ex[0] = t.pad;
            ex[1] = t.idx == INT64_MAX ? 1.0 : ld_agent(&P.W[t.idx]);
        }
    }
    if (WIN && P.nin > 1) {
        // the winner's window coefficients Wt[p][0..nw) travel with it (the
        // column may live on another rank's shard; one rank reads Wt directly)
        double* wo = reinterpret_cast<double*>(P.price_out + 1);
        if (tid < KW)
            wo[tid] = (t.idx == INT64_MAX || tid >= nw) ? 0.0 : (tid == tau ? t.w : P.Wt[t.idx * KW + tid]);
    }
    stamp_tail(slot, t_tail, win);
}

// ---------------------------------------------------------------------------
// Fused: pending rank-1 update + FTRAN + x_b update + ratio test + leaving
// argmin + pivot tail
// ---------------------------------------------------------------------------
// Block-wide sum: wave butterflies, then the per-wave sums in wave order.
template <int BLOCK>
__device__ double block_sum(double a, double* sa) {
    constexpr int WAVES = BLOCK / 64;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    a = wave_sum(a);
    if (lane == 0) sa[wave] = a;
    __syncthreads();
    double t = sa[0];
#pragma unroll
    for (int w = 1; w < WAVES; ++w) t += sa[w];
    __syncthreads();
    return t;
}

// Ratio-test partials of the k_update workgroups, stored field-major: field f
// of workgroup g at upd_soa[f * upd_cap + g].  A wave's loads of one field
// over 64 workgroups are then 512 contiguous bytes; with 64-byte records every
// lane's field load was a line of its own (7 x 512 line requests from the one
// CU that runs the tail).
// PLAIN: read only after the kernel boundary (the deferred tail)
template <bool PLAIN = false>
__device__ __forceinline__ void upd_publish(const Params& P, int g, const UpdPartial& w) {
    double* const s = P.upd_soa + g;
    const int64_t c = P.upd_cap;
    auto st = [](auto* q, auto v) {
        if constexpr (PLAIN) *q = v;
        else st_agent(q, v);
    };
    st(&s[0 * c], w.theta);
    st(reinterpret_cast<int64_t*>(&s[1 * c]), w.idx);
    st(reinterpret_cast<int64_t*>(&s[2 * c]), w.nonpos);
    st(&s[3 * c], w.T);
    st(&s[4 * c], w.a_w);
    st(&s[5 * c], w.cb_w);
    st(reinterpret_cast<int64_t*>(&s[6 * c]), w.bix_w);
}
// PLAIN: after a kernel boundary (the deferred tail) the partials are read
// with ordinary loads, so each XCD's L2 serves its workgroups after the first
// miss; inside the producing launch they need agent-scope loads
template <bool PLAIN>
__device__ __forceinline__ UpdPartial upd_fetch(const Params& P, int g) {
    const double* const s = P.upd_soa + g;
    const int64_t c = P.upd_cap;
    auto ld = [](const auto* q) { return PLAIN ? *q : ld_agent(q); };
    UpdPartial v;
    v.theta = ld(&s[0 * c]);
    v.idx = ld(reinterpret_cast<const int64_t*>(&s[1 * c]));
    v.nonpos = ld(reinterpret_cast<const int64_t*>(&s[2 * c]));
    v.T = ld(&s[3 * c]);
    v.a_w = ld(&s[4 * c]);
    v.cb_w = ld(&s[5 * c]);
    v.bix_w = ld(reinterpret_cast<const int64_t*>(&s[6 * c]));
    v.pad = 0;
    return v;
}

// Tagged hand-off (P.upd_tag, the default on replicated B^-1): wave 0 of every
// workgroup publishes its partial as UPD_WORDS 8-byte granules {32-bit half,
// tag} with one sc1 store instruction (lane l = word l; field-major, so the
// poll's loads coalesce), and the last workgroup polls each slot until all
// its words carry this pass's tag (MI355X_MICROARCH.md, handoff-1to1).  The
// slowest workgroup's partial then reaches the tail in one one-way hop; the
// counted form (upd_soa + arrive_last) pays a store drain and two atomic
// round trips first.  The tail clears every slot it consumed, so a slot holds
// a live tag only between its publish and the tail of the same pass.
__device__ __forceinline__ uint64_t upd_field_bits(const UpdPartial& w, int f) {
    switch (f) {
        case 0: return (uint64_t)__double_as_longlong(w.theta);
        case 1: return (uint64_t)w.idx;
        case 2: return (uint64_t)w.nonpos;
        case 3: return (uint64_t)__double_as_longlong(w.T);
        case 4: return (uint64_t)__double_as_longlong(w.a_w);
        case 5: return (uint64_t)__double_as_longlong(w.cb_w);
        default: return (uint64_t)w.bix_w;
    }
}
__device__ __forceinline__ void upd_publish_tagged(const Params& P, int g, const UpdPartial& w, uint32_t tag,
                                                   int lane) {
    if (lane < UPD_WORDS) {
        const uint64_t u = upd_field_bits(w, lane >> 1);
        const uint32_t half = (lane & 1) ? (uint32_t)(u >> 32) : (uint32_t)u;
        st_agent(&P.upd_tag[(int64_t)lane * P.upd_cap + g], ((uint64_t)tag << 32) | half);
    }
}
// Poll slot g until its UPD_WORDS words carry tag; false after ~2^20 rounds.
__device__ __forceinline__ bool upd_poll_tagged(const Params& P, int g, uint32_t tag, UpdPartial& v) {
    uint64_t w[UPD_WORDS];
    for (uint32_t spins = 0;; ++spins) {
        bool ok = true;
#pragma unroll
        for (int k = 0; k < UPD_WORDS; ++k) w[k] = ld_agent(&P.upd_tag[(int64_t)k * P.upd_cap + g]);
#pragma unroll
        for (int k = 0; k < UPD_WORDS; ++k) ok = ok && (uint32_t)(w[k] >> 32) == tag;
        if (ok) break;
        if (spins > (1u << 20)) return false;
        __builtin_amdgcn_s_sleep(1);
    }
    uint64_t f[7];
#pragma unroll
    for (int k = 0; k < 7; ++k) f[k] = (w[2 * k] & 0xffffffffull) | (w[2 * k + 1] << 32);
    v.theta = __longlong_as_double((long long)f[0]);
    v.idx = (int64_t)f[1];
    v.nonpos = (int64_t)f[2];
    v.T = __longlong_as_double((long long)f[3]);
    v.a_w = __longlong_as_double((long long)f[4]);
    v.cb_w = __longlong_as_double((long long)f[5]);
    v.bix_w = (int64_t)f[6];
    v.pad = 0;
    return true;
}
__device__ __forceinline__ void upd_clear_tagged(const Params& P, int g) {
#pragma unroll
    for (int k = 0; k < UPD_WORDS; ++k) P.upd_tag[(int64_t)k * P.upd_cap + g] = 0ull;
}

// Leaving argmin over the k_update workgroup partials + unbounded count
// (v4:317-325), carrying the winner's scalars.  One dependent round trip
// (the sc1 partial loads); result broadcast to every thread.  The T sum's
// order is fixed for a given launch geometry.
// The workgroup's merge of its threads' ratio-test partials (the second half
// of reduce_update_partials; the deferred tail calls it on partials it
// requested at kernel entry)
// wave: DPP argmin on (theta, idx) and DPP sums (no LDS round trips); the
// winner's scalars come from its lane by readlane
__device__ __forceinline__ UpdPartial wave_reduce_partial(const UpdPartial& w) {
    double th = w.theta;
    int64_t ix = w.idx;
    double T = w.T;
    int np = (int)w.nonpos;
    lane_argmin<64>(th, ix);
    lane_sum<64>(T);
    lane_isum<64>(np);
    th = readlane_d(th, 63);
    ix = readlane_l(ix, 63);
    const uint64_t hit = __ballot(w.theta == th && w.idx == ix);
    const int wl = hit ? (int)__builtin_ctzll(hit) : 0;
    UpdPartial o;  // (cross-lane reads outside the lane-0 branch)
    o.theta = th;
    o.idx = ix;
    o.nonpos = __builtin_amdgcn_readlane(np, 63);
    o.T = readlane_d(T, 63);
    o.a_w = readlane_d(w.a_w, wl);
    o.cb_w = readlane_d(w.cb_w, wl);
    o.bix_w = readlane_l(w.bix_w, wl);
    o.pad = 0;
    return o;
}
template <int BLOCK, bool PLAIN>
__device__ __forceinline__ UpdPartial reduce_partial_block(const UpdPartial& w, UpdPartial* red) {
    constexpr int WAVES = BLOCK / 64;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const UpdPartial o = wave_reduce_partial(w);
    if (lane == 0) red[wave] = o;
    lds_barrier();
    if constexpr (PLAIN) {
        // the deferred tail (k_price's prologue, k_apply_tail): every wave
        // partial requested before a branch-free merge, and no closing
        // barrier (the callers pass an LDS array of their own).  (In the
        // FTRAN pass's tail the 8 partials in registers spilled.)
        UpdPartial r[WAVES];
#pragma unroll
        for (int k = 0; k < WAVES; ++k) r[k] = red[k];
        UpdPartial t = r[0];
#pragma unroll
        for (int k = 1; k < WAVES; ++k) upd_merge_sel(t, r[k]);
        return t;
    } else {
        UpdPartial t = red[0];
#pragma unroll
        for (int k = 1; k < WAVES; ++k) upd_merge(t, red[k]);
        lds_barrier();
        return t;
    }
}

// The 2*BLOCK-thread merge above (PLAIN) with BLOCK threads, bit for bit:
// thread tid holds the partials of that shape's threads tid (wa) and
// tid + BLOCK (wb), so its waves w and w + WAVES reduce the same lanes in the
// same order, and the 2*WAVES wave partials merge in the same order.
template <int BLOCK>
__device__ __forceinline__ UpdPartial reduce_partial_pair(const UpdPartial& wa, const UpdPartial& wb,
                                                          UpdPartial* red) {
    constexpr int WAVES = BLOCK / 64;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const UpdPartial oa = wave_reduce_partial(wa);
    const UpdPartial ob = wave_reduce_partial(wb);
    if (lane == 0) {
        red[wave] = oa;
        red[wave + WAVES] = ob;
    }
    lds_barrier();
    UpdPartial r[2 * WAVES];
#pragma unroll
    for (int k = 0; k < 2 * WAVES; ++k) r[k] = red[k];
    UpdPartial t = r[0];
#pragma unroll
    for (int k = 1; k < 2 * WAVES; ++k) upd_merge_sel(t, r[k]);
    return t;
}

template <int BLOCK, bool PLAIN>
__device__ UpdPartial reduce_update_partials(const Params& P, UpdPartial* red, int nparts, uint32_t tag,
                                             bool* timed_out) {
    const int tid = threadIdx.x;
    UpdPartial w = upd_empty();
    if (tag) {  // tagged hand-off: poll, then clear the consumed slots
        bool ok = true;
        for (int g = tid; g < nparts; g += BLOCK) {
            UpdPartial v;
            if (!upd_poll_tagged(P, g, tag, v)) {
                ok = false;
                break;
            }
            upd_merge(w, v);
            upd_clear_tagged(P, g);
        }
        if (!ok) *timed_out = true;  // (a benign race: every writer stores true)
    } else {
        // every slot's seven fields are loaded before any is used (one round trip)
        w = (tid < nparts) ? upd_fetch<PLAIN>(P, tid) : upd_empty();
        for (int g = tid + BLOCK; g < nparts; g += BLOCK) upd_merge(w, upd_fetch<PLAIN>(P, g));
    }
    return reduce_partial_block<BLOCK, PLAIN>(w, red);
}

// LDS carve-up of k_update (dynamic, 16-byte aligned pieces)
template <int BLOCK>
struct UpdLds {
    static constexpr int WAVES = BLOCK / 64;
    static constexpr size_t red = 0;                                    // UpdPartial[WAVES]
    static constexpr size_t last = red + sizeof(UpdPartial) * WAVES;    // int
    static constexpr size_t bytes = last + 16;
};

// Explicit in-place update (v4:331-333): the pivot row r, A_p and b are
// staged in LDS once per workgroup (read from L2 per element they were three
// operand streams beside the B stream), and each wave loads its next chunk of
// B rows before storing this one (vmcnt counts stores too, so loads issued
// behind a chunk's stores could not be waited for without them).  Needs the
// three vectors in LDS and whole 4-chunk steps; from L = 2048 (C3 8.16k ->
// 8.59k it/s, k_update 56 -> 47 us; at C2, L = 1024, the fill cost 1 %).
__host__ __device__ inline bool upd_xlds(const Params& P) {
    return !P.win && !P.row_shard && P.L >= 2048 && P.L * 24 <= 96 * 1024 && ((P.L >> 1) % 256) == 0;
}

// Basis bookkeeping (v4:339-342) + non-basic list swap-remove / append and
// the deferred pivot state (spx_device.h).  One thread.
// Scalars of the bookkeeping that only depend on the entering column, loaded
// by every k_update workgroup at its start so the last one's tail does not
// wait on a chain of dependent global loads.
// (32-bit flags: with bool members the partly-assigned struct was kept in
// scratch rather than registers)
struct TailPre {
    int32_t valid;
    double c_p;
    int32_t cnt, kp, last;
    double wp;  // Devex: the entering column's weight
    int32_t has_e;
    double e_enter;  // deferred pricing tail: the entering column's reduced cost
    int32_t nw;      // eta window: pivots in the window (stable until the tail)
};
// the list tail depends on cnt: loaded at the start of the tail, beside the
// partial loads, instead of as a dependent pair at kernel entry
__device__ __forceinline__ void tail_last(const Params& P, TailPre* t) {
    if (t && t->valid && t->kp >= 0) t->last = P.nb_list[t->cnt - 1];
}

// Devex / steepest edge on a column-shard group: the winning rank's record
// carries the entering column's reduced cost and weight after its window
// coefficients (Params::pr_stride), since only that rank prices the column
__device__ __forceinline__ const double* dvx_payload(const Params& P, int gw) {
    return reinterpret_cast<const double*>(P.price_in + gw * P.pr_stride + 1 + P.win / 2);
}

__device__ __forceinline__ TailPre tail_prefetch(const Params& P, int32_t nw, int32_t cnt, int64_t p) {
    TailPre t{0, 0.0, 0, -1, -1, 0.0, 0, 0.0, 0};
    if (p < 0 || p >= P.n) return t;
    if (P.win) t.nw = nw;
    t.c_p = P.c[p];
    t.cnt = cnt;
    if (owns_col(P, p)) t.kp = P.nb_pos[p];  // (nb_list[cnt - 1] is loaded by the tail: tail_last)
    if (P.devex) t.wp = P.W[p];
    t.valid = true;
    return t;
}

__device__ __forceinline__ void pivot_bookkeeping(const Params& P, DevState* st, int64_t p, int64_t q,
                                                  int64_t leave, double aq, double s_y, double min_e,
                                                  int64_t it, const TailPre* pre = nullptr) {
    P.c_B[q] = pre ? pre->c_p : P.c[p];
    P.b_ixs[q] = p;
    if (P.rleft) P.rleft[q] = 1;  // column q of B^-1 may stop being e_q
    int cnt = pre ? pre->cnt : st->nb_count;
    if (owns_col(P, p)) {
        const int kp = pre ? pre->kp : P.nb_pos[p];
        const int last = pre ? pre->last : P.nb_list[cnt - 1];
        P.nb_list[kp] = last;
        P.nb_pos[last] = kp;
        P.nb_pos[p] = -1;
        --cnt;
    }
    if (owns_col(P, leave)) {
        P.nb_list[cnt] = (int32_t)leave;
        P.nb_pos[leave] = cnt;
        ++cnt;
    }
    st->nb_count = cnt;
    st->aq = aq;
    st->s_y = s_y;
    if (P.win) {  // eta window: the pivot joins the window as its pending entry
        const int32_t nw = (pre && pre->valid) ? pre->nw : st->nw;
        P.SY[nw] = s_y;
        st->nw = nw + 1;
    } else {
        if (st->y_applied < it) st->y_buf ^= 1;  // k_price of this pass persisted y
        st->y_applied = it;
    }
    st->xb_applied = it;
    if (P.devex) {
        st->leave = leave;
        st->wp = pre ? pre->wp : P.W[p];
    }
    st->p = p;
    st->q = q;
    st->min_e = min_e;  // the entering reduced cost (callers resolve Devex's key)
    st->iter = it + 1;
    record_pivot(P, it, p, q);
}

// The last workgroup of k_update (single rank / replicated B^-1): leaving
// row q, unboundedness (v4:317-325), alpha_q, s_y and the bookkeeping.  The
// vector updates are deferred (spx_device.h).
template <int BLOCK>
__device__ void update_tail(const Params& P, DevState* st, int64_t p, double min_e, int64_t it,
                            unsigned char* smem, int nparts, TailPre* pre = nullptr, uint32_t tag = 0) {
    unsigned long long tm = P.stamps ? rtime() : 0;
    if (threadIdx.x == 0) tail_last(P, pre);
    UpdPartial* red = reinterpret_cast<UpdPartial*>(smem + UpdLds<BLOCK>::red);
    __shared__ bool s_to;
    if (threadIdx.x == 0) s_to = false;
    if (tag) lds_barrier();
    const UpdPartial t = reduce_update_partials<BLOCK>(P, red, nparts, tag, &s_to);
    tm = tail_mark(P, 0, tm);
    if (threadIdx.x != 0) return;
    if (tag && s_to) {  // a partial never arrived (a fault elsewhere): stop loudly
        st->status = ST_HANDOFF_TIMEOUT;
        return;
    }
    const int64_t q = t.idx;
    if (t.nonpos == P.m || q < 0 || q >= P.m) {
        // every alpha_i <= 0: Unbounded (v4:319-322).  A ratio test with no
        // valid candidate (NaN-poisoned x_b) stops the same way.  The deferred
        // state of the previous pivot (q, aq, s_y) is left intact for k_flush.
        st->p = p;
        st->min_e = min_e;
        st->status = ST_UNBOUNDED;
        return;
    }
    const double c_p = pre ? pre->c_p : P.c[p];
    const double e_rep = !P.devex ? min_e : (pre && pre->has_e ? pre->e_enter : *P.dvx_e);
    pivot_bookkeeping(P, st, p, q, t.bix_w, t.a_w, y_scalar(t.T, t.a_w, t.cb_w, c_p), e_rep, it, pre);
    tail_mark(P, 1, tm);
}

// The deferred tail's bookkeeping from the reduced partial t (update_tail's,
// with the FTRAN pass's TailRec in place of its prefetched scalars).  One
// thread: workgroup 0 of the next pricing pass, or k_apply_tail.
__device__ __forceinline__ void apply_deferred_tail(const Params& P, DevState* st, const TailRec& R,
                                                    const UpdPartial& t) {
    const int64_t q = t.idx;
    if (t.nonpos == P.m || q < 0 || q >= P.m) {  // Unbounded (v4:319-322)
        st->p = R.p;
        st->min_e = R.e_rep;
        st->status = ST_UNBOUNDED;
        return;
    }
    const TailPre pre{1, R.c_p, R.cnt, R.kp, R.last, R.wp, 0, 0.0, R.nw};
    pivot_bookkeeping(P, st, R.p, q, t.bix_w, t.a_w, y_scalar(t.T, t.a_w, t.cb_w, R.c_p), R.e_rep, R.it, &pre);
}

// A pending deferred tail applied on its own (before a fold, at the end of a
// batch of passes, before any readback): one workgroup of 512 threads, the
// reduction shape of the FTRAN tail and of k_price (the same bits).  Clears
// the record either way.
__global__ __launch_bounds__(512) void k_apply_tail(Params P) {
    DevState* st = P.st;
    const TailRec R = *P.trec;
    if (!R.fresh) return;
    if (R.it == st->iter) {  // not yet applied by a pricing pass
        __shared__ UpdPartial s_ured[9];
        const UpdPartial t = reduce_update_partials<512, true>(P, s_ured, P.tail_parts);
        if (threadIdx.x == 0) apply_deferred_tail(P, st, R, t);
    }
    if (threadIdx.x == 0) P.trec->fresh = 0;
}

hipError_t launch_apply_tail(const Params& P, hipStream_t s) {
    if (!P.trec) return hipSuccess;
    hipLaunchKernelGGL(k_apply_tail, dim3(1), dim3(512), 0, s, P);
    return hipGetLastError();
}

template <int BLOCK>
__device__ void update_tail_rs(const Params& P, DevState* st, int64_t it, int par, const double* a_prev,
                               unsigned char* smem, int nparts);

// Eta-window FTRAN rows: acc[u] += B_w[row u,:] . A_p for R full rows, U dbl2
// loads of B per lane per round trip.  a: A_p in global memory or in LDS.
template <int U, int R, int BNT>
__device__ __forceinline__ void win_rows(const dbl2* __restrict__ a, const dbl2* __restrict__ src, int64_t base,
                                         int64_t L2, int lane, double (&acc)[R], const dbl2 (*pre)[R],
                                         const dbl2 (&apre)[U], bool have_apre) {
    int64_t k = lane;
    if (pre) {  // the first U chunks were loaded at kernel entry (A_p's too when have_apre)
        dbl2 av[U];
#pragma unroll
        for (int t = 0; t < U; ++t) av[t] = have_apre ? apre[t] : a[k + t * 64];
#pragma unroll
        for (int t = 0; t < U; ++t) {
#pragma unroll
            for (int u = 0; u < R; ++u) {
                acc[u] = fma(pre[t][u].x, av[t].x, acc[u]);
                acc[u] = fma(pre[t][u].y, av[t].y, acc[u]);
            }
        }
        k += U * 64;
    }
    for (; k + (U - 1) * 64 < L2; k += U * 64) {
        dbl2 av[U], bv[U][R];
#pragma unroll
        for (int t = 0; t < U; ++t) {
            av[t] = a[k + t * 64];
#pragma unroll
            for (int u = 0; u < R; ++u) bv[t][u] = ld2<BNT>(&src[base + u * L2 + k + t * 64]);
        }
#pragma unroll
        for (int t = 0; t < U; ++t) {
#pragma unroll
            for (int u = 0; u < R; ++u) {
                acc[u] = fma(bv[t][u].x, av[t].x, acc[u]);
                acc[u] = fma(bv[t][u].y, av[t].y, acc[u]);
            }
        }
    }
    for (; k < L2; k += 64) {
        const dbl2 av = a[k];
#pragma unroll
        for (int u = 0; u < R; ++u) {
            const dbl2 bv = src[base + u * L2 + k];
            acc[u] = fma(bv.x, av.x, acc[u]);
            acc[u] = fma(bv.y, av.y, acc[u]);
        }
    }
}

// row i clamped into [0, m): an unconditional prefetch of a row past the end
// reads the last row instead, and is never consumed
__device__ __forceinline__ int64_t clamp_row(int64_t i, int64_t m) { return i < m ? i : m - 1; }

template <int BLOCK, int R, bool RS, bool WIN, int BNT, bool BC>
__global__ __launch_bounds__(BLOCK) void k_update(Params P) {
    DevState* st = P.st;
    using Lds = UpdLds<BLOCK>;
    constexpr int WAVES = BLOCK / 64;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    // eta window: B_w is read-only, so this wave's rows can be in flight
    // before anything else is known (status, entering column, pivot state);
    // a short-lived wave otherwise starts its stream after that chain of
    // dependent loads (tools/stream_bench.hip: the bare 134 MB one-shot
    // stream takes 23 us)
    // (the explicit in-place update measured slower with its old rows loaded
    // this way: C3 59 -> 66 us, so window only)
    // Issue order (vmcnt retires in issue order): the deferred pricing
    // partials, then this wave's first B_w chunks -- unconditional with
    // clamped indices, so the waits below count exactly and the price
    // reduction does not wait for the B prefetch -- then the loop state,
    // field by field (scalar loads: still in the entry block, after no store;
    // a whole-struct snapshot's dead registers were reused at once, and as
    // vector loads the uniform values were moved to scalar registers at once,
    // both waits that held the prefetch), then the multi-rank candidate
    // records and A_p's first chunks.  The status check comes after the price
    // reduction; no store precedes it.
    const int pgi = tid < P.price_grid ? tid : P.price_grid - 1;
    const PricePartial pwl = P.price_partials[pgi];
    constexpr int PFU = WIN ? ((R == 1) ? SPX_WIN_U1 : ((R == 2) ? 8 : ((R == 4) ? 4 : 2))) : ((R >= 4) ? 2 : 4);
    dbl2 pfb[PFU][R];
    const int64_t pf_row = ((int64_t)blockIdx.x * WAVES + wave) * R;
    const bool pf_ok = WIN && !RS && !BC && pf_row + R <= P.m && (P.L >> 1) >= PFU * 64;
    if constexpr (WIN && !RS) {
        const int64_t L2c = P.L >> 1;
        // (compact FTRAN, P.bc: the first BC_PF chunks of this wave's
        // compact rows, the later ones re-requesting chunk 0 (cache hits), so
        // the loads stay unconditional and the waits below exact)
        // (each row clamped on its own: in a partly filled last wave, row u <
        // nvalid must be row pf_row + u, which the compact path consumes)
        const dbl2* b0 = reinterpret_cast<const dbl2*>(BC ? bc_buf(P, P.bc_n[2]) : P.B0);
        const int64_t ld2r = BC ? (int64_t)(P.bc_n[1] >> 1) : L2c;  // row pitch (compact: bc_pitch)
#pragma unroll
        for (int t = 0; t < PFU; ++t) {
            const int64_t k = (BC && t >= BC_PF) ? lane : (lane + t * 64 < L2c ? lane + t * 64 : L2c - 1);
#pragma unroll
            for (int u = 0; u < R; ++u) pfb[t][u] = ld2<BNT>(&b0[clamp_row(pf_row + u, P.m) * ld2r + k]);
        }
    }
    // compact FTRAN: the column list and this wave's unit flags, ahead of p
    int32_t rlv[BC_RL];
    int32_t rmv[R];
    if constexpr (BC) {
#pragma unroll
        for (int j = 0; j < BC_RL; ++j) {
            const int64_t c = tid + (int64_t)j * BLOCK;
            rlv[j] = P.rlist[c < P.m ? c : 0];
        }
#pragma unroll
        for (int u = 0; u < R; ++u) {
            const int64_t i = pf_row + u;
            rmv[u] = P.rmap[i < P.m ? i : 0];
        }
    }
    __builtin_amdgcn_sched_barrier(0);
    struct {
        int32_t status, nb_count, nw;
        int64_t iter, limit, q, xb_applied;
        double aq;
    } Sv;
    Sv.status = st->status;
    Sv.nb_count = st->nb_count;
    Sv.iter = st->iter;
    Sv.limit = st->limit;
    Sv.q = st->q;
    Sv.aq = st->aq;
    Sv.xb_applied = st->xb_applied;
    Sv.nw = st->nw;
    const unsigned long long t_wg0 = (P.stamps && blockIdx.x == 0) ? rtime() : 0ull;
    PricePartial pw0{INFINITY, INT64_MAX, 0.0, 0.0};
    if (P.defer_price && tid < P.price_grid) pw0 = pwl;
    // the merged entering candidates (k_price's last workgroup, one record
    // per rank: MINLOC, v4:294-302), and then A_p's first chunks
    double min_e0 = INFINITY;
    int64_t p0 = INT64_MAX;
    int gw0 = 0;
    if (!P.defer_price) {
        for (int g = 0; g < P.nin; ++g) {
            const ArgMinEntry e = P.price_in[g * P.pr_stride];
            if (argmin_better(e.val, e.idx, min_e0, p0)) { min_e0 = e.val; p0 = e.idx; gw0 = g; }
        }
    }
    dbl2 apf[PFU];
    const bool apf_ok = pf_ok && !P.defer_price && p0 >= 0 && p0 < P.n;
    if (apf_ok) {
        const dbl2* a0 = reinterpret_cast<const dbl2*>(P.A + p0 * P.L);
#pragma unroll
        for (int t = 0; t < PFU; ++t) apf[t] = a0[lane + t * 64];
    }
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

    // entering column: MINLOC over all ranks' candidates (v4:294-302), or,
    // with the pricing tail deferred, over k_price's workgroup partials
    // (every workgroup the same reduction: the same winner)
    double min_e = INFINITY, e_enter = 0.0;
    int64_t p = INT64_MAX;
    int gw = 0;
    if (P.defer_price) {
        PricePartial w = pw0;
        for (int g = tid + BLOCK; g < P.price_grid; g += BLOCK) {
            const PricePartial v = P.price_partials[g];
            if (argmin_better(v.val, v.idx, w.val, w.idx)) w = v;
        }
        // DPP argmin; the winner's reduced cost from its lane (cross-lane
        // reads outside the lane-0 branch)
        double bv = w.val;
        int64_t bj = w.idx;
        lane_argmin<64>(bv, bj);
        bv = readlane_d(bv, 63);
        bj = readlane_l(bj, 63);
        const uint64_t hit = __ballot(w.val == bv && w.idx == bj);
        const double be = readlane_d(w.pad, hit ? (int)__builtin_ctzll(hit) : 0);
        __shared__ PricePartial s_pw[WAVES];
        if (lane == 0) s_pw[wave] = PricePartial{bv, bj, 0.0, be};
        lds_barrier();  // (not __syncthreads: its vmcnt(0) would wait for the B prefetch)
        PricePartial t = s_pw[0];
        for (int i = 1; i < WAVES; ++i)
            if (argmin_better(s_pw[i].val, s_pw[i].idx, t.val, t.idx)) t = s_pw[i];
        min_e = t.val;
        p = t.idx;
        e_enter = t.pad;
    } else {
        min_e = min_e0;
        p = p0;
        gw = gw0;
    }
    const bool dvx_grp = P.devex && P.nin > 1;
    double wp_grp = 1.0;
    if (dvx_grp) {
        const double* ex = dvx_payload(P, gw);
        e_enter = ex[0];
        wp_grp = ex[1];
    }
    if (Sv.status != ST_RUNNING || Sv.iter >= Sv.limit) return;
    wg0_mark(P, 0, t_wg0);
    unsigned long long* const slot = P.stamps ? P.stamps + 4 : nullptr;
    stamp_start(slot);
    wg0_mark(P, 1, t_wg0);
    if (no_entering(P, min_e, p)) {  // OptimumFound (v4:299-302)
        if (blockIdx.x == 0 && tid == 0) {
            st->p = p;
            st->min_e = (P.devex && (P.defer_price || dvx_grp)) ? e_enter : min_e;
            st->status = ST_OPTIMAL;
        }
        return;
    }

    // compact FTRAN (BC): with p known, the operands that depend on it or on
    // S are requested now, ahead of the row scalars (vmcnt retires in order):
    // this row's chunks BC_PF..BC_PF2-1 (chunks past S re-request chunk 0, a
    // cache hit, so the loads stay unconditional), A_p on the column list
    // and A_p[i] for the unit term
    int Sbc = 0;
    dbl2 pf2[BC_PF2 - BC_PF][R];
    double apv[BC_RL], auv[R];
    if constexpr (BC) {
        Sbc = P.bc_n[0];
        const int64_t L2c = P.L >> 1;
        const int64_t ld2r = P.bc_n[1] >> 1;
        const dbl2* b0 = reinterpret_cast<const dbl2*>(bc_buf(P, P.bc_n[2]));
#pragma unroll
        for (int t = BC_PF; t < BC_PF2; ++t) {
            const int k2 = lane + 64 * t;
            const int kk = (2 * k2 < Sbc && k2 < L2c) ? k2 : lane;
#pragma unroll
            for (int u = 0; u < R; ++u) pf2[t - BC_PF][u] = b0[clamp_row(pf_row + u, P.m) * ld2r + kk];
        }
        const double* apd = P.A + p * P.L;
#pragma unroll
        for (int j = 0; j < BC_RL; ++j) apv[j] = apd[rlv[j]];
#pragma unroll
        for (int u = 0; u < R; ++u) auv[u] = apd[clamp_row(pf_row + u, P.m)];
    }
    const int64_t it = Sv.iter;
    const int par = (int)(it & 1);
    const int64_t m = P.m, L = P.L, L2 = L >> 1;
    // row-sharded storage always ping-pongs (its tail recomputes the winner
    // row from the old rows); replicated storage per SPX_INPLACE
    constexpr bool INPL = (SPX_INPLACE || WIN) && !RS;
    const double* S = INPL ? P.B0 : (par ? P.B1 : P.B0);
    const dbl2* src = reinterpret_cast<const dbl2*>(S);
    dbl2* dst = reinterpret_cast<dbl2*>(INPL ? P.B0 : (par ? P.B0 : P.B1));
    const double* a_prev = par ? P.alpha1 : P.alpha0;  // alpha of pivot it-1
    double* a_new = par ? P.alpha0 : P.alpha1;
    // the pending pivot it-1: r = S[q,:], E from a_prev and aq
    const int nw = WIN ? Sv.nw : 0;
    const int tau = nw - 1;  // eta window: the pending pivot
    const bool pend = WIN ? nw > 0 : it > 0;
    const int64_t qp = Sv.q;
    const double aqp = Sv.aq;
    const double* rrow = !pend ? P.zeros : ((SPX_INPLACE || RS) ? P.rbuf : S + qp * L);
    const dbl2* __restrict__ rp = reinterpret_cast<const dbl2*>(rrow);
    const dbl2* __restrict__ ap = reinterpret_cast<const dbl2*>(P.A + p * L);
    const bool upd_x = Sv.xb_applied < it;

    // s_x = r.b (v4:347) for the deferred x_b update is accumulated inside the
    // row stream (every wave streams all of r; lane-strided, k ascending, then
    // a 64-lane butterfly: the same bits in every wave and in k_flush)
    const dbl2* __restrict__ bp = reinterpret_cast<const dbl2*>(P.b);
    double sxa = 0.0;

    // rows of this wave: local storage rows lr0.., global rows gr0..
    const int64_t nrows = RS ? P.mloc : m;
    const int64_t lr0 = ((int64_t)blockIdx.x * WAVES + wave) * R;
    const int64_t gr0 = (RS ? P.r0 : 0) + lr0;
    const int nvalid = (int)((lr0 >= nrows) ? 0 : ((nrows - lr0 < R) ? (nrows - lr0) : R));
    double ei[R], acc[R], cbv[R], xbv[R];
    int64_t bixv[R];
#pragma unroll
    for (int u = 0; u < R; ++u) {
        ei[u] = (pend && u < nvalid) ? eta_entry(a_prev[gr0 + u], gr0 + u, qp, aqp) : 0.0;
        acc[u] = 0.0;
        // row scalars of the epilogue, loaded ahead of the stream
        cbv[u] = u < nvalid ? P.c_B[gr0 + u] : 0.0;
        xbv[u] = u < nvalid ? P.x_b[gr0 + u] : 0.0;
        bixv[u] = u < nvalid ? P.b_ixs[gr0 + u] : -1;
    }
    double ucv[R];  // eta window: this row's U coefficients of the earlier window pivots
#pragma unroll
    for (int u = 0; u < R; ++u)
        ucv[u] = (WIN && u < nvalid && lane < tau) ? P.U[(lr0 + u) * P.win + lane] : 0.0;
    TailPre tpre{0, 0.0, 0, -1, -1, 0.0, 0, 0.0, 0};
    if (!RS && tid == 0 && !P.split_tail) tpre = tail_prefetch(P, Sv.nw, Sv.nb_count, p);
    if (P.defer_price || dvx_grp) {
        tpre.has_e = true;
        tpre.e_enter = e_enter;
    }
    if (dvx_grp) tpre.wp = wp_grp;
    const int64_t base = lr0 * L2;
    unsigned long long* const win = slot ? P.stamps + 16 : nullptr;
    stamp_stream(win, true);
    wg0_mark(P, 2, t_wg0);
    // explicit update with r / A_p / b in LDS (upd_xlds): the whole workgroup
    // stages them (every wave, whatever its rows)
    const bool xl = !WIN && !RS && INPL && upd_xlds(P);
    const dbl2* xr = reinterpret_cast<const dbl2*>(smem + Lds::bytes);
    const dbl2* xa = xr + L2;
    const dbl2* xb = xa + L2;
    if constexpr (!WIN && !RS) {
        if (xl) {
            dbl2* d = reinterpret_cast<dbl2*>(smem + Lds::bytes);
            for (int64_t kk = tid; kk < L2; kk += BLOCK) {
                const dbl2 r2 = rp[kk], a2 = ap[kk], b2 = bp[kk];
                d[kk] = r2;
                d[L2 + kk] = a2;
                d[2 * L2 + kk] = b2;
            }
            lds_barrier();
        }
    }
    if constexpr (WIN) {
        // eta window: B_w is only read; alpha_i = B_w[i,:] . A_p +
        // sum_tau U[i][tau] Wt[p][tau], the window terms (lane tau) joining the
        // lane partials; the pending pivot's eta column is stored into U
        const int KW = P.win;
        const double* wrec = P.nin > 1 ? reinterpret_cast<const double*>(P.price_in + gw * P.pr_stride + 1)
                                       : P.Wt + p * KW;
        const double wl = lane < nw ? wrec[lane] : 0.0;
        // s_x = r_tau . b = xw[q] + sum_{s<tau} U[q][s] Wt[n][s] (v4:347), also
        // kept as Wt[n][tau] for later pivots and the fold: the operands are
        // loaded here, the sum is formed after the stream (a dependent load +
        // butterfly here delayed every wave's stream)
        double sx_u = 0.0, sx_w = 0.0, sx_x = 0.0;
        if (pend) {
            if (lane < tau) {
                sx_u = P.U[qp * KW + lane];
                sx_w = P.Wt[P.n * KW + lane];
            }
            sx_x = P.xw[qp];
        }
        // A_p staged in LDS once per workgroup (SPX_WIN_APLDS) instead of
        // every wave re-reading it through L1/L2 beside the B stream
        const bool aplds = SPX_WIN_APLDS && L * 8 <= 65536;
        if (SPX_WIN_APLDS && aplds) {
            dbl2* d = reinterpret_cast<dbl2*>(smem + Lds::bytes);
            for (int64_t kk = tid; kk < L2; kk += BLOCK) d[kk] = ap[kk];
            __syncthreads();
        }
        if constexpr (BC) {
            // compact FTRAN: B_w[i,:].A_p = sum_c bc[i][c] A_p[rlist[c]] (+ A_p[i]
            // when column i is e_i).  Per lane: the unit term first (lane 0),
            // then its dbl2 chunks lane + 64 t ascending, .x before .y: one
            // order for every geometry and dispatch.  A_p gathered onto the
            // list in LDS; the first BC_PF chunks of each row were requested at
            // kernel entry (pfb), the rest here.
            double* apc = reinterpret_cast<double*>(smem + Lds::bytes);
            const int S = Sbc;
            const double* apd = P.A + p * L;
            const dbl2* apc2 = reinterpret_cast<const dbl2*>(apc);
            double a[R];
#pragma unroll
            for (int u = 0; u < R; ++u) a[u] = (u < nvalid && lane == 0 && rmv[u] < 0) ? auv[u] : 0.0;
            // column blocks of BC_APC (one at S <= 8192): A_p on the block's
            // list entries into LDS, then every row's chunks of the block
            for (int cb = 0; cb < S || cb == 0; cb += BC_APC) {
                const int ce = S < cb + BC_APC ? S : cb + BC_APC;
                if (cb > 0) lds_barrier();  // the previous block's reads are done
#pragma unroll
                for (int j = 0; j < BC_RL; ++j) {
                    const int c = tid + j * BLOCK;
                    if (cb == 0 && c < ce) apc[c] = apv[j];
                }
                for (int c = cb + (cb == 0 ? BC_RL * BLOCK : 0) + tid; c < ce; c += BLOCK) apc[c - cb] = apd[P.rlist[c]];
                lds_barrier();
                const int kb = cb >> 1, ke = (ce + 1) >> 1;  // this block's dbl2 chunks
#pragma unroll
                for (int u = 0; u < R; ++u) {
                    if (u < nvalid) {
                        // the active buffer (bc_n[2]), as the prefetches above read it
                        const dbl2* brow = reinterpret_cast<const dbl2*>(bc_buf(P, P.bc_n[2])) +
                                           (lr0 + u) * (int64_t)(P.bc_n[1] >> 1);
                        auto take = [&](dbl2 v, int k2) {
                            const dbl2 w = apc2[k2 - kb];
                            if (2 * k2 < S) a[u] = fma(v.x, w.x, a[u]);
                            if (2 * k2 + 1 < S) a[u] = fma(v.y, w.y, a[u]);
                        };
                        if (cb == 0) {
#pragma unroll
                            for (int t = 0; t < BC_PF; ++t) {
                                const int k2 = lane + 64 * t;
                                if (k2 < ke) take(pfb[t][u], k2);
                            }
#pragma unroll
                            for (int t = BC_PF; t < BC_PF2; ++t) {
                                const int k2 = lane + 64 * t;
                                if (k2 < ke) take(pf2[t - BC_PF][u], k2);
                            }
                        }
                        for (int k0 = (cb == 0 ? BC_PF2 * 64 : kb); k0 < ke; k0 += 8 * 64) {
                            dbl2 v[8];
#pragma unroll
                            for (int t = 0; t < 8; ++t) {
                                const int k2 = k0 + lane + 64 * t;
                                v[t] = brow[k2 < ke ? k2 : kb];
                            }
#pragma unroll
                            for (int t = 0; t < 8; ++t) {
                                const int k2 = k0 + lane + 64 * t;
                                if (k2 < ke) take(v[t], k2);
                            }
                        }
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < R; ++u)
                if (u < nvalid) acc[u] = a[u];
        } else {
        if (nvalid == R) {
            // 16 dbl2 loads of B per lane in flight: a 32 KiB row is two round trips
            constexpr int U = (R == 1) ? SPX_WIN_U1 : ((R == 2) ? 8 : ((R == 4) ? 4 : 2));
            static_assert(U == PFU, "prefetch and stream chunking agree");
            if (SPX_WIN_APLDS && aplds)
                win_rows<U, R, BNT>(reinterpret_cast<const dbl2*>(smem + Lds::bytes), src, base, L2, lane, acc,
                               pf_ok ? pfb : nullptr, apf, false);
            else
                win_rows<U, R, BNT>(ap, src, base, L2, lane, acc, pf_ok ? pfb : nullptr, apf, apf_ok);
        } else if (nvalid > 0) {
            for (int64_t k = lane; k < L2; k += 64) {
                const dbl2 av = ap[k];
                for (int u = 0; u < nvalid; ++u) {
                    const dbl2 bv = src[base + u * L2 + k];
                    acc[u] = fma(bv.x, av.x, acc[u]);
                    acc[u] = fma(bv.y, av.y, acc[u]);
                }
            }
        }
        }
#pragma unroll
        for (int u = 0; u < R; ++u) {
            if (u < nvalid) {
                const int64_t li = lr0 + u;
                const double cu = lane < tau ? ucv[u] : (lane == tau ? ei[u] : 0.0);
                acc[u] = fma(cu, wl, acc[u]);
                if (pend && lane == 0) P.U[li * KW + tau] = ei[u];
            }
        }
        double sxw = 0.0;
        if (pend) {
            sxw = sx_x + wave_sum(mul_nc(sx_u, sx_w));
            if (blockIdx.x == 0 && tid == 0) P.Wt[P.n * KW + tau] = sxw;
            if (lane == 0) {
                // the exact Wt entries of the basic columns for the pending
                // pivot: r_tau . A_j = aq for its entering column, 0 for the
                // others (their B^-1 A_j is a unit vector)
                for (int u = 0; u < nvalid; ++u) {
                    const int64_t i = gr0 + u;
                    P.Wt[bixv[u] * KW + tau] = (i == qp) ? aqp : 0.0;
                }
            }
        }
        if (upd_x) sxa = sxw;
    } else if (xl && nvalid == R) {
        // r / A_p / b from LDS, B rows one 4-chunk step ahead (upd_xlds)
        constexpr int U = (R >= 4) ? 2 : 4;
        const int nit = (int)(L2 / (U * 64));
        dbl2 bc[U][R], bn[U][R];
        int64_t k = lane;
#pragma unroll
        for (int t = 0; t < U; ++t)
#pragma unroll
            for (int u = 0; u < R; ++u) bc[t][u] = ld2<SPX_NT_BLOAD>(&src[base + u * L2 + k + t * 64]);
        for (int itn = 0; itn < nit; ++itn, k += U * 64) {
            // the next step's rows (the first step's again on the last one:
            // an unconditional load keeps the waits exact)
            const int64_t kn = (itn + 1 < nit) ? k + U * 64 : (int64_t)lane;
#pragma unroll
            for (int t = 0; t < U; ++t)
#pragma unroll
                for (int u = 0; u < R; ++u) bn[t][u] = ld2<SPX_NT_BLOAD>(&src[base + u * L2 + kn + t * 64]);
            dbl2 rv[U], av[U], bb[U];
#pragma unroll
            for (int t = 0; t < U; ++t) {
                rv[t] = xr[k + t * 64];
                av[t] = xa[k + t * 64];
                bb[t] = xb[k + t * 64];
            }
#pragma unroll
            for (int t = 0; t < U; ++t) {
                sxa = fma(rv[t].x, bb[t].x, sxa);
                sxa = fma(rv[t].y, bb[t].y, sxa);
#pragma unroll
                for (int u = 0; u < R; ++u) {
                    dbl2 nv;
                    nv.x = fma(ei[u], rv[t].x, bc[t][u].x);
                    nv.y = fma(ei[u], rv[t].y, bc[t][u].y);
                    st2<SPX_NT_BSTORE>(nv, &dst[base + u * L2 + k + t * 64]);
                    acc[u] = fma(nv.x, av[t].x, acc[u]);
                    acc[u] = fma(nv.y, av[t].y, acc[u]);
                }
            }
#pragma unroll
            for (int t = 0; t < U; ++t)
#pragma unroll
                for (int u = 0; u < R; ++u) bc[t][u] = bn[t][u];
        }
    } else if (nvalid == R) {
        constexpr int U = (R >= 4) ? 2 : 4;
        static_assert(WIN || U == PFU, "prefetch and stream chunking agree");
        int64_t k = lane;
        bool first = pf_ok;
        for (; k + (U - 1) * 64 < L2; k += U * 64) {
            dbl2 rv[U], av[U], bb[U], bv[U][R];
#pragma unroll
            for (int t = 0; t < U; ++t) {
                rv[t] = rp[k + t * 64];
                av[t] = ap[k + t * 64];
                bb[t] = bp[k + t * 64];
#pragma unroll
                for (int u = 0; u < R; ++u)
                    bv[t][u] = first ? pfb[t < PFU ? t : 0][u] : ld2<SPX_NT_BLOAD>(&src[base + u * L2 + k + t * 64]);
            }
            first = false;
#pragma unroll
            for (int t = 0; t < U; ++t) {
                sxa = fma(rv[t].x, bb[t].x, sxa);
                sxa = fma(rv[t].y, bb[t].y, sxa);
#pragma unroll
                for (int u = 0; u < R; ++u) {
                    dbl2 nv;
                    nv.x = fma(ei[u], rv[t].x, bv[t][u].x);
                    nv.y = fma(ei[u], rv[t].y, bv[t][u].y);
                    st2<SPX_NT_BSTORE>(nv, &dst[base + u * L2 + k + t * 64]);
                    acc[u] = fma(nv.x, av[t].x, acc[u]);
                    acc[u] = fma(nv.y, av[t].y, acc[u]);
                }
            }
        }
        for (; k < L2; k += 64) {
            const dbl2 rv = rp[k], av = ap[k], bb = bp[k];
            sxa = fma(rv.x, bb.x, sxa);
            sxa = fma(rv.y, bb.y, sxa);
#pragma unroll
            for (int u = 0; u < R; ++u) {
                const dbl2 bv = src[base + u * L2 + k];
                dbl2 nv;
                nv.x = fma(ei[u], rv.x, bv.x);
                nv.y = fma(ei[u], rv.y, bv.y);
                dst[base + u * L2 + k] = nv;
                acc[u] = fma(nv.x, av.x, acc[u]);
                acc[u] = fma(nv.y, av.y, acc[u]);
            }
        }
    } else if (nvalid > 0) {
        for (int64_t k = lane; k < L2; k += 64) {
            const dbl2 rv = rp[k], av = ap[k], bb = bp[k];
            sxa = fma(rv.x, bb.x, sxa);
            sxa = fma(rv.y, bb.y, sxa);
            for (int u = 0; u < nvalid; ++u) {
                const dbl2 bv = src[base + u * L2 + k];
                dbl2 nv;
                nv.x = fma(ei[u], rv.x, bv.x);
                nv.y = fma(ei[u], rv.y, bv.y);
                dst[base + u * L2 + k] = nv;
                acc[u] = fma(nv.x, av.x, acc[u]);
                acc[u] = fma(nv.y, av.y, acc[u]);
            }
        }
    }

    stamp_stream(win, false);
    wg0_mark(P, 3, t_wg0);
    const double s_x = (upd_x && nvalid > 0) ? (WIN ? sxa : wave_sum(sxa)) : 0.0;

    // x_b += s_x E (v4:348) for the owned rows; alpha_i, theta_i
    // (compute_theta, v4:199-208) and the wave's ratio-test partial
    UpdPartial wp = upd_empty();
#pragma unroll
    for (int u = 0; u < R; ++u) {
        if (u < nvalid) {
            const double a = wave_sum(acc[u]);
            const int64_t i = gr0 + u;
            const double cb = cbv[u];
            double xb = xbv[u];
            if (upd_x) xb = fma(s_x, ei[u], xb);
            if (lane == 0) {
                a_new[i] = a;  // read back by the next pass (own row) / k_flush
                if (upd_x) P.x_b[i] = xb;
            }
            const bool pos = a > P.piv_tol;  // 0 for the reference rule (v4:202)
            const double th = ratio_key(P, xb, a);
            wp.nonpos += !pos;
            wp.T = fma(cb, a, wp.T);
            if (argmin_better(th, i, wp.theta, wp.idx)) {
                wp.theta = th;
                wp.idx = i;
                wp.a_w = a;
                wp.cb_w = cb;
                wp.bix_w = bixv[u];
            }
        }
    }
    UpdPartial* red = reinterpret_cast<UpdPartial*>(smem + Lds::red);
    int* s_last = reinterpret_cast<int*>(smem + Lds::last);
    if (lane == 0) red[wave] = wp;
    // only the partial crosses workgroups inside the launch (thread 0 drains
    // it below), so the barrier waits for LDS only; the row-sharded tail
    // reads other workgroups' alpha: full barrier
    if constexpr (RS) __syncthreads();
    else lds_barrier();
    if (P.split_tail) {  // k_tail merges after the kernel boundary: plain stores, no fan-in
        if (tid == 0) {
            UpdPartial w = red[0];
            for (int i = 1; i < WAVES; ++i) upd_merge(w, red[i]);
            upd_publish(P, blockIdx.x, w);
        }
        return;
    }
    if (!RS && P.upd_tag) {  // tagged hand-off to the last workgroup (upd_publish_tagged)
        const uint32_t tag = (uint32_t)(it + 1);
        if (wave == 0) {
            UpdPartial w = red[0];
            for (int i = 1; i < WAVES; ++i) upd_merge(w, red[i]);
            upd_publish_tagged(P, blockIdx.x, w, tag, lane);
            wg0_mark(P, 4, t_wg0);
        }
        if (blockIdx.x != gridDim.x - 1) return;
        const unsigned long long t_tail = slot ? rtime() : 0;
        update_tail<BLOCK>(P, st, p, min_e, it, smem, gridDim.x, &tpre, tag);
        stamp_tail(slot, t_tail, win);
        return;
    }
    if (tid == 0) {
        UpdPartial w = red[0];
        for (int i = 1; i < WAVES; ++i) upd_merge(w, red[i]);
        upd_publish(P, blockIdx.x, w);
        drain_vmem();  // the partial is visible before the ticket
        *s_last = arrive_last(arrive_group(P.arrive, ARR_UPDATE), gridDim.x, blockIdx.x);
    }
    if constexpr (RS) __syncthreads();
    else lds_barrier();
    if (!*s_last) return;
    const unsigned long long t_tail = slot ? rtime() : 0;
    if constexpr (RS)
        update_tail_rs<BLOCK>(P, st, it, par, a_prev, smem, gridDim.x);
    else
        update_tail<BLOCK>(P, st, p, min_e, it, smem, gridDim.x, &tpre);
    stamp_tail(slot, t_tail, win);
}

// Compact-operand FTRAN pass, one B_w row per wave (the default window
// geometry at C3 / C4: k_update<512, 1, false, true, 0, true>'s work, term for
// term and in the same per-lane order, so the same bits).  What changes is the
// dependency chain.  Everything that does not depend on the entering column
// is requested at kernel entry: the pricing partials, the loop state and the
// list size S, the column list, this row's unit flag, both alpha parities,
// c_B / x_b / b_ixs, its U row, the first BC_PF2 chunks of its compact row
// (chunks past S re-request chunk 0: unconditional loads, exact waits) and the
// s_x operands.  Once p is known a single round trip remains: A_p on the
// column list, A_p[i] and the winner's window coefficients Wt[p][.].  (In
// k_update the chunks past the first waited for S, A_p's gather for the row
// prefetch, and alpha for A_p's gather.)
// (launch bounds: 4 waves per SIMD, <= 128 VGPRs, so two 512-thread
// workgroups share a CU and the C3 grid, 512 workgroups, is resident at once:
// at 130 VGPRs it ran in two rounds, 11.6 -> 17.0 us)
//
// RPW > 1 (deferred tail only; SPX_FTRAN_RPW): each wave takes RPW rows, so
// a workgroup covers RPW of the one-row grid's slots -- slot g = blockIdx.x *
// RPW + r holds rows g * WAVES + wave, exactly the rows the one-row grid's
// workgroup g holds -- and publishes one partial per slot, merged over its
// waves in the same order.  Every row's terms, every slot's partial and the
// next pass's reduction over the slots are therefore those of RPW = 1, bit
// for bit; what changes is that the per-workgroup work (the pricing
// partials' reduction, A_p's gather on the list) is done by RPW times fewer
// workgroups, each wave keeps RPW rows' loads in flight, and the grid fits
// one workgroup per CU (<= 256 VGPRs).
// SEF (steepest edge, Params::se_fused): its own instantiation, so the
// Dantzig / Devex pass keeps its code
template <int BLOCK, bool DEFER, int RPW, bool SEF = false>
__global__ __launch_bounds__(BLOCK, RPW == 1 ? 4 : 2) void k_ftran_bc(Params P) {
    static_assert(RPW == 1 || DEFER, "several rows per wave: the deferred-tail form only");
    DevState* st = P.st;
    using Lds = UpdLds<BLOCK>;
    constexpr int WAVES = BLOCK / 64;
    constexpr int NCH = BC_PF2;  // dbl2 chunks of the compact row requested at entry
    // LDS: the RPW x WAVES wave partials, then A_p on the list
    constexpr size_t RED_BYTES = RPW == 1 ? Lds::bytes : sizeof(UpdPartial) * WAVES * RPW + 16;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int64_t m = P.m, L2 = P.L >> 1;
    const int KW = P.win;
    int64_t irow[RPW], icl[RPW];
    bool rowv[RPW];
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
        irow[r] = ((int64_t)blockIdx.x * RPW + r) * WAVES + wave;  // this wave's rows
        rowv[r] = irow[r] < m;
        icl[r] = rowv[r] ? irow[r] : m - 1;
    }
    // ---- entry: everything independent of p (issue order = retire order)
    const int pgi = tid < P.price_grid ? tid : P.price_grid - 1;
    const PricePartial pwl = P.price_partials[pgi];
    int32_t rlv[BC_RL];
#pragma unroll
    for (int j = 0; j < BC_RL; ++j) {
        const int64_t c = tid + (int64_t)j * BLOCK;
        rlv[j] = P.rlist[c < m ? c : 0];
    }
    int32_t rmv[RPW];
    double al0[RPW], al1[RPW], cbv[RPW], xb0[RPW], urow[RPW];
    int64_t bix[RPW];
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
        rmv[r] = P.rmap[icl[r]];
        al0[r] = P.alpha0[icl[r]];
        al1[r] = P.alpha1[icl[r]];
        cbv[r] = P.c_B[icl[r]];
        xb0[r] = P.x_b[icl[r]];
        bix[r] = P.b_ixs[icl[r]];
        if constexpr (!(SPX_FTRAN_TRIM & 2)) urow[r] = P.U[icl[r] * KW + (lane < KW ? lane : 0)];
    }
    const double sxw_w = P.Wt[P.n * KW + (lane < KW ? lane : 0)];
    struct {
        int32_t status, nb_count, nw;
        int64_t iter, limit, q, xb_applied;
        double aq;
    } Sv;
    Sv.status = st->status;
    Sv.nb_count = st->nb_count;
    Sv.iter = st->iter;
    Sv.limit = st->limit;
    Sv.q = st->q;
    Sv.aq = st->aq;
    Sv.xb_applied = st->xb_applied;
    Sv.nw = st->nw;
    const int Sbc = P.bc_n[0];
    const int64_t ldc = P.bc_n[1];  // compact row pitch (k_bc_list)
    const double* const bcb = bc_buf(P, P.bc_n[2]);  // the active buffer
    // (the entry clock goes here: taken first, its kernel-argument test ahead
    // of the loads reordered them, 11.7 -> 13.0 us)
    const unsigned long long t_wg_entry = P.stamps ? rtime() : 0ull;
    // the compact rows' first NCH chunks (S and the state are scalars: one wait)
    const dbl2* brow[RPW];
    dbl2 pf[RPW][NCH];
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
        brow[r] = reinterpret_cast<const dbl2*>(bcb + icl[r] * ldc);
#pragma unroll
        for (int t = 0; t < NCH; ++t) {
            const int k2 = lane + 64 * t;
            const int kk = t == 0 ? ((SPX_FTRAN_TRIM & 1) ? (2 * k2 < Sbc ? k2 : (lane & 7)) : (k2 < L2 ? k2 : (int)L2 - 1))
                                  : ((2 * k2 < Sbc && k2 < L2) ? k2 : ((SPX_FTRAN_TRIM & 1) ? (lane & 7) : lane));
            pf[r][t] = brow[r][kk];
        }
    }
    if constexpr ((SPX_FTRAN_TRIM & 2) != 0) {
#pragma unroll
        for (int r = 0; r < RPW; ++r) urow[r] = P.U[icl[r] * KW + (lane < Sv.nw - 1 ? lane : 0)];
    }
    const int64_t qp = Sv.q;
    const bool pend = Sv.nw > 0;
    const int tau = Sv.nw - 1;
    const double sxw_u = P.U[(pend ? qp : 0) * KW + (lane < KW ? lane : 0)];
    const double sx_x = P.xw[pend ? qp : 0];
    __builtin_amdgcn_sched_barrier(0);
    // ---- entering column (v4:294-302): k_price's workgroup partials (every
    // workgroup the same reduction), or the ranks' merged candidates
    double min_e = INFINITY, e_enter = 0.0;
    int64_t p = INT64_MAX;
    int gw = 0;
    // (fused exchange: the polled entries, the winner's record after its
    // entry -- KW window coefficients, then Devex's two -- and a timeout flag)
    __shared__ uint32_t s_fh[4 * MBOX_FUSED_MAX_G];
    __shared__ double s_fw[64 + 2];
    __shared__ int s_fto;
    if (P.defer_price) {
        PricePartial w = tid < P.price_grid ? pwl : PricePartial{INFINITY, INT64_MAX, 0.0, 0.0};
        for (int g = tid + BLOCK; g < P.price_grid; g += BLOCK) {
            const PricePartial v = P.price_partials[g];
            if (argmin_better(v.val, v.idx, w.val, w.idx)) w = v;
        }
        double bv = w.val;
        int64_t bj = w.idx;
        lane_argmin<64>(bv, bj);
        bv = readlane_d(bv, 63);
        bj = readlane_l(bj, 63);
        const uint64_t hit = __ballot(w.val == bv && w.idx == bj);
        const double be = readlane_d(w.pad, hit ? (int)__builtin_ctzll(hit) : 0);
        __shared__ PricePartial s_pw[WAVES];
        if (lane == 0) s_pw[wave] = PricePartial{bv, bj, 0.0, be};
        lds_barrier();
        if constexpr (WAVES <= 8) {
            // every wave's entry requested, then a branch-free scan (a branch
            // per step on the uniform LDS values waited for each read in turn)
            double pv[WAVES], pe[WAVES];
            int64_t pj[WAVES];
#pragma unroll
            for (int k = 0; k < WAVES; ++k) {
                pv[k] = s_pw[k].val;
                pj[k] = s_pw[k].idx;
                pe[k] = s_pw[k].pad;
            }
            min_e = pv[0];
            p = pj[0];
            e_enter = pe[0];
#pragma unroll
            for (int k = 1; k < WAVES; ++k) {
                const bool b = argmin_better(pv[k], pj[k], min_e, p);
                min_e = b ? pv[k] : min_e;
                p = b ? pj[k] : p;
                e_enter = b ? pe[k] : e_enter;
            }
        } else {  // (16 waves: the preloaded entries spilled)
            PricePartial t = s_pw[0];
            for (int k = 1; k < WAVES; ++k)
                if (argmin_better(s_pw[k].val, s_pw[k].idx, t.val, t.idx)) t = s_pw[k];
            min_e = t.val;
            p = t.idx;
            e_enter = t.pad;
        }
    } else if (P.mbox_fused) {
        // fused exchange: wave 0 polls the ranks' entries in this rank's
        // mailbox, every wave merges them (the same rule as the all-gather's
        // consumers), then wave 0 polls the winner's window coefficients and
        // Devex payload; both reach the other waves through LDS
        const int G = P.nin;
        const bool live = Sv.status == ST_RUNNING && Sv.iter < Sv.limit;
        const uint32_t tag = mbox_tag(st->mbox_epoch, Sv.iter);
        const int64_t par = Sv.iter & 1;
        if (tid == 0) s_fto = 0;
        if (wave == 0 && live) {
            bool ok = true;
            for (int k = lane; k < 4 * G; k += 64) {
                uint32_t hf = 0u;
                ok = mbox_poll(P, par, k >> 2, k & 3, tag, &hf) && ok;
                s_fh[k] = hf;
            }
            if (!ok) s_fto = 1;  // (a benign race: every writer stores 1)
        }
        lds_barrier();
        if (live) {
            for (int g = 0; g < G; ++g) {
                const double v = __longlong_as_double((long long)(((uint64_t)s_fh[4 * g + 1] << 32) | s_fh[4 * g]));
                const int64_t j = (int64_t)(((uint64_t)s_fh[4 * g + 3] << 32) | s_fh[4 * g + 2]);
                if (argmin_better(v, j, min_e, p)) { min_e = v; p = j; gw = g; }
            }
            const int nw2 = P.pr_stride * 2 - 2;  // 8-byte fields after the entry: KW (+ 2 with Devex)
            if (wave == 0 && !s_fto) {
                bool ok = true;
                for (int k = lane; k < nw2; k += 64) {
                    uint32_t lo = 0u, hi = 0u;
                    ok = mbox_poll(P, par, gw, 4 + 2 * k, tag, &lo) && ok;
                    ok = mbox_poll(P, par, gw, 5 + 2 * k, tag, &hi) && ok;
                    s_fw[k] = __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
                }
                if (!ok) s_fto = 1;
            }
            lds_barrier();
            if (s_fto) {
                if (tid == 0) {
                    st->status = ST_HANDOFF_TIMEOUT;
                    if (DEFER) P.trec->fresh = 0;
                }
                return;
            }
        }
    } else {
        for (int g = 0; g < P.nin; ++g) {
            const ArgMinEntry e = P.price_in[g * P.pr_stride];
            if (argmin_better(e.val, e.idx, min_e, p)) { min_e = e.val; p = e.idx; gw = g; }
        }
    }
    const bool dvx_grp = P.devex && P.nin > 1;
    double wp_grp = 1.0;
    if (dvx_grp) {
        const double* ex = P.mbox_fused ? s_fw + KW : dvx_payload(P, gw);
        e_enter = ex[0];
        wp_grp = ex[1];
    }
    if (Sv.status != ST_RUNNING || Sv.iter >= Sv.limit) {
        if (DEFER && blockIdx.x == 0 && tid == 0) P.trec->fresh = 0;  // no pivot: nothing deferred
        return;
    }
    // (diagnostics: plain per-workgroup stores only -- the atomic phase
    // stamps of the other kernels, 512 workgroups on one address, would
    // themselves delay this kernel's waits)
    unsigned long long* const slot = nullptr;
    unsigned long long* const wgt =
        (P.stamps && tid == 0 && blockIdx.x < 4096) ? P.stamps + STAMP_FTRAN + (Sv.iter & 1) * 4 * 4096 + 4 * (int64_t)blockIdx.x
                                                    : nullptr;
    if (wgt) {
        wgt[0] = t_wg_entry;
        wgt[1] = rtime();
    }
    if (no_entering(P, min_e, p)) {  // OptimumFound (v4:299-302)
        if (blockIdx.x == 0 && tid == 0) {
            st->p = p;
            st->min_e = (P.devex && (P.defer_price || dvx_grp)) ? e_enter : min_e;
            st->status = ST_OPTIMAL;
            if (DEFER) P.trec->fresh = 0;
        }
        return;
    }
    // ---- the one p-dependent round trip: A_p on the list and at row i, the
    // winner's window coefficients, the bookkeeping scalars (thread 0)
    // (only the S list slots: every workgroup gathers the same column, so
    // slots past S would multiply the L2 requests for nothing)
    const double* apd = P.A + p * P.L;
    double apv[BC_RL];
#pragma unroll
    for (int j = 0; j < BC_RL; ++j) apv[j] = (tid + j * BLOCK < Sbc) ? apd[rlv[j]] : 0.0;
    double auv[RPW];
#pragma unroll
    for (int r = 0; r < RPW; ++r) auv[r] = apd[icl[r]];
    const double* wrec = P.mbox_fused ? s_fw
                                      : (P.nin > 1 ? reinterpret_cast<const double*>(P.price_in + gw * P.pr_stride + 1)
                                                   : P.Wt + p * KW);
    const double wlr = wrec[lane < KW ? lane : 0];
    TailPre tpre{0, 0.0, 0, -1, -1, 0.0, 0, 0.0, 0};
    if (!DEFER && tid == 0 && !P.split_tail) tpre = tail_prefetch(P, Sv.nw, Sv.nb_count, p);
    // deferred tail: workgroup 0 records tail_prefetch's scalars (as scalars:
    // the record written from tpre kept tpre in scratch)
    double rc_p = 0.0, rwp = 0.0;
    int32_t rkp = -1, rlast = -1;
    if (DEFER && blockIdx.x == 0 && tid == 0) {
        rc_p = P.c[p];
        if (owns_col(P, p)) {
            rkp = P.nb_pos[p];
            rlast = P.nb_list[Sv.nb_count - 1];
        }
        if (P.devex) rwp = dvx_grp ? wp_grp : P.W[p];
    }
    if (P.defer_price || dvx_grp) {
        tpre.has_e = true;
        tpre.e_enter = e_enter;
    }
    if (dvx_grp) tpre.wp = wp_grp;
    const int64_t it = Sv.iter;
    const int par = (int)(it & 1);
    double* a_new = par ? P.alpha0 : P.alpha1;
    const double aqp = Sv.aq;
    const bool upd_x = Sv.xb_applied < it;
    double ei[RPW];
#pragma unroll
    for (int r = 0; r < RPW; ++r) ei[r] = (pend && rowv[r]) ? eta_entry(par ? al1[r] : al0[r], irow[r], qp, aqp) : 0.0;
    unsigned long long* const win = nullptr;
    // ---- compact FTRAN (as k_update BC): the unit term first (lane 0), then
    // this lane's chunks lane + 64 t ascending, .x before .y; A_p gathered
    // onto the list in LDS blocks of BC_APC columns
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    double* apc = reinterpret_cast<double*>(smem + RED_BYTES);
    const dbl2* apc2 = reinterpret_cast<const dbl2*>(apc);
    const int S = Sbc;
    double a[RPW];
#pragma unroll
    for (int r = 0; r < RPW; ++r) a[r] = (rowv[r] && lane == 0 && rmv[r] < 0) ? auv[r] : 0.0;
    for (int cb = 0; cb < S || cb == 0; cb += BC_APC) {
        const int ce = S < cb + BC_APC ? S : cb + BC_APC;
        if (cb > 0) lds_barrier();  // the previous block's reads are done
#pragma unroll
        for (int j = 0; j < BC_RL; ++j) {
            const int c = tid + j * BLOCK;
            if (cb == 0 && c < ce) apc[c] = apv[j];
        }
        for (int c = cb + (cb == 0 ? BC_RL * BLOCK : 0) + tid; c < ce; c += BLOCK) apc[c - cb] = apd[P.rlist[c]];
        lds_barrier();
        if (wgt && cb == 0) wgt[2] = rtime();
        const int kb = cb >> 1, ke = (ce + 1) >> 1;  // this block's dbl2 chunks
#pragma unroll
        for (int r = 0; r < RPW; ++r) {
            if (rowv[r]) {
                auto take = [&](dbl2 v, int k2) {
                    const dbl2 w = apc2[k2 - kb];
                    if (2 * k2 < S) a[r] = fma(v.x, w.x, a[r]);
                    if (2 * k2 + 1 < S) a[r] = fma(v.y, w.y, a[r]);
                };
                if (cb == 0) {
#pragma unroll
                    for (int t = 0; t < NCH; ++t) {
                        const int k2 = lane + 64 * t;
                        if (k2 < ke) take(pf[r][t], k2);
                    }
                }
                for (int k0 = (cb == 0 ? NCH * 64 : kb); k0 < ke; k0 += 8 * 64) {
                    dbl2 v[8];
#pragma unroll
                    for (int t = 0; t < 8; ++t) {
                        const int k2 = k0 + lane + 64 * t;
                        v[t] = brow[r][k2 < ke ? k2 : kb];
                    }
#pragma unroll
                    for (int t = 0; t < 8; ++t) {
                        const int k2 = k0 + lane + 64 * t;
                        if (k2 < ke) take(v[t], k2);
                    }
                }
            }
        }
    }
    // ---- window terms, the pending eta column, s_x (the row's stores wait
    // until the partial is out: a wave's vmcnt counts its stores, so stores
    // issued before the merge put their write acknowledgements on the path
    // to the publish)
    const double wl = lane < Sv.nw ? wlr : 0.0;
    double acc[RPW];
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
        acc[r] = 0.0;
        if (rowv[r]) {
            const double cu = lane < tau ? urow[r] : (lane == tau ? ei[r] : 0.0);
            acc[r] = fma(cu, wl, a[r]);
        }
    }
    double sxw = 0.0;
    if (pend) sxw = sx_x + wave_sum(lane < tau ? mul_nc(sxw_u, sxw_w) : 0.0);
    const double s_x = upd_x ? sxw : 0.0;

    // ---- x_b += s_x E (v4:348), alpha_i, theta_i (v4:199-208), the partials
    // (the RPW rows' butterflies interleaved: each value's own bits)
    auto rows_step = [&](auto off_t) {
        constexpr int OFF = decltype(off_t)::value;
        double t[RPW];
#pragma unroll
        for (int r = 0; r < RPW; ++r) t[r] = xor_partner<OFF>(acc[r]);
#pragma unroll
        for (int r = 0; r < RPW; ++r) acc[r] += t[r];
    };
    rows_step(std::integral_constant<int, 32>());
    rows_step(std::integral_constant<int, 16>());
    rows_step(std::integral_constant<int, 8>());
    rows_step(std::integral_constant<int, 4>());
    rows_step(std::integral_constant<int, 2>());
    rows_step(std::integral_constant<int, 1>());
    UpdPartial wp[RPW];
    double al[RPW], xb[RPW];
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
        wp[r] = upd_empty();
        al[r] = 0.0;
        xb[r] = xb0[r];
        if (rowv[r]) {
            al[r] = acc[r];
            if (upd_x) xb[r] = fma(s_x, ei[r], xb[r]);
            const bool pos = al[r] > P.piv_tol;
            const double th = ratio_key(P, xb[r], al[r]);
            wp[r].nonpos += !pos;
            wp[r].T = fma(cbv[r], al[r], wp[r].T);
            if (argmin_better(th, irow[r], wp[r].theta, wp[r].idx)) {
                wp[r].theta = th;
                wp[r].idx = irow[r];
                wp[r].a_w = al[r];
                wp[r].cb_w = cbv[r];
                wp[r].bix_w = bix[r];
            }
        }
    }
    // alpha_i (read back by the next pass / k_flush), x_b, the pending eta
    // entry into U, and the basic columns' Wt entries (s_x in Wt[n])
    auto store_row = [&]() {
#pragma unroll
        for (int r = 0; r < RPW; ++r) {
            if (rowv[r] && lane == 0) {
                const int64_t i = irow[r];
                if (pend) P.U[i * KW + tau] = ei[r];
                a_new[i] = al[r];
                if (upd_x) P.x_b[i] = xb[r];
                if (pend) P.Wt[bix[r] * KW + tau] = (i == qp) ? aqp : 0.0;
            }
        }
        if (pend && blockIdx.x == 0 && tid == 0) P.Wt[P.n * KW + tau] = sxw;
    };
    // (the counted and tagged hand-offs: stores first, as their tail's polls
    // would otherwise wait behind them; deferred: after the publish)
    if constexpr (!DEFER) store_row();
    UpdPartial* red = reinterpret_cast<UpdPartial*>(smem + Lds::red);
    int* s_last = reinterpret_cast<int*>(smem + Lds::last);
    if (lane == 0) {
#pragma unroll
        for (int r = 0; r < RPW; ++r) red[r * WAVES + wave] = wp[r];
    }
    lds_barrier();
    if (P.split_tail) {  // k_tail merges after the kernel boundary
        if (tid == 0) {
            UpdPartial w = red[0];
            for (int k = 1; k < WAVES; ++k) upd_merge(w, red[k]);
            upd_publish(P, blockIdx.x, w);
        }
        return;
    }
    if constexpr (DEFER) {  // the next pricing pass (or k_apply_tail) reduces the partials
        if (tid < RPW) {
            const int r = tid;
            const int g = blockIdx.x * RPW + r;
            UpdPartial w = red[r * WAVES];
            for (int k = 1; k < WAVES; ++k) upd_merge(w, red[r * WAVES + k]);
            if (g < P.tail_parts) upd_publish<true>(P, g, w);
            if (wgt) wgt[3] = rtime();
            if (g == 0) {
                TailRec* rec = P.trec;
                rec->it = it;
                rec->p = p;
                rec->e_rep = !P.devex ? min_e : ((P.defer_price || dvx_grp) ? e_enter : *P.dvx_e);
                rec->c_p = rc_p;
                rec->wp = rwp;
                rec->cnt = Sv.nb_count;
                rec->kp = rkp;
                rec->last = rlast;
                rec->nw = Sv.nw;
                rec->fresh = 1;
            }
        }
        if constexpr (SEF && RPW == 1) {
            {
                // steepest edge, k_se_part's sums fused (the pending pivot is
                // this pass's: alpha = al, U[i][s] for s <= tau = cu): this
                // workgroup's rows' terms of M^T alpha for M = [B_w at the S
                // listed columns | U[:, s < nw] | alpha], summed over its waves
                // in row order, in LDS blocks of sec columns (the A_p list's
                // space: every wave has passed its last read of it)
                const int64_t Ls = P.L;
                const int ncol = S + KW + 1;
                const int sec = (int)((Ls < BC_APC ? Ls : BC_APC) / WAVES);
                const double av = rowv[0] ? al[0] : 0.0;
                const double cuv = rowv[0] ? (lane < tau ? urow[0] : (lane == tau ? ei[0] : 0.0)) : 0.0;
                const double* rowp = bcb + icl[0] * ldc;
                double* outp = P.se_part + (int64_t)blockIdx.x * (Ls + KW + 1);
                double* sp = apc + wave * sec;
                for (int c0 = 0; c0 < ncol; c0 += sec) {
                    const int c1 = ncol < c0 + sec ? ncol : c0 + sec;
                    if (c0 > 0) lds_barrier();  // the previous block's sums are read
                    for (int c = c0 + lane; c < c1; c += 64) {
                        if (c < S) sp[c - c0] = rowp[c] * av;
                        else if (c == S + KW) sp[c - c0] = av * av;
                    }
                    if (lane < KW && S + lane >= c0 && S + lane < c1) sp[S + lane - c0] = cuv * av;
                    lds_barrier();
                    for (int c = c0 + tid; c < c1; c += BLOCK) {
                        double t = apc[c - c0];
#pragma unroll
                        for (int w = 1; w < WAVES; ++w) t += apc[w * sec + c - c0];
                        outp[c] = t;
                    }
                }
            }
        }
        store_row();
        return;
    }
    if (P.upd_tag) {  // tagged hand-off to the last workgroup
        const uint32_t tag = (uint32_t)(it + 1);
        if (wave == 0) {
            UpdPartial w = red[0];
            for (int k = 1; k < WAVES; ++k) upd_merge(w, red[k]);
            upd_publish_tagged(P, blockIdx.x, w, tag, lane);
            if (wgt) wgt[3] = rtime();
        }
        if (blockIdx.x != gridDim.x - 1) return;
        const unsigned long long t_tail = slot ? rtime() : 0;
        update_tail<BLOCK>(P, st, p, min_e, it, smem, gridDim.x, &tpre, tag);
        stamp_tail(slot, t_tail, win);
        if (wgt) P.stamps[STAMP_TAIL + (it & 1)] = rtime();  // the bookkeeping is issued
        return;
    }
    if (tid == 0) {
        UpdPartial w = red[0];
        for (int k = 1; k < WAVES; ++k) upd_merge(w, red[k]);
        upd_publish(P, blockIdx.x, w);
        drain_vmem();  // the partial is visible before the ticket
        *s_last = arrive_last(arrive_group(P.arrive, ARR_UPDATE), gridDim.x, blockIdx.x);
    }
    lds_barrier();
    if (!*s_last) return;
    const unsigned long long t_tail = slot ? rtime() : 0;
    update_tail<BLOCK>(P, st, p, min_e, it, smem, gridDim.x, &tpre);
    stamp_tail(slot, t_tail, win);
}
// Window tableau FTRAN (spx_tabdev.h): one lane per row,
// alpha_i = T_w[i,p] + sum_s U[i][s] Wt[p][s] — no B_w stream — then the
// pending eta column into U, the basic columns' Wt entries, x_b, the ratio
// test (v4:199-208) and, in the last workgroup, k_update's tail.
template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_tab_update(Params P) {
    DevState* st = P.st;
    if (stopped(st)) return;
    constexpr int WAVES = BLOCK / 64;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ double s_wp[64];
    // entering column, as k_update
    double min_e = INFINITY, e_enter = 0.0;
    int64_t p = INT64_MAX;
    if (P.defer_price) {
        PricePartial w{INFINITY, INT64_MAX, 0.0, 0.0};
        for (int g = tid; g < P.price_grid; g += BLOCK) {
            const PricePartial v = P.price_partials[g];
            if (argmin_better(v.val, v.idx, w.val, w.idx)) w = v;
        }
        wave_price_min(w.val, w.idx, w.w, w.pad);
        __shared__ PricePartial s_pw[WAVES];
        if (lane == 0) s_pw[wave] = w;
        __syncthreads();
        PricePartial t = s_pw[0];
        for (int i = 1; i < WAVES; ++i)
            if (argmin_better(s_pw[i].val, s_pw[i].idx, t.val, t.idx)) t = s_pw[i];
        min_e = t.val;
        p = t.idx;
        e_enter = t.pad;
    } else {
        for (int g = 0; g < P.nin; ++g) {
            const ArgMinEntry e = P.price_in[g * P.pr_stride];
            if (argmin_better(e.val, e.idx, min_e, p)) { min_e = e.val; p = e.idx; }
        }
    }
    if (no_entering(P, min_e, p)) {  // OptimumFound (v4:299-302)
        if (blockIdx.x == 0 && tid == 0) {
            st->p = p;
            st->min_e = (P.devex && P.defer_price) ? e_enter : min_e;
            st->status = ST_OPTIMAL;
        }
        return;
    }
    const int64_t it = st->iter;
    const int par = (int)(it & 1);
    const int64_t m = P.m, L = P.L;
    const int KW = P.win;
    const double* a_prev = par ? P.alpha1 : P.alpha0;
    double* a_new = par ? P.alpha0 : P.alpha1;
    const int nw = st->nw;
    const int tau = nw - 1;
    const bool pend = nw > 0;
    const int64_t qp = st->q;
    const double aqp = st->aq;
    const bool upd_x = st->xb_applied < it;
    if (tid < 64) s_wp[tid] = (tid < nw) ? P.Wt[p * KW + tid] : 0.0;
    // s_x = r_tau . b = xw[q] + sum_{s<tau} U[q][s] Wt[n][s] (v4:347), as k_update
    double sxw = 0.0;
    if (pend) {
        sxw = lane < tau ? mul_nc(P.U[qp * KW + lane], P.Wt[P.n * KW + lane]) : 0.0;
        sxw = P.xw[qp] + wave_sum(sxw);
        if (blockIdx.x == 0 && tid == 0) P.Wt[P.n * KW + tau] = sxw;
    }
    const double s_x = upd_x ? sxw : 0.0;
    TailPre tpre{0, 0.0, 0, -1, -1, 0.0, 0, 0.0, 0};
    if (tid == 0 && !P.split_tail) tpre = tail_prefetch(P, st->nw, st->nb_count, p);
    if (P.defer_price) {
        tpre.has_e = true;
        tpre.e_enter = e_enter;
    }
    __syncthreads();
    const int64_t i = (int64_t)blockIdx.x * BLOCK + tid;
    const bool rv = i < m;
    UpdPartial wp = upd_empty();
    if (rv) {
        const double t = P.T[p * L + i];
        const double ei = pend ? eta_entry(a_prev[i], i, qp, aqp) : 0.0;
        const double a = tab_ftran_row(t, tau, ei, s_wp, [&](int s2) { return P.U[i * KW + s2]; });
        const int64_t bix = P.b_ixs[i];
        const double cb = P.c_B[i];
        double x = P.x_b[i];
        if (pend) {
            P.U[i * KW + tau] = ei;
            P.Wt[bix * KW + tau] = (i == qp) ? aqp : 0.0;  // r_tau.A_j of the basic columns
        }
        if (upd_x) {
            x = fma(s_x, ei, x);
            P.x_b[i] = x;
        }
        a_new[i] = a;
        // one row: the candidate whatever its key (first index on ties, as
        // k_update's argmin_better against the empty partial)
        wp.theta = ratio_key(P, x, a);
        wp.idx = i;
        wp.nonpos = !(a > P.piv_tol);
        wp.T = cb * a;
        wp.a_w = a;
        wp.cb_w = cb;
        wp.bix_w = bix;
    }
    wp = wave_upd_merge(wp);
    UpdPartial* red = reinterpret_cast<UpdPartial*>(smem + UpdLds<BLOCK>::red);
    int* s_last = reinterpret_cast<int*>(smem + UpdLds<BLOCK>::last);
    if (lane == 0) red[wave] = wp;
    __syncthreads();
    if (tid == 0) {
        UpdPartial w = red[0];
        for (int k = 1; k < WAVES; ++k) upd_merge(w, red[k]);
        if (P.split_tail) {
            upd_publish(P, blockIdx.x, w);
        } else {
            upd_publish(P, blockIdx.x, w);
            drain_vmem();
            *s_last = arrive_last(arrive_group(P.arrive, ARR_UPDATE), gridDim.x, blockIdx.x);
        }
    }
    if (P.split_tail) return;  // k_tail merges after the kernel boundary
    __syncthreads();
    if (!*s_last) return;
    update_tail<BLOCK>(P, st, p, min_e, it, smem, gridDim.x, &tpre);
}

// Row-sharded tail (last workgroup of k_update on this rank): the local
// leaving candidate with its scalars, the local sum T of c_B[i] * alpha_i, and
// the candidate's row of B^-1_new — recomputed from the old rows exactly as the
// stream wrote it — into rs_send for the ratio-test all-gather.  No global
// state changes: k_finalize_rs does them after the exchange.
template <int BLOCK>
__device__ void update_tail_rs(const Params& P, DevState* st, int64_t it, int par, const double* a_prev,
                               unsigned char* smem, int nparts) {
    const int tid = threadIdx.x;
    UpdPartial* red = reinterpret_cast<UpdPartial*>(smem + UpdLds<BLOCK>::red);
    const UpdPartial t = reduce_update_partials<BLOCK>(P, red, nparts);
    RsHeader* h = reinterpret_cast<RsHeader*>(P.rs_send);
    double* row = reinterpret_cast<double*>(P.rs_send + sizeof(RsHeader));
    const bool have = t.idx >= P.r0 && t.idx < P.r0 + P.mloc;
    if (have) {
        const int64_t i = t.idx, L2 = P.L >> 1;
        const double e = (it > 0) ? eta_entry(a_prev[i], i, st->q, st->aq) : 0.0;
        const dbl2* sr = reinterpret_cast<const dbl2*>((par ? P.B1 : P.B0) + (i - P.r0) * P.L);
        const dbl2* rb = reinterpret_cast<const dbl2*>(it > 0 ? P.rbuf : P.zeros);
        dbl2* out = reinterpret_cast<dbl2*>(row);
        for (int64_t k = tid; k < L2; k += BLOCK) {
            const dbl2 bv = sr[k], rv = rb[k];
            dbl2 nv;
            nv.x = fma(e, rv.x, bv.x);
            nv.y = fma(e, rv.y, bv.y);
            out[k] = nv;
        }
    }
    if (tid == 0) {
        h->theta = t.theta;
        h->idx = have ? t.idx : INT64_MAX;
        h->nonpos = t.nonpos;
        h->T = t.T;
        h->a_w = t.a_w;
        h->cb_w = t.cb_w;
        h->bix_w = t.bix_w;
    }
}

// Harris ratio test, second pass (SPX_RATIO_HARRIS; runs in k_tail, after
// the k_update boundary made every row's alpha and updated x_b visible).  The
// partials carry theta_max = min (max(x_b,0) + feas_tol) / alpha_i, the
// nonpos count and T; the leaving row is the largest alpha_i among rows with
// max(x_b_i,0) / alpha_i <= theta_max, first index on ties (the same rule as
// oracle/simplex_oracle.c ratio_harris).
template <int BLOCK>
__device__ void harris_tail(const Params& P, DevState* st, int64_t p, double min_e, int64_t it,
                            unsigned char* smem, int nparts) {
    constexpr int WAVES = BLOCK / 64;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    UpdPartial* red = reinterpret_cast<UpdPartial*>(smem + UpdLds<BLOCK>::red);
    const UpdPartial t = reduce_update_partials<BLOCK>(P, red, nparts);
    if (t.nonpos == P.m || t.idx < 0 || t.idx >= P.m) {
        if (tid == 0) {  // Unbounded (v4:319-322), as update_tail
            st->p = p;
            st->min_e = min_e;
            st->status = ST_UNBOUNDED;
        }
        return;
    }
    const double thmax = t.theta;
    const double* a_new = (it & 1) ? P.alpha0 : P.alpha1;
    double bv = INFINITY;  // -alpha of the best candidate
    int64_t bi = INT64_MAX;
    for (int64_t i = tid; i < P.m; i += BLOCK) {
        const double a = a_new[i];
        if (a > P.piv_tol) {
            const double xb = P.x_b[i];
            const double xc = xb > 0.0 ? xb : 0.0;
            if (xc / a <= thmax && argmin_better(-a, i, bv, bi)) { bv = -a; bi = i; }
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const double v = __shfl_xor(bv, off, 64);
        const int64_t i = __shfl_xor(bi, off, 64);
        if (argmin_better(v, i, bv, bi)) { bv = v; bi = i; }
    }
    __syncthreads();
    ArgMinEntry* wr = reinterpret_cast<ArgMinEntry*>(red);  // reuse the partial slots
    if (lane == 0) wr[wave] = ArgMinEntry{bv, bi};
    __syncthreads();
    if (tid != 0) return;
    ArgMinEntry w = wr[0];
    for (int k = 1; k < WAVES; ++k)
        if (argmin_better(wr[k].val, wr[k].idx, w.val, w.idx)) w = wr[k];
    const int64_t q = w.idx;  // exists: pass 1's winner satisfies the bound
    const double aq = a_new[q], cbq = P.c_B[q];
    pivot_bookkeeping(P, st, p, q, P.b_ixs[q], aq, y_scalar(t.T, aq, cbq, P.c[p]), P.devex ? *P.dvx_e : min_e, it);
}

// The pivot tail as its own one-workgroup launch (split_tail): the k_update
// workgroups stored their partials plainly and returned; the kernel boundary
// makes them visible here.
__global__ __launch_bounds__(1024) void k_tail(Params P, int nparts) {
    DevState* st = P.st;
    if (stopped(st)) return;  // also when k_update found the optimum
    __shared__ __attribute__((aligned(16))) unsigned char smem[UpdLds<1024>::bytes];
    double min_e = INFINITY;
    int64_t p = INT64_MAX;
    for (int g = 0; g < P.nin; ++g) {
        const ArgMinEntry e = P.price_in[g * P.pr_stride];
        if (argmin_better(e.val, e.idx, min_e, p)) { min_e = e.val; p = e.idx; }
    }
    const int64_t it = st->iter;
    if (P.row_shard)
        update_tail_rs<1024>(P, st, it, (int)(it & 1), (it & 1) ? P.alpha1 : P.alpha0, smem, nparts);
    else if (P.ratio == RATIO_HARRIS)
        harris_tail<1024>(P, st, p, min_e, it, smem, nparts);
    else
        update_tail<1024>(P, st, p, min_e, it, smem, nparts);
}

// Row-sharded pivot finalisation (one workgroup, after the ratio-test
// all-gather): global leaving row q = MINLOC over the ranks' headers
// (v4:324), Unbounded if every alpha_i <= 0 (v4:317-322), the pivot row into
// rbuf, s_y (v4:352-355; c_B_new.E_q evaluated from the gathered sum
// T = sum_i c_B[i] alpha_i as -(T - c_Bq alpha_q)/alpha_q + c_p (1/alpha_q - 1),
// since alpha is distributed), and the basis bookkeeping (v4:339-342).
__global__ __launch_bounds__(256) void k_finalize_rs(Params P) {
    DevState* st = P.st;
    if (stopped(st)) return;
    const int tid = threadIdx.x;
    double min_e = INFINITY;
    int64_t p = INT64_MAX;
    for (int g = 0; g < P.nin; ++g) {
        const ArgMinEntry e = P.price_in[g * P.pr_stride];
        if (argmin_better(e.val, e.idx, min_e, p)) { min_e = e.val; p = e.idx; }
    }
    // merge the ranks' ratio-test headers (rank order: deterministic T sum)
    double th = INFINITY, T = 0.0;
    int64_t q = INT64_MAX, nonpos = 0;
    int w = -1;
    for (int g = 0; g < P.nin; ++g) {
        const RsHeader* h = reinterpret_cast<const RsHeader*>(P.rs_recv + g * P.rs_stride);
        if (argmin_better(h->theta, h->idx, th, q)) { th = h->theta; q = h->idx; w = g; }
        nonpos += h->nonpos;
        T += h->T;
    }
    const int64_t it = st->iter;
    if (nonpos == P.m || q < 0 || q >= P.m || w < 0) {
        if (tid == 0) {
            st->p = p;
            st->min_e = min_e;
            st->status = ST_UNBOUNDED;
        }
        return;
    }
    const RsHeader* hw = reinterpret_cast<const RsHeader*>(P.rs_recv + w * P.rs_stride);
    const dbl2* row = reinterpret_cast<const dbl2*>(P.rs_recv + w * P.rs_stride + sizeof(RsHeader));
    dbl2* rb = reinterpret_cast<dbl2*>(P.rbuf);
    for (int64_t k = tid; k < (P.L >> 1); k += 256) rb[k] = row[k];
    if (tid == 0)
        pivot_bookkeeping(P, st, p, q, hw->bix_w, hw->a_w, y_scalar(T, hw->a_w, hw->cb_w, P.c[p]), min_e, it);
}

// ---------------------------------------------------------------------------
// Eta-window fold (spx_device.h): B_w += U[:, 0..nf) R, y_w += SY[0..nf) R for
// the nf = nw - 1 complete pivots of the window; the pending pivot stays
// pending as tau = 0.  A workgroup owns a 64-column stripe of B and a range of
// rows (spx_fold.h): its first tiles go in flight, wave 0 rebuilds R for the
// stripe (one column per lane: r_tau = Qrows[tau] + sum_{s<tau} Urows[tau][s]
// r_s) into LDS; then each wave updates 16-row x 64-column tiles with
// v_mfma_f64_16x16x4_f64 (K = the window, 4 pivots per step): the tile of B is
// the accumulator, U the A operand, R the B operand.  B is read and written
// once.  min_nw: fold only when nw >= min_nw (the loop asks for KW, a readback
// for 2).
// ---------------------------------------------------------------------------
template <int KW>
__global__ __launch_bounds__(FOLD_THREADS) void k_fold(Params P, int min_nw) {
    DevState* st = P.st;
    const int nw = st->nw;
    if (nw < min_nw || nw < 2) return;
    const int nf = nw - 1;
    __shared__ double Rl[KW][FOLD_RP];
    __shared__ double NT[KW][FOLD_NP<KW>];
    __shared__ int s_last;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int64_t L = P.L;
    const int64_t c0 = (int64_t)blockIdx.x * 64;
    int64_t i0, i1;
    fold_rows(P.m, i0, i1);
    // spx_fold.h: first tiles in flight, R rebuilt by all four waves, tiles
    // (the rebuild's operands are requested ahead of the first tiles and the
    // barriers wait for LDS only: the rebuild does not wait for the tiles)
    FoldRPre<KW> rpre;
    fold_r_load<KW>(P.Urows, P.Qrows, L, c0, rpre);
    FoldTilePre<KW> pre;
    fold_tile_first<KW>(P.B0, P.U, nf, L, c0, i0, i1, pre);
    fold_stage_N_pre<KW>(rpre, nf, NT);
    lds_barrier();
    if (tid < 256) fold_rebuild_R4<KW, FOLD_RP>(P.Qrows, NT, nf, L, c0, Rl, &rpre);
    lds_barrier();
    fold_tiles<KW, FOLD_RP>(P.B0, P.U, nf, L, c0, i0, i1, Rl, pre, true);
    if (wave == 0 && blockIdx.y == 0) {
        // y_w += SY R for this stripe (t ascending, the rebuild's R)
        double* y = st->y_buf ? P.y1 : P.y0;
        const int sl = fold_slot(lane);
        double d = 0.0;
#pragma unroll
        for (int t = 0; t < KW; ++t)
            if (t < nf) d = fma(P.SY[t], Rl[t][sl], d);
        y[c0 + lane] += d;
    } else if (wave == 1) {
        // xw = B_w b follows B_w: xw += U (R b), R b = Wt[n][0..nf); the rows
        // spread over every workgroup, one lane per row, t ascending
        const double* wb = P.Wt + P.n * KW;
        const int64_t nwg = (int64_t)gridDim.x * gridDim.y;
        const int64_t rpw = (P.m + nwg - 1) / nwg;
        const int64_t r0 = ((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * rpw;
        const int64_t r1 = (r0 + rpw < P.m) ? r0 + rpw : P.m;
        for (int64_t i = r0 + lane; i < r1; i += 64) {
            double d = 0.0;
#pragma unroll
            for (int t = 0; t < KW; ++t)
                if (t < nf) d = fma(P.U[i * KW + t], wb[t], d);
            P.xw[i] += d;
        }
    }
    __syncthreads();
    if (tid == 0) {
        s_last = arrive_last(arrive_group(P.arrive, ARR_FOLD), gridDim.x * gridDim.y,
                             blockIdx.y * gridDim.x + blockIdx.x);
    }
    __syncthreads();
    if (s_last && tid == 0) {
        P.SY[0] = P.SY[nf];
        st->nw = 1;
    }
}

// ---------------------------------------------------------------------------
// Deferred-state flush and readback kernels (off the hot loop)
// ---------------------------------------------------------------------------
// Applies the pending y and x_b updates of the last pivot (one workgroup).
__global__ __launch_bounds__(1024) void k_flush(Params P) {
    constexpr int BLOCK = 1024;
    DevState* st = P.st;
    const int tid = threadIdx.x;
    const int64_t it = st->iter, L = P.L, L2 = L >> 1, m = P.m;
    if (it == 0) return;
    // eta window: the host folded first, so at most the pending pivot is left
    // (nw <= 1) and the state has the explicit-B^-1 form with S = B_w
    const double* S = (SPX_INPLACE || P.win || !(it & 1)) ? P.B0 : P.B1;
    const double* r = P.row_shard ? P.rbuf : S + st->q * L;
    const bool upd_y = P.win ? st->nw == 1 : st->y_applied < it;
    const bool upd_x = st->xb_applied < it;
    if (upd_y) {
        const dbl2* yin = reinterpret_cast<const dbl2*>(st->y_buf ? P.y1 : P.y0);
        dbl2* yout = reinterpret_cast<dbl2*>(st->y_buf ? P.y0 : P.y1);
        const dbl2* r2 = reinterpret_cast<const dbl2*>(r);
        const double sy = P.win ? P.SY[0] : st->s_y;
        for (int64_t k = tid; k < L2; k += BLOCK) yout[k] = y_apply(sy, r2[k], yin[k]);
        // window tableau: dw = y_w A - c follows y_w; the pending pivot is
        // tau = 0 after the fold, so r.A_j = T_w[q, j]
        if (P.tab)
            for (int64_t j = tid; j < P.n; j += BLOCK) P.dw[j] = fma(sy, P.T[j * L + st->q], P.dw[j]);
    }
    if (upd_x) {
        // s_x exactly as k_update's row stream accumulates it (every wave alike)
        const dbl2* r2 = reinterpret_cast<const dbl2*>(r);
        const dbl2* b2 = reinterpret_cast<const dbl2*>(P.b);
        double sxa = 0.0;
        for (int64_t k = tid & 63; k < L2; k += 64) {
            sxa = fma(r2[k].x, b2[k].x, sxa);
            sxa = fma(r2[k].y, b2[k].y, sxa);
        }
        const double s_x = wave_sum(sxa);
        const double* a_prev = (it & 1) ? P.alpha1 : P.alpha0;
        const int64_t q = st->q;
        const double aq = st->aq;
        const int64_t i0 = P.row_shard ? P.r0 : 0, i1 = P.row_shard ? P.r0 + P.mloc : m;  // own rows
        for (int64_t i = i0 + tid; i < i1; i += BLOCK) P.x_b[i] = fma(s_x, eta_entry(a_prev[i], i, q, aq), P.x_b[i]);
    }
    __syncthreads();
    if (tid == 0) {
        if (upd_y) {
            st->y_buf ^= 1;
            st->y_applied = it;
            if (P.win) P.SY[0] = 0.0;  // y_w now includes the pending pivot
        }
        if (upd_x) st->xb_applied = it;
    }
}

// true B^-1 = S + E r^T into out (m x L row-major; row-sharded: own rows only,
// at their global positions)
__global__ void k_materialize(Params P, double* out) {
    const DevState* st = P.st;
    const int64_t it = st->iter;
    const bool rs = P.row_shard != 0;
    const double* S = rs ? ((it & 1) ? P.B1 : P.B0) : ((SPX_INPLACE || P.win || !(it & 1)) ? P.B0 : P.B1);
    const double* r = rs ? P.rbuf : S + st->q * P.L;
    const double* a_prev = (it & 1) ? P.alpha1 : P.alpha0;
    const int64_t q = st->q;
    const double aq = st->aq;
    const int64_t r0 = rs ? P.r0 : 0;
    const int64_t total = (rs ? P.mloc : P.m) * P.L;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t li = t / P.L, k = t - li * P.L, i = r0 + li;
        out[r0 * P.L + t] = (it > 0) ? fma(eta_entry(a_prev[i], i, q, aq), r[k], S[t]) : S[t];
    }
}

// e_j for every column from the current (flushed) y, one wave per column
__global__ __launch_bounds__(256) void k_reduced_costs(Params P, double* e) {
    const int lane = threadIdx.x & 63;
    const int64_t L2 = P.L >> 1;
    const dbl2* y2 = reinterpret_cast<const dbl2*>(P.st->y_buf ? P.y1 : P.y0);
    for (int64_t j = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; j < P.n;
         j += ((int64_t)gridDim.x * blockDim.x) >> 6) {
        const dbl2* col = reinterpret_cast<const dbl2*>(P.A + j * P.L);
        double a0 = 0.0, a1 = 0.0;
        for (int64_t k = lane; k < L2; k += 64) {
            const dbl2 v = col[k], w = y2[k];
            a0 = fma(v.x, w.x, a0);
            a1 = fma(v.y, w.y, a1);
        }
        const double s = wave_sum(a0 + a1) - P.c[j];
        if (lane == 0) e[j] = s;
    }
}

// z = c_B . x_b (v4:365), from the flushed x_b
__global__ __launch_bounds__(256) void k_objective(Params P) {
    __shared__ double sa[4];
    double s = 0.0;
    for (int64_t i = threadIdx.x; i < P.m; i += 256) s = fma(P.c_B[i], P.x_b[i], s);
    s = block_sum<256>(s, sa);
    if (threadIdx.x == 0) P.st->z = s;
}

// ---------------------------------------------------------------------------
// Setup kernels
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
__device__ __forceinline__ double uniform01(uint64_t seed, uint64_t stream, uint64_t idx) {
    const uint64_t key = (seed * 0x9E3779B97F4A7C15ULL) ^ (stream << 56) ^ idx;
    return (double)(splitmix64(key) >> 11) * 0x1.0p-53;
}

__global__ void k_generate(double* A, double* b, double* c, int64_t m, int64_t n, int64_t L,
                           uint64_t seed) {
    const int64_t ns = n - m;
    const int64_t total = L * n;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t j = t / L, i = t - j * L;
        double v = 0.0;
        if (i < m) v = (j < ns) ? uniform01(seed, 1, (uint64_t)(i + j * m)) : ((i == j - ns) ? 1.0 : 0.0);
        A[t] = v;
        if (j == 0) b[i] = (i < m) ? ((double)ns / 4.0) * (1.0 + uniform01(seed, 2, (uint64_t)i)) : 0.0;
        if (i == 0) c[j] = (j < ns) ? uniform01(seed, 3, (uint64_t)j) : 0.0;
    }
}

// slack basis (v4:268-277 with the intended semantics); vectors zeroed by the host
__global__ void k_reset(Params P) {
    const int64_t m = P.m, n = P.n, L = P.L, ns = P.ns;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (int64_t li = t0; li < P.mloc; li += stride) P.B0[li * L + P.r0 + li] = 1.0;  // init_I (v4:182-188)
    for (int64_t i = t0; i < m; i += stride) {
        P.c_B[i] = P.c[ns + i];
        P.x_b[i] = P.b[i];
        P.y0[i] = P.c[ns + i];
        P.b_ixs[i] = ns + i;
        if (P.xw) P.xw[i] = P.b[i];  // B_w = I
    }
    for (int64_t k = t0; k < ARR_GROUPS * ARR_LINES * ARR_STRIDE; k += stride) P.arrive[k] = 0u;
    if (P.trec && t0 == 0) P.trec->fresh = 0;
    if (P.upd_tag)
        for (int64_t k = t0; k < UPD_WORDS * P.upd_cap; k += stride) P.upd_tag[k] = 0ull;
    if (P.price_tag)
        for (int64_t k = t0; k < PRICE_WORDS * P.price_cap; k += stride) P.price_tag[k] = 0ull;
    for (int64_t j = t0; j < n; j += stride) {
        if (P.W) P.W[j] = 1.0;  // Devex reference framework
        int32_t pos = -1;
        if (j < ns && j >= P.s_lo && j < P.s_hi) {
            pos = (int32_t)(j - P.s_lo);
            P.nb_list[pos] = (int32_t)j;
        }
        P.nb_pos[j] = pos;
    }
    if (t0 == 0) {
        DevState* st = P.st;
        st->status = ST_RUNNING;
        st->nb_count = (int32_t)(P.s_hi - P.s_lo);
        st->iter = 0;
        st->limit = 0;
        st->p = -1;
        st->q = -1;
        st->min_e = 0.0;
        st->z = 0.0;
        st->aq = 1.0;
        st->s_y = 0.0;
        st->y_applied = 0;
        st->xb_applied = 0;
        st->y_buf = 0;
        st->nw = 0;
        st->leave = -1;
        st->wp = 1.0;
        st->uncovered = 0u;
        st->mbox_epoch = st->mbox_epoch + 1u;  // (every rank resets alike)
    }
}

// ---------------------------------------------------------------------------
// Host-side launchers
// ---------------------------------------------------------------------------
template <int BLOCK, bool LDS_Y, int WM, bool TK = false>
static hipError_t launch_price_t(const Params& P, int grid, size_t lds, hipStream_t s, hipEvent_t e0,
                                 hipEvent_t e1) {
    if (e0 || e1) {
        hipExtLaunchKernelGGL((k_price<BLOCK, LDS_Y, WM, TK>), dim3(grid), dim3(BLOCK), (uint32_t)lds, s, e0, e1, 0, P);
    } else {
        hipLaunchKernelGGL((k_price<BLOCK, LDS_Y, WM, TK>), dim3(grid), dim3(BLOCK), lds, s, P);
    }
    return hipGetLastError();
}

template <int BLOCK, bool LDS_Y, int WM, bool TK = false>
static hipError_t prep_price_t(size_t lds, int* blocks_per_cu) {
    hipError_t e = hipSuccess;
    if (lds > 65536) {
        e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_price<BLOCK, LDS_Y, WM, TK>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, k_price<BLOCK, LDS_Y, WM, TK>, BLOCK, lds);
}

// (lds_y, wm) variants: (1,0) (0,0) explicit B^-1; (1,1) (1,2) (0,2) eta window
template <int BLOCK>
static hipError_t price_dispatch(const PriceCfg& c, const Params* P, hipStream_t s, hipEvent_t e0, hipEvent_t e1,
                                 int* blocks_per_cu) {
#define SPX_PV(LY, WM)                                                                  \
    return P ? launch_price_t<BLOCK, LY, WM>(*P, c.grid, c.lds_bytes, s, e0, e1)        \
             : prep_price_t<BLOCK, LY, WM>(c.lds_bytes, blocks_per_cu)
    if (c.wm == 0) {
        if (c.lds_y) SPX_PV(true, 0);
        SPX_PV(false, 0);
    }
    if (c.wm == 1 && c.lds_y) {
        if (c.tk) return P ? launch_price_t<BLOCK, true, 1, true>(*P, c.grid, c.lds_bytes, s, e0, e1)
                           : prep_price_t<BLOCK, true, 1, true>(c.lds_bytes, blocks_per_cu);
        SPX_PV(true, 1);
    }
    if (c.wm == 2) {
        if (c.lds_y) SPX_PV(true, 2);
        SPX_PV(false, 2);
    }
    if (c.wm == 3) SPX_PV(false, 3);
    if (c.wm == 4 && c.lds_y) SPX_PV(true, 4);
    if (c.wm == 5) {
        if (c.lds_y) SPX_PV(true, 5);
        SPX_PV(false, 5);
    }
#undef SPX_PV
    return hipErrorInvalidValue;
}

hipError_t price_prepare(const PriceCfg& c, int* blocks_per_cu) {
    switch (c.block) {
        case 256: return price_dispatch<256>(c, nullptr, nullptr, nullptr, nullptr, blocks_per_cu);
        case 512: return price_dispatch<512>(c, nullptr, nullptr, nullptr, nullptr, blocks_per_cu);
        case 1024: return price_dispatch<1024>(c, nullptr, nullptr, nullptr, nullptr, blocks_per_cu);
    }
    return hipErrorInvalidValue;
}

hipError_t launch_price(const Params& P, const PriceCfg& c, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
    switch (c.block) {
        case 256: return price_dispatch<256>(c, &P, s, e0, e1, nullptr);
        case 512: return price_dispatch<512>(c, &P, s, e0, e1, nullptr);
        case 1024: return price_dispatch<1024>(c, &P, s, e0, e1, nullptr);
    }
    return hipErrorInvalidValue;
}

template <int BLOCK, int R, bool RS, bool WIN, int BNT = 1, bool BC = false>
static hipError_t launch_update_k(const Params& P, int grid, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
    const size_t lds = UpdLds<BLOCK>::bytes +
                       ((WIN && BC) ? (size_t)(P.L < BC_APC ? P.L : BC_APC) * 8
                                    : ((WIN && SPX_WIN_APLDS && P.L * 8 <= 65536) ? (size_t)P.L * 8 : 0)) +
                       ((!WIN && !RS && upd_xlds(P)) ? (size_t)P.L * 24 : 0);
    if (lds > 65536) {  // once per instantiation and device (idempotent; not a stream operation)
        static std::atomic<uint64_t> raised{0};
        int dev = 0;
        const hipError_t ed = hipGetDevice(&dev);
        if (ed != hipSuccess) return ed;
        const uint64_t bit = 1ull << (dev & 63);
        if (!(raised.load(std::memory_order_acquire) & bit)) {
            const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_update<BLOCK, R, RS, WIN, BNT, BC>),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, 100 * 1024);
            if (e != hipSuccess) return e;
            raised.fetch_or(bit, std::memory_order_release);
        }
    }
    if (e0 || e1) {
        hipExtLaunchKernelGGL((k_update<BLOCK, R, RS, WIN, BNT, BC>), dim3(grid), dim3(BLOCK), (uint32_t)lds, s, e0, e1, 0,
                              P);
    } else {
        hipLaunchKernelGGL((k_update<BLOCK, R, RS, WIN, BNT, BC>), dim3(grid), dim3(BLOCK), lds, s, P);
    }
    return hipGetLastError();
}

// grid: the one-row grid's workgroups (= partial slots); RPW rows per wave
// take ceil(grid / RPW) workgroups
template <int BLOCK, bool DEFER, int RPW, bool SEF = false>
static hipError_t launch_ftran_bc_t(const Params& P, int grid, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
    const size_t red = RPW == 1 ? UpdLds<BLOCK>::bytes : sizeof(UpdPartial) * (BLOCK / 64) * RPW + 16;
    const size_t lds = red + (size_t)(P.L < BC_APC ? P.L : BC_APC) * 8;
    const int g = (grid + RPW - 1) / RPW;
    if (lds > 65536) {
        const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_ftran_bc<BLOCK, DEFER, RPW, SEF>),
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, 100 * 1024);
        if (e != hipSuccess) return e;
    }
    if (e0 || e1)
        hipExtLaunchKernelGGL((k_ftran_bc<BLOCK, DEFER, RPW, SEF>), dim3(g), dim3(BLOCK), (uint32_t)lds, s, e0, e1, 0, P);
    else
        hipLaunchKernelGGL((k_ftran_bc<BLOCK, DEFER, RPW, SEF>), dim3(g), dim3(BLOCK), lds, s, P);
    return hipGetLastError();
}

// deferred ratio-test tail: its own instantiation (no tail code, and the
// tail's registers stay out of the hand-off kernel); rows per wave (the
// deferred form only; bc_entry = SPX_FTRAN_RPW, UpdateCfg)
template <int BLOCK>
static hipError_t launch_ftran_bc(const Params& P, int grid, int rpw, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
    if (!P.defer_tail) return launch_ftran_bc_t<BLOCK, false, 1>(P, grid, s, e0, e1);
    if constexpr (BLOCK == 512) {
        if (rpw == 2) return launch_ftran_bc_t<BLOCK, true, 2>(P, grid, s, e0, e1);
        if (rpw == 4) return launch_ftran_bc_t<BLOCK, true, 4>(P, grid, s, e0, e1);
        if (P.se_fused) return launch_ftran_bc_t<BLOCK, true, 1, true>(P, grid, s, e0, e1);
    }
    return launch_ftran_bc_t<BLOCK, true, 1>(P, grid, s, e0, e1);
}

template <int BLOCK, int R>
static hipError_t launch_update_t(const Params& P, int grid, int bc_entry, hipStream_t s, hipEvent_t e0,
                                  hipEvent_t e1) {
    if (P.row_shard) return launch_update_k<BLOCK, R, true, false>(P, grid, s, e0, e1);
    if (!P.win) return launch_update_k<BLOCK, R, false, false>(P, grid, s, e0, e1);
    // B_w loads: default policy while B_w fits the Infinity Cache beside the
    // window state (spx_common.h SPX_NT_BWIN), non-temporal beyond
    if (P.bc) {  // compact FTRAN
        if (R == 1 && bc_entry) return launch_ftran_bc<BLOCK>(P, grid, bc_entry, s, e0, e1);
        return launch_update_k<BLOCK, R, false, true, 0, true>(P, grid, s, e0, e1);
    }
    if (win_b_cached(P)) return launch_update_k<BLOCK, R, false, true, 0>(P, grid, s, e0, e1);
    return launch_update_k<BLOCK, R, false, true, 1>(P, grid, s, e0, e1);
}

hipError_t launch_cfold(const Params& P, int min_nw, int cus, hipStream_t s);
hipError_t launch_fold(const Params& P, int min_nw, int cus, hipStream_t s) {
    if (P.bc && P.cfold) return launch_cfold(P, min_nw, cus, s);  // the listed columns only
    if (P.tab) {  // T_w and dw first: k_fold resets the window
        const hipError_t e = launch_tab_fold(P, min_nw, cus, s);
        if (e != hipSuccess) return e;
        // A[:, n-m:] = I: B_w is T_w's slack block and the tableau fold has
        // updated y_w and xw too (and reset the window); B_w itself is rebuilt
        // from T_w only for readbacks (launch_tab_binv)
        if (P.tab_slack) return hipSuccess;
    }
    const int nx = (int)(P.L / 64);
    const dim3 grid((unsigned)nx, (unsigned)fold_grid_y(P.m, nx, cus));
    switch (P.win) {
        case 8: hipLaunchKernelGGL(k_fold<8>, grid, dim3(FOLD_THREADS), 0, s, P, min_nw); break;
        case 16: hipLaunchKernelGGL(k_fold<16>, grid, dim3(FOLD_THREADS), 0, s, P, min_nw); break;
        case 32: hipLaunchKernelGGL(k_fold<32>, grid, dim3(FOLD_THREADS), 0, s, P, min_nw); break;
        case 64: hipLaunchKernelGGL(k_fold<64>, grid, dim3(FOLD_THREADS), 0, s, P, min_nw); break;
        default: return hipErrorInvalidValue;
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return launch_compact(P, s);  // the compact FTRAN operand follows B_w
}



hipError_t launch_tail(const Params& P, int nparts, hipStream_t s) {
    hipLaunchKernelGGL(k_tail, dim3(1), dim3(1024), 0, s, P, nparts);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Compact FTRAN operand (Params::bc): after every fold (and reset or
// reinversion) the rows that have left join the column list in ascending
// order (k_bc_list, one workgroup), then every row of B_w is gathered onto
// those columns (k_bc_gather).  The dense B_w stays the master copy.
// ---------------------------------------------------------------------------
// min_nw > 0 (the compact fold): only when that fold runs (k_fold's test),
// recording S and the pitch before the append in bc_n[3] / bc_n[4]
__global__ __launch_bounds__(1024) void k_bc_list(Params P, int min_nw) {
    __shared__ int s_w[16];
    __shared__ int s_base;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (min_nw > 0) {
        const int nw = P.st->nw;
        if (nw < min_nw || nw < 2) return;
    }
    if (tid == 0) {
        s_base = P.bc_n[0];
        P.bc_n[3] = P.bc_n[0];
        P.bc_n[4] = P.bc_n[1];
    }
    __syncthreads();
    for (int64_t k0 = 0; k0 < P.m; k0 += 1024) {
        const int64_t k = k0 + tid;
        const bool nu = k < P.m && P.rleft[k] != 0 && P.rmap[k] < 0;
        const uint64_t bal = __ballot(nu);
        const int pre = __popcll(bal & ((1ull << lane) - 1ull));
        if (lane == 0) s_w[wave] = __popcll(bal);
        __syncthreads();
        int off = s_base, tot = 0;
        for (int w = 0; w < 16; ++w) {
            if (w < wave) off += s_w[w];
            tot += s_w[w];
        }
        if (nu) {
            P.rmap[k] = off + pre;
            P.rlist[off + pre] = (int32_t)k;
        }
        __syncthreads();
        if (tid == 0) s_base += tot;
        __syncthreads();
    }
    if (tid == 0) {
        P.bc_n[0] = s_base;
        // row pitch of bc: S rounded up to 64 doubles (512 B).  Rows then lie
        // back to back (m x pitch, contiguous), so a wave's rows spread over
        // the HBM channels; at the full pitch L every row started a multiple
        // of L * 8 bytes apart
        P.bc_n[1] = s_base > 0 ? ((s_base + 63) / 64) * 64 : 64;
    }
}
constexpr int BC_ROWS = 4;  // rows per k_bc_gather workgroup
__global__ __launch_bounds__(256) void k_bc_gather(Params P) {
    const int S = P.bc_n[0];
    const int64_t L = P.L, ldc = P.bc_n[1];
    double* const bc = bc_buf(P, P.bc_n[2]);
    for (int r = 0; r < BC_ROWS; ++r) {
        const int64_t i = (int64_t)blockIdx.x * BC_ROWS + r;
        if (i >= P.m) break;
        for (int c = threadIdx.x; c < S; c += 256) bc[i * ldc + c] = P.B0[i * L + P.rlist[c]];
    }
}
// the whole operand from the dense B_w (reset, reinversion, warm start; and
// after a dense fold, SPX_DENSE_FOLD=1)
hipError_t launch_compact(const Params& P, hipStream_t s) {
    if (!P.bc) return hipSuccess;
    hipLaunchKernelGGL(k_bc_list, dim3(1), dim3(1024), 0, s, P, 0);
    hipLaunchKernelGGL(k_bc_gather, dim3((unsigned)((P.m + BC_ROWS - 1) / BC_ROWS)), dim3(256), 0, s, P);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Compact fold (Params::bc): the eta-window fold of k_fold
// restricted to B_w's non-unit columns.  A column of B_w outside the list is
// e_k and stays e_k (every r_t has an exact 0 there: B_w[q_t, k] = 0 for the
// unit column k != q_t, and the window's leaving rows q_t join the list
// first, k_bc_list), so only the m x S' listed entries change -- the dense
// fold rewrites all m x L of them.  Per 64-column group of the new list:
//   R: r_t = Qrows[t][k_c] + sum_{s<t} Urows[t][s] r_s (Qrows: the base rows
//      k_price staged), by one wave, one lane per column, the s terms of each
//      r_t in ascending order with the fold's zero coefficients -- the fma
//      sequence of fold_rebuild_R4, so the bits of k_fold's R;
//   tiles: the fold's MFMA tiles (fold_tile_take, v_mfma_f64_16x16x4f64, the
//      same K order), rows read from the active buffer at the old pitch
//      (columns the window added read as e_k), written to the other buffer
//      at the new pitch, and the same values scattered into the dense B_w at
//      (i, rlist[c]) -- so the dense B_w is k_fold's, entry for entry, and
//      the operand is what k_bc_gather would gather from it;
//   y_w += SY R over the group's columns, xw += U (R b) as k_fold.
// The last workgroup resets the window and flips the active buffer.  The
// grid is fixed (host-side, captured in graphs): workgroup b takes group
// b % ng and row range b / ng of the floor(grid / ng) ranges; the rest only
// count in.
// ---------------------------------------------------------------------------
template <int KW>
__device__ __forceinline__ void cfold_tile_issue(const double* Bo, int64_t ldo, int S0, const double* U, int64_t c0,
                                                 int64_t r0, int64_t i1, FoldTilePre<KW>& t) {
    const int lane = threadIdx.x & 63;
    const int kr = lane >> 4, cl = lane & 15;
    const int64_t ilast = i1 > 0 ? i1 - 1 : 0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int64_t i0r = r0 + kr + 4 * r;
        const int64_t i = i0r < ilast ? i0r : ilast;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int64_t c = c0 + 32 * h + 2 * cl;  // even; the pair lies inside the old pitch when c < S0
            t.b[r][h] = *reinterpret_cast<const fdbl2*>(&Bo[i * ldo + (c < S0 ? c : 0)]);
        }
    }
#pragma unroll
    for (int j = 0; j < KW / 8; ++j) {
        const int e = 128 * j + 2 * lane;
        const int64_t ia0 = r0 + e / KW;
        const int64_t ia = ia0 < ilast ? ia0 : ilast;
        t.u[j] = *reinterpret_cast<const fdbl2*>(&U[ia * KW + e % KW]);
    }
}
// the old entries of the tile's columns, or e_k for the columns past S0
// (rlv: rlist of this lane's four columns, -1 past S)
__device__ __forceinline__ double cfold_old(double v, int64_t i, int64_t c, int S0, int k) {
    return c < S0 ? v : (k == i ? 1.0 : 0.0);
}

template <int KW>
__global__ __launch_bounds__(FOLD_THREADS) void k_cfold(Params P, int min_nw) {
    static_assert(SPX_FOLD_ULDS, "the compact fold stages U through LDS");
    DevState* st = P.st;
    // (the list's shape read beside the window count: one round trip)
    const int nw = st->nw;
    const int S = P.bc_n[0], sel = P.bc_n[2], S0 = P.bc_n[3];
    const int64_t ldn = P.bc_n[1], ldo = P.bc_n[4] > 0 ? P.bc_n[4] : 64;
    asm volatile("" ::"s"(S), "s"(sel), "s"(S0), "s"(ldn), "s"(ldo));  // (kept ahead of the branch)
    if (nw < min_nw || nw < 2) return;
    const int nf = nw - 1;
    constexpr int KS = KW / 4;
    __shared__ double Rl[KW][FOLD_RP];
    __shared__ double NT[KW][FOLD_NP<KW>];
    __shared__ double Ush[FOLD_THREADS / 64][16][FOLD_UP<KW>];
    __shared__ int s_last;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int kr = lane >> 4, cl = lane & 15;
    const int64_t L = P.L, m = P.m;
    const double* const Bo = bc_buf(P, sel);
    double* const Bn = bc_buf(P, sel ^ 1);
    const int ng = (int)(ldn / 64);
    const int nper = (int)gridDim.x / ng;  // row ranges per group
    const int g = (int)blockIdx.x % ng, yr = (int)blockIdx.x / ng;
    const bool work = yr < nper;
    unsigned long long* const fst =
        (P.stamps && tid == 0 && blockIdx.x < 1024) ? P.stamps + STAMP_FOLD + STAMP_FOLD_PER * (int64_t)blockIdx.x
                                                    : nullptr;
    // (lane 0 of every wave: the y / xw waves' own end stamps, slots 7 / 6)
    unsigned long long* const fsx =
        (P.stamps && lane == 0 && blockIdx.x < 1024) ? P.stamps + STAMP_FOLD + STAMP_FOLD_PER * (int64_t)blockIdx.x
                                                     : nullptr;
    if (fst) fst[0] = rtime();
    const int64_t c0 = (int64_t)g * 64;
    const int64_t per = ((m + nper - 1) / nper + 15) / 16 * 16;
    const int64_t i0 = work ? (int64_t)yr * per : m;
    const int64_t i1 = (i0 + per < m) ? i0 + per : m;
    if (work && i0 < m) {
        const int64_t cc = c0 + lane;
        // (the list entry of this lane's column, for y_w: read unconditionally
        // and pinned below, so the compiler cannot turn it into a guarded
        // load waited for on the spot)
        int kcl = P.rlist[cc < L ? cc : L - 1];
        // R, one lane per row t and eight columns per wave (columns
        // c0 + 8 wave + j): lane t holds N[t][s] = Urows[t][s] (0 unless
        // s < t < nf) and r_t of each column; step s hands r_s (final after
        // step s - 1) from lane s to the lanes t > s, which take
        // fma(N[t][s], r_s, r_t) -- every r_t its s terms in ascending s,
        // fold_rebuild_R4's fma sequence, so its bits
        constexpr int CPW = 64 / (FOLD_THREADS / 64);
        const int64_t cw0 = c0 + CPW * wave;
        const bool rows = cw0 < S;  // (wave-uniform) any listed column
        const int tl = lane < KW ? lane : KW - 1;
        double rt[CPW];
        // every operand read unconditionally (clamped): the coefficients
        // (staged transposed into LDS, NT[s][t] = N[t][s], as k_fold), the
        // list entries, then the base-row entries, which wait only for the
        // first two (vmcnt retires in issue order)
        FoldRPre<KW> rpre;
#pragma unroll
        for (int j = 0; j < FoldRPre<KW>::NPT; ++j) {
            const int k = tid + j * FOLD_THREADS;
            rpre.n[j] = P.Urows[k < KW * KW ? k : KW * KW - 1];
        }
        int kl[CPW];
#pragma unroll
        for (int j = 0; j < CPW; ++j) kl[j] = P.rlist[cw0 + j < L ? cw0 + j : L - 1];
#pragma unroll
        for (int j = 0; j < CPW; ++j) {
            const int k = (unsigned)kl[j] < (unsigned)L ? kl[j] : 0;
            rt[j] = P.Qrows[(int64_t)tl * L + k];
        }
        // the list entries of this lane's tile columns (unit entries past S0)
        int rk[4];
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int x = 0; x < 2; ++x) {
                const int64_t c = c0 + 32 * h + 2 * cl + x;
                rk[2 * h + x] = c < S ? P.rlist[c] : -1;
            }
        // the wave's first tile in flight during the rebuild
        const int64_t step = 16 * (int64_t)(FOLD_THREADS / 64);
        int64_t r0 = i0 + 16 * wave;
        FoldTilePre<KW> cur;
        // (unconditional: rows clamped into the range, a branch here made
        // the compiler wait for everything before the rebuild)
        cfold_tile_issue<KW>(Bo, ldo, S0, P.U, c0, r0, i1, cur);
        fold_stage_N_pre<KW>(rpre, nf, NT);
        lds_barrier();
        // (the pins: every read above is issued before anything waits)
#pragma unroll
        for (int j = 0; j < CPW; ++j) {
            asm volatile("" : "+v"(rt[j]));
            rt[j] = (lane < nf && cw0 + j < S) ? rt[j] : 0.0;
        }
        asm volatile("" : "+v"(kcl));
        if (fst) fst[1] = rtime();
        if (rows) {
#pragma unroll
            for (int s = 0; s < KW - 1; ++s) {
                const double co = NT[s][tl];
                // one exec mask per step for the wave's columns
                double rs[CPW];
#pragma unroll
                for (int j = 0; j < CPW; ++j) rs[j] = readlane_d(rt[j], s);
                if (lane > s) {
#pragma unroll
                    for (int j = 0; j < CPW; ++j) rt[j] = fma(co, rs[j], rt[j]);
                }
            }
        } else {
#pragma unroll
            for (int j = 0; j < CPW; ++j) rt[j] = 0.0;
        }
        if (lane < KW) {
#pragma unroll
            for (int j = 0; j < CPW; ++j) Rl[lane][fold_slot(CPW * wave + j)] = rt[j];
        }
        lds_barrier();
        if (fst) fst[2] = rtime();
        // tiles (fold_tiles' k-step order), the first one already in flight
        double (*Us)[FOLD_UP<KW>] = Ush[wave];
        for (; r0 < i1; r0 += step) {
            dbl4 acc[4];
            double af[KS];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int64_t i = r0 + kr + 4 * r;
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int64_t c = c0 + 32 * h + 2 * cl;
                    cur.b[r][h].x = cfold_old(cur.b[r][h].x, i, c, S0, rk[2 * h]);
                    cur.b[r][h].y = cfold_old(cur.b[r][h].y, i, c + 1, S0, rk[2 * h + 1]);
                }
            }
            fold_tile_take<KW>(cur, r0, i1, nf, acc, af, Us);
            if (r0 + step < i1) cfold_tile_issue<KW>(Bo, ldo, S0, P.U, c0, r0 + step, i1, cur);
            double rf[2][4];
            double uf[2];
            uf[0] = Us[cl][kr];
#pragma unroll
            for (int jb = 0; jb < 4; ++jb) rf[0][jb] = Rl[kr][16 * jb + cl];
#pragma unroll
            for (int s2 = 0; s2 < KS; ++s2) {
                if (s2 + 1 < KS) {
                    uf[(s2 + 1) & 1] = Us[cl][4 * (s2 + 1) + kr];
#pragma unroll
                    for (int jb = 0; jb < 4; ++jb) rf[(s2 + 1) & 1][jb] = Rl[4 * (s2 + 1) + kr][16 * jb + cl];
                }
                const double a = uf[s2 & 1];
#pragma unroll
                for (int jb = 0; jb < 4; ++jb)
                    acc[jb] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, rf[s2 & 1][jb], acc[jb], 0, 0, 0);
                __builtin_amdgcn_sched_barrier(0);
            }
            // the new operand rows (whole pitch: zeros past S) and the dense B_w
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int64_t i = r0 + kr + 4 * r;
                if (i < i1) {
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        fdbl2 v;
                        v.x = acc[2 * h][r];
                        v.y = acc[2 * h + 1][r];
                        *reinterpret_cast<fdbl2*>(&Bn[i * ldn + c0 + 32 * h + 2 * cl]) = v;
                        if (rk[2 * h] >= 0) P.B0[i * L + rk[2 * h]] = v.x;
                        if (rk[2 * h + 1] >= 0) P.B0[i * L + rk[2 * h + 1]] = v.y;
                    }
                }
            }
        }
        if (fst) fst[3] = rtime();
        if (wave == 0 && yr == 0) {
            // y_w += SY R for the group's columns (k_fold's sum, t ascending;
            // the terms past nf dropped by a select). SY[t] is read once by
            // lane t and handed on by readlane, so it is read before the
            // column guard: every lane must hold its entry.
            double syl = P.SY[lane < KW ? lane : KW - 1];
            asm volatile("" : "+v"(syl));  // (so the read cannot sink under the guard)
            if (cc < S) {
                double* y = st->y_buf ? P.y1 : P.y0;
                const int sl = fold_slot(lane);
                double d = 0.0;
#pragma unroll
                for (int t = 0; t < KW; ++t) {
                    const double v = fma(readlane_d(syl, t), Rl[t][sl], d);
                    d = t < nf ? v : d;
                }
                y[kcl] += d;
                if (fsx) fsx[7] = rtime();
            }
        }
    }
    if (wave == FOLD_THREADS / 64 - 1) {
        // xw += U (R b), R b = Wt[n][0..nf): the rows spread over every
        // workgroup, one lane per row, t ascending (k_fold's); the last
        // wave, which has tiles only when a range passes 112 rows
        // (R b: lane t holds entry t, handed to every row by readlane)
        double wbl = P.Wt[P.n * KW + (lane < KW ? lane : KW - 1)];
        asm volatile("" : "+v"(wbl));  // (read by every lane, not sunk into the row loop)
        const int64_t nwg = (int64_t)gridDim.x;
        const int64_t rpw = (m + nwg - 1) / nwg;
        const int64_t r0 = (int64_t)blockIdx.x * rpw;
        const int64_t r1 = (r0 + rpw < m) ? r0 + rpw : m;
        for (int64_t i = r0 + lane; i < r1; i += 64) {
            double u[KW];
#pragma unroll
            for (int t2 = 0; t2 < KW / 2; ++t2) {
                const fdbl2 v = *reinterpret_cast<const fdbl2*>(&P.U[i * KW + 2 * t2]);
                u[2 * t2] = v.x;
                u[2 * t2 + 1] = v.y;
            }
            double d = 0.0;
#pragma unroll
            for (int t = 0; t < KW; ++t) {
                const double v = fma(u[t], readlane_d(wbl, t), d);
                d = t < nf ? v : d;
            }
            P.xw[i] += d;
        }
        if (fsx) fsx[6] = rtime();
    }
    __syncthreads();
    if (fst) fst[4] = rtime();
    if (tid == 0) s_last = arrive_last(arrive_group(P.arrive, ARR_FOLD), gridDim.x, blockIdx.x);
    __syncthreads();
    if (fst) fst[5] = rtime();
    if (s_last && tid == 0) {
        P.SY[0] = P.SY[nf];
        P.bc_n[2] = sel ^ 1;
        st->nw = 1;
    }
}

// compact fold: k_bc_list (the window's leaving rows join the list) then
// k_cfold over the listed columns only (P.bc, one workgroup per CU)
hipError_t launch_cfold(const Params& P, int min_nw, int cus, hipStream_t s) {
    hipLaunchKernelGGL(k_bc_list, dim3(1), dim3(1024), 0, s, P, min_nw);
    // every column group of the list needs a workgroup (m > 16,384: more
    // groups than CUs)
    const int64_t ngmax = P.L / 64;
    const int64_t nc = cus > 0 ? cus : 256;
    const dim3 grid((unsigned)(nc > ngmax ? nc : ngmax));
    switch (P.win) {
        case 8: hipLaunchKernelGGL(k_cfold<8>, grid, dim3(FOLD_THREADS), 0, s, P, min_nw); break;
        case 16: hipLaunchKernelGGL(k_cfold<16>, grid, dim3(FOLD_THREADS), 0, s, P, min_nw); break;
        case 32: hipLaunchKernelGGL(k_cfold<32>, grid, dim3(FOLD_THREADS), 0, s, P, min_nw); break;
        case 64: hipLaunchKernelGGL(k_cfold<64>, grid, dim3(FOLD_THREADS), 0, s, P, min_nw); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// MINLOC exchange through peer mailboxes (spx_mbox_attach): the replacement
// for the all-gather of the candidate records (v4:294-302 runs the argmin on
// one device; across ranks every rank needs every record).  One workgroup:
// this rank's record (price_out, written by k_price) is stored as tagged
// words into slot [seq & 1][rank] of every rank's mailbox, then the nin
// slots of this rank's own mailbox are polled until every word carries seq
// and unpacked into price_in, which k_update reads as it reads the RCCL
// all-gather's output.  Each 8-byte word is stored and loaded whole, so a
// record is complete when all its tags match, with no fence or flag.  Two
// parities suffice: a rank reaches exchange seq + 2 only after every rank's
// record of seq + 1, which each stored after consuming seq.  System-scope
// stores and loads (the mailboxes are fine-grained, mapped over xGMI on other
// devices).  A rank that polls for MBOX_TIMEOUT_TICKS without seeing a peer
// stops with ST_HANDOFF_TIMEOUT, and its later exchanges only send.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_exchange(Params P) {
    const int tid = threadIdx.x;
    const int G = P.nin;
    const int nh = P.pr_stride * (int)(sizeof(ArgMinEntry) / 4);  // 32-bit halves per record
    const uint32_t seq = ld_agent(P.mbox_seq) + 1u;
    const int64_t par = seq & 1u;
    const uint32_t* src = reinterpret_cast<const uint32_t*>(P.price_out);
    for (int k = tid; k < G * nh; k += 256) {
        const int g = k / nh, h = k - g * nh;
        const uint64_t w = ((uint64_t)seq << 32) | src[h];
        __hip_atomic_store(&P.mbox_peer[g][(par * G + P.mbox_rank) * nh + h], w, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
    }
    const bool dead = ld_agent(&P.st->status) == ST_HANDOFF_TIMEOUT;
    __shared__ int s_to;
    if (tid == 0) s_to = 0;
    __syncthreads();
    uint32_t* dst = reinterpret_cast<uint32_t*>(const_cast<ArgMinEntry*>(P.price_in));
    const unsigned long long t0 = rtime();
    for (int k = tid; k < G * nh; k += 256) {
        const uint64_t* p = &P.mbox[par * G * nh + k];
        uint64_t w = 0;
        bool ok = false;
        while (!dead) {
            w = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            if ((uint32_t)(w >> 32) == seq) {
                ok = true;
                break;
            }
            if (rtime() - t0 > MBOX_TIMEOUT_TICKS) break;
            __builtin_amdgcn_s_sleep(2);
        }
        if (!ok) s_to = 1;  // (a benign race: every writer stores 1)
        dst[k] = (uint32_t)w;
    }
    __syncthreads();
    if (tid == 0) {
        st_agent(P.mbox_seq, seq);
        if (s_to) P.st->status = ST_HANDOFF_TIMEOUT;
    }
}

hipError_t launch_exchange(const Params& P, hipStream_t s) {
    hipLaunchKernelGGL(k_exchange, dim3(1), dim3(256), 0, s, P);
    return hipGetLastError();
}

hipError_t launch_finalize_rs(const Params& P, hipStream_t s) {
    hipLaunchKernelGGL(k_finalize_rs, dim3(1), dim3(256), 0, s, P);
    return hipGetLastError();
}

template <int BLOCK>
static hipError_t launch_update_b(const Params& P, const UpdateCfg& c, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
    switch (c.rows) {
        case 1: return launch_update_t<BLOCK, 1>(P, c.grid, c.bc_entry, s, e0, e1);
        case 2: return launch_update_t<BLOCK, 2>(P, c.grid, c.bc_entry, s, e0, e1);
        case 4: return launch_update_t<BLOCK, 4>(P, c.grid, c.bc_entry, s, e0, e1);
        case 8:
            if constexpr (BLOCK <= 512) return launch_update_t<BLOCK, 8>(P, c.grid, c.bc_entry, s, e0, e1);
            break;
    }
    return hipErrorInvalidValue;
}

// Diagnostic (SPX_DIAG_MARK=1 with stamps): a one-wave kernel before the
// FTRAN launch records when it starts, splitting the pricing -> FTRAN
// boundary into the pricing kernel's end and the FTRAN kernel's start
__global__ __launch_bounds__(64) void k_mark(Params P) {
    const unsigned long long now = rtime();
    if (threadIdx.x == 0 && P.stamps) P.stamps[STAMP_TAIL + 2 + (P.st->iter & 1)] = now;
}

hipError_t launch_update(const Params& P, const UpdateCfg& c, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
    if (P.stamps && c.mark) hipLaunchKernelGGL(k_mark, dim3(1), dim3(64), 0, s, P);
    if (P.tab) {  // window tableau: k_tab_update, 256 rows per workgroup
        const size_t lds = UpdLds<256>::bytes;
        if (e0 || e1)
            hipExtLaunchKernelGGL((k_tab_update<256>), dim3(c.grid), dim3(256), (uint32_t)lds, s, e0, e1, 0, P);
        else
            hipLaunchKernelGGL((k_tab_update<256>), dim3(c.grid), dim3(256), lds, s, P);
        return hipGetLastError();
    }
    switch (c.block) {
        case 256: return launch_update_b<256>(P, c, s, e0, e1);
        case 512: return launch_update_b<512>(P, c, s, e0, e1);
        case 1024: return launch_update_b<1024>(P, c, s, e0, e1);
    }
    return hipErrorInvalidValue;
}

static int grid_for(int64_t work, int block) {
    int64_t g = (work + block - 1) / block;
    if (g > 4096) g = 4096;
    if (g < 1) g = 1;
    return (int)g;
}

hipError_t launch_generate(double* A, double* b, double* c, int64_t m, int64_t n, int64_t L, uint64_t seed,
                           hipStream_t s) {
    hipLaunchKernelGGL(k_generate, dim3(grid_for(L * n, 256) * 4), dim3(256), 0, s, A, b, c, m, n, L, seed);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Steepest-edge pricing (SPX_PRICING_STEEPEST; oracle se_choose).  Weights
// gamma_j = 1 + ||B^-1 A_j||^2: exact at the slack basis (k_se_init), then
// kept by the Goldfarb-Reid recurrence inside k_price, which needs for the
// pending pivot (alpha = its FTRAN column, a_prev of the coming pass; B^-1
// before it = B_w + sum_{s<tau} eta_s r_s^T):
//   A_j . B^-T alpha = (B_w^T alpha) . A_j + sum_{s<tau} (U[:, s] . alpha) Wt[j][s]
// and gamma_p = 1 + ||alpha||^2.  k_se_part / k_se_fin form those before each
// pricing pass (after any fold): the column sums of M^T alpha for M = [B_w's
// columns (the compact list, or all of B_w) | U | alpha], per row block in
// ascending row order, then over the blocks in ascending order.
// ---------------------------------------------------------------------------
// Round 5: both kernels latency-bound no more (C3 steepest pass: the two took
// about 28 us): k_se_part's threads request a 16-row block of their column at
// once, and k_se_fin sums the row-block partials in slices of threads
// (coalesced, several loads in flight per thread), then the slices in
// ascending order.  Round 6: k_ftran_bc forms k_se_part's sums itself on
// every pass but a window's first (Params::se_fused, 8-row partials).
constexpr int SE_RB = 16;     // rows per k_se_part workgroup

// The pending pivot (its alpha parity and the window position): from the
// state, or -- when the FTRAN pass deferred its tail (TailRec) -- from the
// record, as the next k_price derives it
__device__ __forceinline__ bool se_pending(const Params& P, int& nw, const double*& al) {
    const DevState* st = P.st;
    int64_t iter = st->iter;
    int32_t nwv = st->nw;
    if (P.trec) {
        const TailRec R = *P.trec;
        if (R.fresh) {
            iter = R.it + 1;
            nwv = R.nw + 1;
        }
    }
    if (st->status != ST_RUNNING || iter >= st->limit) return false;
    nw = nwv;
    al = (iter & 1) ? P.alpha1 : P.alpha0;  // alpha of the pending pivot
    return nw > 0;
}

__global__ __launch_bounds__(256) void k_se_part(Params P) {
    int nw;
    const double* al;
    if (!se_pending(P, nw, al)) return;
    const int64_t m = P.m, L = P.L;
    const int KW = P.win, tau = nw - 1;
    const int S = P.bc ? P.bc_n[0] : (int)m;
    const int ncols = S + KW + 1;
    const int64_t i0 = (int64_t)blockIdx.x * SE_RB;
    const int nr = (int)(m - i0 < SE_RB ? m - i0 : SE_RB);
    __shared__ double sa[SE_RB];
    if (threadIdx.x < SE_RB) sa[threadIdx.x] = threadIdx.x < nr ? al[i0 + threadIdx.x] : 0.0;
    __syncthreads();
    const double* Mw = P.bc ? bc_buf(P, P.bc_n[2]) : P.B0;
    const int64_t ldm = P.bc ? (int64_t)P.bc_n[1] : L;  // row pitch (compact: bc_pitch)
    double* out = P.se_part + (int64_t)blockIdx.x * (L + KW + 1);
    for (int c = threadIdx.x; c < ncols; c += blockDim.x) {
        // the block's rows of column c, requested together (rows clamped;
        // the sum takes rows < nr in ascending order)
        const double* src;
        int64_t ld;
        if (c < S) {
            src = Mw + c;
            ld = ldm;
        } else if (c < S + KW) {
            const int sc = c - S;
            src = P.U + (sc < tau ? sc : 0);
            ld = KW;
        } else {
            src = al;
            ld = 1;
        }
        double v[SE_RB];
#pragma unroll
        for (int r = 0; r < SE_RB; ++r) v[r] = src[(i0 + (r < nr ? r : nr - 1)) * ld];
        double acc = 0.0;
        const bool live = c < S || c >= S + KW || c - S < tau;
#pragma unroll
        for (int r = 0; r < SE_RB; ++r)
            if (r < nr && live) acc = fma(c < S + KW ? v[r] : sa[r], sa[r], acc);
        out[c] = acc;
    }
}

// (Round 6: SE_FC columns per workgroup and SE_FS slices of partials each --
// 16 x 64 instead of 64 x 16 -- so the sums of a C3 pass's ~520 columns
// spread over ~33 workgroups instead of 9: with the fused path's 512
// partials the 9 were bound by their CUs' load rate)
constexpr int SE_FC = 16;
constexpr int SE_FS = 1024 / SE_FC;
constexpr int SE_FB = 8;  // partials per slice per round trip

__global__ __launch_bounds__(1024) void k_se_fin(Params P) {
    int nw;
    const double* al;
    if (!se_pending(P, nw, al)) return;
    const int64_t m = P.m, L = P.L;
    const int KW = P.win;
    const int S = P.bc ? P.bc_n[0] : (int)m;
    const int ncols = S + KW + 1;
    const int64_t stride = L + KW + 1;
    const int tid = threadIdx.x, cl = tid % SE_FC, sl = tid / SE_FC;  // column in the group, slice
    const int64_t c = (int64_t)blockIdx.x * SE_FC + cl;
    __shared__ double red[SE_FS][SE_FC];
    // slice sl sums the partials g = sl, sl + SE_FS, ... (ascending), SE_FB at a time
    double v = 0.0;
    const int64_t cc = c < ncols ? c : 0;
    const int gend = (int64_t)blockIdx.x * SE_FC < ncols ? P.se_parts : 0;  // (groups past the columns: nothing)
    for (int g0 = sl; g0 < gend; g0 += SE_FS * SE_FB) {
        double t[SE_FB];
#pragma unroll
        for (int k = 0; k < SE_FB; ++k) {
            const int g = g0 + k * SE_FS;
            t[k] = P.se_part[(int64_t)(g < P.se_parts ? g : 0) * stride + cc];
        }
#pragma unroll
        for (int k = 0; k < SE_FB; ++k)
            if (g0 + k * SE_FS < P.se_parts) v += t[k];
    }
    red[sl][cl] = v;
    __syncthreads();
    if (sl == 0 && c < ncols) {
        double w = red[0][cl];
#pragma unroll 16
        for (int k = 1; k < SE_FS; ++k) w += red[k][cl];
        if (c < S) P.se_v[P.bc ? (int64_t)P.rlist[c] : c] = w;
        else if (c < S + KW) P.se_cg[c - S] = w;
        else P.se_cg[KW] = 1.0 + w;
    }
    if (P.bc) {  // the unit columns of B_w: (B_w^T alpha)_k = alpha_k
        const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + tid, nt = (int64_t)gridDim.x * blockDim.x;
        for (int64_t k = t0; k < m; k += nt)
            if (P.rmap[k] < 0) P.se_v[k] = al[k];
    }
}

// gamma_j = 1 + ||A_j||^2 for every column (the slack basis B = I), one wave
// per column, lane-strided then a butterfly
__global__ __launch_bounds__(256) void k_se_init(Params P) {
    const int lane = threadIdx.x & 63;
    const int64_t w0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t nwv = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t j = w0; j < P.n; j += nwv) {
        const double* col = P.A + j * P.L;
        double a = 0.0;
        for (int64_t k = lane; k < P.m; k += 64) a = fma(col[k], col[k], a);
        a = wave_sum(a);
        if (lane == 0) P.W[j] = 1.0 + a;
    }
}

hipError_t launch_se_init(const Params& P, hipStream_t s) {
    if (!P.steep) return hipSuccess;
    hipLaunchKernelGGL(k_se_init, dim3(grid_for(P.n * 64, 256)), dim3(256), 0, s, P);
    return hipGetLastError();
}

hipError_t launch_se_prep(const Params& P, hipStream_t s, int fused_parts) {
    if (!P.steep) return hipSuccess;
    Params Q = P;
    if (fused_parts > 0) {
        Q.se_parts = fused_parts;  // the previous k_ftran_bc's workgroup partials (Params::se_fused)
    } else {
        hipLaunchKernelGGL(k_se_part, dim3((unsigned)P.se_parts), dim3(256), 0, s, P);
    }
    // SE_FC columns per workgroup (the columns in use, S + KW + 1, are at most L + KW + 1)
    hipLaunchKernelGGL(k_se_fin, dim3((unsigned)((P.L + P.win + 1 + SE_FC - 1) / SE_FC)), dim3(1024), 0, s, Q);
    return hipGetLastError();
}

int se_parts_for(int64_t m) { return (int)((m + SE_RB - 1) / SE_RB); }

hipError_t launch_reset(const Params& P, hipStream_t s) {
    const int64_t w = P.m > P.n ? P.m : P.n;
    hipLaunchKernelGGL(k_reset, dim3(grid_for(w, 256)), dim3(256), 0, s, P);
    return hipGetLastError();
}

hipError_t launch_flush(const Params& P, hipStream_t s) {
    hipLaunchKernelGGL(k_flush, dim3(1), dim3(1024), 0, s, P);
    return hipGetLastError();
}

hipError_t launch_materialize(const Params& P, double* out, hipStream_t s) {
    hipLaunchKernelGGL(k_materialize, dim3(grid_for((P.row_shard ? P.mloc : P.m) * P.L, 256)), dim3(256), 0, s, P,
                       out);
    return hipGetLastError();
}

hipError_t launch_reduced_costs(const Params& P, double* e, hipStream_t s) {
    hipLaunchKernelGGL(k_reduced_costs, dim3(grid_for(P.n * 64, 256)), dim3(256), 0, s, P, e);
    return hipGetLastError();
}

hipError_t launch_objective(const Params& P, hipStream_t s) {
    hipLaunchKernelGGL(k_objective, dim3(1), dim3(256), 0, s, P);
    return hipGetLastError();
}

}  // namespace spx

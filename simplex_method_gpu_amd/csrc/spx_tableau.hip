// spx_tableau.hip — gfx950 kernels of the window tableau (SPX_FLAG_TABLEAU,
// spx_device.h).
//
// The eta window keeps B^-1 = B_w + U R for up to KW-1 pivots.  The tableau
// variant also keeps T_w = B_w A (L x n, column-major like A) and
// dw = y_w A - c, so a loop pass needs neither the A stream of pricing
// (8(m+1)(n-m) bytes) nor the B_w stream of FTRAN (8 m^2 bytes): pricing
// reads T_w[q_tau, j], dw[j] and the Wt row of each non-basic column, FTRAN
// reads the column T_w[:, p].  What those streams did every pivot is done
// here once per window, as a rank-(KW-1) fp64 MFMA update:
//   T_w += U Wt^T   (m x n x nf, U = the eta columns, Wt[j][tau] = r_tau.A_j)
//   dw  += SY Wt^T
// which moves 16 L n bytes per window instead of 8(m+1)(n-m) + 8m^2 per pivot.
// k_tab_build rebuilds T_w = B_w A after a reinversion or a warm start;
// k_tab_loop runs whole passes in one launch of a co-resident grid.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "spx_common.h"
#include "spx_fold.h"
#include "spx_grid.h"
#include "spx_loop.h"
#include "spx_tableau.h"
#include "spx_tabdev.h"

namespace spx {

namespace {

// ---------------------------------------------------------------------------
// Active columns of a fold: j with Wt[j][t] != 0 for some t < nf (non-basic
// columns, and basic ones that entered during the window).  A column basic
// through the whole window has an all-zero Wt row (k_update writes the exact
// entries of basic columns), so folding it adds U 0 = 0: skipping it changes
// nothing (but the sign of an exact zero).  One thread per column; a wave
// appends its active columns with one atomic (the list order does not matter:
// each column's fold is independent of which wave does it).  P.tab_cnt is
// zeroed by the launcher.
// ---------------------------------------------------------------------------
template <int KW>
__global__ __launch_bounds__(256) void k_tab_active(Params P, int min_nw) {
    const int nw = P.st->nw;
    if (nw < min_nw || nw < 2) return;
    const int nf = nw - 1;
    const int lane = threadIdx.x & 63;
    const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
    bool act = false;
    if (j < P.n) {
        const dbl2* w = reinterpret_cast<const dbl2*>(P.Wt + j * KW);
#pragma unroll
        for (int k = 0; k < KW / 2; ++k) {
            const dbl2 v = w[k];
            act |= (2 * k < nf && v.x != 0.0) || (2 * k + 1 < nf && v.y != 0.0);  // NaN counts as nonzero
        }
    }
    // xw = B_w b follows B_w: xw += U (R b), R b = Wt[n][0..nf) (k_fold's
    // formula, t ascending), here when k_fold is skipped (P.tab_slack)
    if (P.tab_slack && j < P.m) {
        const double* wb = P.Wt + P.n * KW;
        double d = 0.0;
#pragma unroll
        for (int t = 0; t < KW; ++t)
            if (t < nf) d = fma(P.U[j * KW + t], wb[t], d);
        P.xw[j] += d;
    }
    const unsigned long long b = __ballot(act);
    int base = 0;
    if (lane == 0 && b) base = atomicAdd(P.tab_cnt, (int)__popcll(b));
    base = __shfl(base, 0, 64);
    if (act) P.tab_list[base + __popcll(b & ((1ull << lane) - 1ull))] = (int32_t)j;
}

// T_w += U Wt^T, dw += SY Wt^T over the active columns (k_tab_active).  A
// task is 16 TF_WAVES consecutive slots of the active list (their columns of
// T_w) by a 64-row block; a workgroup (TF_WAVES waves) walks an equal,
// contiguous range of tasks.  Wave
// w keeps the Wt fragments of its 16 columns in registers (MFMA A operand,
// lane: Wt[j0 + cl][4 s + kr]).  The eta rows U[i0 .. i0+64) of a block — 32
// KiB, contiguous — are staged once per workgroup into LDS with 16-byte loads
// (double-buffered: the next block's are loaded before this block's MFMAs)
// and read from there as the B operand (lane: U[i + cl][4 s + kr]).  The 4
// accumulator tiles of a wave (lane: T_w[i + 16 it + cl, j0 + kr + 4 r]) are
// T_w itself, read and written once; the next block's tiles are loaded after
// this block's stores (holding them across the MFMAs cost 32 VGPRs and
// measured slower).  8 waves sharing one U staging, 120 VGPRs, 2 workgroups
// per CU: 320 -> 260 us at C3 (round-1 tools/fold_bench.hip, in git history; MALL flushed),
// bit-identical (the per-element MFMA chain is unchanged).
// ---------------------------------------------------------------------------
constexpr int TF_WAVES = 8;
constexpr int TF_BLOCK = 64 * TF_WAVES;
constexpr int TF_RB = 64;  // rows per block
constexpr int TF_UP = 68;  // LDS pitch of a staged eta row (doubles): 16-B aligned, spreads banks

template <int KW>
__global__ __launch_bounds__(TF_BLOCK, 4) void k_tab_fold(Params P, int min_nw) {  // 4 waves per SIMD: 2 workgroups per CU
    const DevState* st = P.st;
    const int nw = st->nw;
    if (nw < min_nw || nw < 2) return;
    const int nf = nw - 1;
    constexpr int KS = KW / 4;
    constexpr int KW2 = KW / 2;             // dbl2 per eta row
    constexpr int NST = TF_RB * KW2;                       // dbl2 staged per block
    constexpr int UPT = (NST + TF_BLOCK - 1) / TF_BLOCK;  // per thread (KW = 8: half the threads)
    __shared__ __attribute__((aligned(16))) double Ub[2][TF_RB * TF_UP];
    const int ks = (nf + 3) / 4;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int cl = lane & 15, kr = lane >> 4;
    const int64_t m = P.m, L = P.L;
    const double* __restrict__ U = P.U;
    const double* __restrict__ Wt = P.Wt;
    double* __restrict__ T = P.T;
    const int cnt = *P.tab_cnt;  // active columns (k_tab_active)
    const int32_t* __restrict__ lst = P.tab_list;
    // tasks: (group of 16 TF_WAVES list slots, 64-row block), group-major; a
    // workgroup takes a contiguous range, so every workgroup has the same
    // amount of work whatever the active count (a grid over all n columns with
    // early exits left a half-empty second round of workgroups)
    const int64_t nblk = (m + TF_RB - 1) / TF_RB;
    const int64_t ngrp = (cnt + 16 * TF_WAVES - 1) / (16 * TF_WAVES);
    const int64_t K = ngrp * nblk;
    const int64_t k_lo = K * blockIdx.x / gridDim.x, k_hi = K * (blockIdx.x + 1) / gridDim.x;
    if (k_lo >= k_hi) return;  // uniform per workgroup

    double wf[KS];
    int32_t jc[4];  // the columns of this lane's accumulator entries (slot s0 + kr + 4 r), -1: none
    auto set_group = [&](int64_t g) {
        const int s0 = (int)g * 16 * TF_WAVES + 16 * wave;  // this wave's 16 slots
        const int64_t jw = (s0 + cl < cnt) ? (int64_t)lst[s0 + cl] : -1;
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const int t = 4 * s + kr;
            wf[s] = (jw >= 0 && t < nf) ? Wt[jw * KW + t] : 0.0;
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) jc[r] = (s0 + kr + 4 * r < cnt) ? lst[s0 + kr + 4 * r] : -1;
    };
    const int64_t ns = P.n - m;  // first slack column
    double* __restrict__ yw = st->y_buf ? P.y1 : P.y0;
    auto dw_group = [&](int64_t g) {  // dw[j] += sum_{t<nf} SY[t] Wt[j][t], once per group
        const int sl = (int)g * 16 * TF_WAVES + tid;
        if (tid < 16 * TF_WAVES && sl < cnt) {
            const int64_t j = lst[sl];
            double d = 0.0;
            for (int t = 0; t < nf; ++t) d = fma(P.SY[t], Wt[j * KW + t], d);
            P.dw[j] += d;
            // y_w += SY R (k_fold's term) when k_fold is skipped: R[t][i] =
            // r_t . e_i = Wt[ns + i][t] for slack column ns + i (an inactive
            // slack's row is all zero: no change)
            if (P.tab_slack && j >= ns) yw[j - ns] += d;
        }
    };
    auto stage_load = [&](int64_t i0, dbl2 (&ur)[UPT]) {
#pragma unroll
        for (int k = 0; k < UPT; ++k) {
            const int pce = tid + TF_BLOCK * k;
            const int64_t i = i0 + pce / KW2;
            ur[k] = (pce < NST && i < m) ? reinterpret_cast<const dbl2*>(U)[i0 * KW2 + pce] : dbl2{0.0, 0.0};
        }
    };
    auto stage_write = [&](int buf, const dbl2 (&ur)[UPT]) {
#pragma unroll
        for (int k = 0; k < UPT; ++k) {
            const int pce = tid + TF_BLOCK * k;
            if (pce < NST) *reinterpret_cast<dbl2*>(&Ub[buf][(pce / KW2) * TF_UP + 2 * (pce % KW2)]) = ur[k];
        }
    };
    auto tile_load = [&](int64_t i0, dbl4 (&acc)[4]) {
#pragma unroll
        for (int it = 0; it < 4; ++it) {
            const int64_t i = i0 + 16 * it + cl;
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[it][r] = (jc[r] >= 0 && i < m) ? T[(int64_t)jc[r] * L + i] : 0.0;
        }
    };

    int64_t g = k_lo / nblk, blk = k_lo % nblk;
    set_group(g);
    if (blk == 0) dw_group(g);
    dbl2 ur[UPT];
    dbl4 acc[4];
    stage_load(blk * TF_RB, ur);
    tile_load(blk * TF_RB, acc);
    stage_write(0, ur);
    __syncthreads();
    int buf = 0;
    for (int64_t k = k_lo; k < k_hi; ++k, buf ^= 1) {
        const int64_t i0 = blk * TF_RB;
        const bool more = k + 1 < k_hi;
        int64_t gn = g, bn = blk + 1;
        if (bn == nblk) {
            bn = 0;
            gn = g + 1;
        }
        if (more) stage_load(bn * TF_RB, ur);
        const double* ub = Ub[buf];
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            if (s < ks) {
#pragma unroll
                for (int it = 0; it < 4; ++it) {
                    const double bv = ub[(16 * it + cl) * TF_UP + 4 * s + kr];
                    acc[it] = __builtin_amdgcn_mfma_f64_16x16x4f64(wf[s], bv, acc[it], 0, 0, 0);
                }
            }
        }
#pragma unroll
        for (int it = 0; it < 4; ++it) {
            const int64_t i = i0 + 16 * it + cl;
            if (i < m) {
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    if (jc[r] >= 0) T[(int64_t)jc[r] * L + i] = acc[it][r];
            }
        }
        if (more) {
            stage_write(buf ^ 1, ur);
            if (gn != g) {  // next group: its Wt fragments and columns (bn == 0)
                set_group(gn);
                dw_group(gn);
            }
            tile_load(bn * TF_RB, acc);
        }
        g = gn;
        blk = bn;
        __syncthreads();
    }
}

// T_w = B_w A: one 64-row x 64-column block of T_w per workgroup, full K.
// Wave w: rows 16w..16w+15 of the block, 4 column tiles of 16; per 32-wide K
// chunk a lane loads 8 consecutive doubles of its B_w row (row-major) and of
// its A column (column-major): k = k0 + 8 (lane>>4) + s for MFMA step s on
// both operands (the k_rv_gemm pattern, spx_reinv.hip).
__global__ __launch_bounds__(256) void k_tab_build(Params P) {
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int cl = lane & 15, kr = lane >> 4;
    const int64_t L = P.L, m = P.m, n = P.n;
    const int64_t r0 = (int64_t)blockIdx.x * 64 + 16 * wave;
    const int64_t jb0 = (int64_t)blockIdx.y * 64;
    const int64_t row = r0 + cl;
    const bool rowok = row < m;
    const double* xr = P.B0 + (rowok ? row : 0) * L;
    const double* ac[4];
    bool cok[4];
#pragma unroll
    for (int jb = 0; jb < 4; ++jb) {
        const int64_t j = jb0 + 16 * jb + cl;
        cok[jb] = j < n;
        ac[jb] = P.A + (cok[jb] ? j : 0) * L;
    }
    dbl4 acc[4];
#pragma unroll
    for (int jb = 0; jb < 4; ++jb) acc[jb] = dbl4{0.0, 0.0, 0.0, 0.0};
    for (int64_t k0 = 0; k0 < L; k0 += 32) {
        const int64_t k = k0 + 8 * kr;
        double xv[8], av[4][8];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const dbl2 v = rowok ? *reinterpret_cast<const dbl2*>(xr + k + 2 * u) : dbl2{0.0, 0.0};
            xv[2 * u] = v.x;
            xv[2 * u + 1] = v.y;
        }
#pragma unroll
        for (int jb = 0; jb < 4; ++jb)
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const dbl2 v = cok[jb] ? *reinterpret_cast<const dbl2*>(ac[jb] + k + 2 * u) : dbl2{0.0, 0.0};
                av[jb][2 * u] = v.x;
                av[jb][2 * u + 1] = v.y;
            }
#pragma unroll
        for (int s2 = 0; s2 < 8; ++s2)
#pragma unroll
            for (int jb = 0; jb < 4; ++jb)
                acc[jb] = __builtin_amdgcn_mfma_f64_16x16x4f64(xv[s2], av[jb][s2], acc[jb], 0, 0, 0);
    }
#pragma unroll
    for (int jb = 0; jb < 4; ++jb) {
        const int64_t j = jb0 + 16 * jb + cl;
        if (!cok[jb]) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int64_t i = r0 + kr + 4 * r;
            if (i < m) P.T[j * L + i] = acc[jb][r];
        }
    }
}

// ---------------------------------------------------------------------------
// Persistent tableau loop: whole passes in ONE launch (co-resident grid), two grid
// barriers per pass, as k_loop (spx_loop.h) does for the eta window.  A
// tableau pass moves a few MB, so what it pays for is dependent round trips
// and barriers; the loop runs on few workgroups (cheap barriers: 1.3 us at
// 64, tools/barrier_bench.hip) and keeps what each owns on chip:
//   columns: wave v = g W + w owns list slots v + c G W, one per lane c
//     (c < cpw <= 64); LDS holds each slot's column j, dw[j], its Devex
//     weight and its window row Wt[j][0..tau];
//   rows: wave w owns rows row0 + w + r W, one per lane r; registers hold
//     alpha_prev, b_ixs, c_B, x_b, LDS the row's eta coefficients U[i][.].
// Per pass (the arithmetic of k_price WM 3 / k_tab_update, spx_tabdev.h):
//   A  lane c prices column c: T_w[q, j] (one gather per wave, issued with
//      the re-cache of list slots the last pivot changed) and the window
//      sums from LDS; workgroup argmin -> partial (with the candidate's
//      window entry and list slot).                           -> barrier 1
//   B  the column results of A go to HBM (off barrier 1's drain); every
//      workgroup reduces the pricing partials (same p everywhere); lane r:
//      alpha_i from T_w[i,p] and its LDS row; x_b; ratio test.  -> barrier 2
//   C  every workgroup reduces the ratio-test partials (q, s_y) and loads
//      U[q][.] for the next pricing; workgroup 0 writes the bookkeeping;
//      owners note the two list slots the pivot changed; the new pending
//      base row B_w[q,:] goes to Qrows for k_fold, one slice per workgroup.
// Global copies of everything cached (Wt, U, W, x_b, alpha) are written as
// they change, so the two-kernel passes, the folds and readbacks see the
// same state.
// ---------------------------------------------------------------------------
constexpr int TKW = 64;
constexpr int TKP = TKW + 1;  // LDS row pitch (doubles): lane-per-row reads hit distinct banks
#ifndef SPX_TAB_CLK
// diagnostic stamps of workgroup 0 (round-1 tools/tab_clk.sh, in git history): clk[0] = pass start,
// clk[2] = barrier 2 done; clk[1] = barrier 1 done (0), or point k of the
// pass (k = 1 .. 11, TAB_STAMP below) in a build with SPX_TAB_CLK = k
#define SPX_TAB_CLK 0
#endif
#define TAB_STAMP(k)                                  \
    do {                                              \
        if (SPX_TAB_CLK == (k) && clk) clk[1] = rtime(); \
    } while (0)

// Cross-workgroup partials without a grid barrier.  Each 8-byte field of a
// workgroup's partial travels as two tagged words, (tag << 32) | 32-bit half,
// stored field-major (word k of workgroup g at [k * G + g], so a wave reading
// word k of all G touches G * 8 contiguous bytes).  An aligned 8-byte store
// is single-copy atomic, so a reader that sees the current tag in every word
// of a partial has all of it; it polls the words until then.  The tag is
// unique per launch and exchange: (epoch << 7) | (pass << 1) | phase, epoch
// the host's launch counter (the buffers start as 0xFF..: no tag matches).
// Data that crosses workgroups beside the partials (the phase-B deferred
// writes: Wt entries, U entries, Devex weights) is stored agent-scope, and
// every wave drains (s_waitcnt vmcnt(0)) before its workgroup publishes the
// ratio-test partial: whoever has read all ratio-test partials of a pass sees
// those writes (MI355X_MICROARCH.md's hand-off rule, with the tag as flag).
// Pricing partial: val, idx, w, e, slot; ratio test: the UpdPartial fields.
constexpr int TAB_PP_FIELDS = 5;
constexpr int TAB_UP_FIELDS = 8;
__device__ __forceinline__ uint32_t tab_tag(uint32_t epoch, int pass, int phase) {
    return (epoch << 7) | ((uint32_t)pass << 1) | (uint32_t)phase;
}
template <typename T>
__device__ __forceinline__ void st_tagged(uint64_t* X, int f, int G, int g, uint32_t tag, T v) {
    static_assert(sizeof(T) == 8, "8-byte partial fields");
    uint64_t u;
    __builtin_memcpy(&u, &v, 8);
    const uint64_t t = (uint64_t)tag << 32;
    st_agent(&X[(int64_t)(2 * f) * G + g], (uint64_t)(t | (u & 0xffffffffull)));
    st_agent(&X[(int64_t)(2 * f + 1) * G + g], (uint64_t)(t | (u >> 32)));
}
template <typename T>
__device__ __forceinline__ T tagged_field(const uint64_t* w, int f) {
    const uint64_t u = (uint64_t)((w[2 * f] & 0xffffffffull) | (w[2 * f + 1] << 32));
    T v;
    __builtin_memcpy(&v, &u, 8);
    return v;
}
// Wave-wide poll (one wave per workgroup polls): every lane with g < G
// watches word 0 of workgroup g's partial until it carries tag, then loads
// all 2 NF words (again until all carry it; normally once).  false: the poll
// timed out (err is set).
template <int NF>
__device__ __forceinline__ bool poll_tagged(const uint64_t* X, int G, int g, uint32_t tag, uint64_t (&w)[2 * NF],
                                            LoopState* ls) {
    uint32_t spins = 0;
    for (;;) {
        const bool ok = g >= G || (uint32_t)(ld_agent(&X[g]) >> 32) == tag;
        if (__ballot(!ok) == 0) break;
        if ((++spins & 255u) == 0 && (spins > (1u << 22) || ld_agent(&ls->err))) {
            st_agent(&ls->err, 1);
            return false;
        }
    }
    for (;;) {
        bool ok = true;
        if (g < G) {
#pragma unroll
            for (int k = 0; k < 2 * NF; ++k) w[k] = ld_agent(&X[(int64_t)k * G + g]);
#pragma unroll
            for (int k = 0; k < 2 * NF; ++k) ok = ok && (uint32_t)(w[k] >> 32) == tag;
        }
        if (__ballot(!ok) == 0) return true;
        if ((++spins & 255u) == 0 && (spins > (1u << 22) || ld_agent(&ls->err))) {
            st_agent(&ls->err, 1);
            return false;
        }
    }
}

struct TabPick {  // a pricing candidate being merged
    double val;
    int64_t idx;
    double w, e;
    int64_t slot;
};
__device__ __forceinline__ void pick_merge(TabPick& a, const TabPick& b) {
    if (argmin_better(b.val, b.idx, a.val, a.idx)) a = b;
}

// ratio-test merge carrying UpdPartial::pad (the winner's eta entry) with the winner
__device__ __forceinline__ void tup_merge(UpdPartial& a, const UpdPartial& b) {
    const bool take = argmin_better(b.theta, b.idx, a.theta, a.idx);
    upd_merge(a, b);
    if (take) a.pad = b.pad;
}

template <int WAVES>
struct TabLds {
    double SY[TKW];
    double Uq[TKW];
    double Wp[TKW];
    TabPick ppick[WAVES];
    UpdPartial ured[WAVES];
    TabPick pwin;
    UpdPartial uwin;
    int fail;
};

// dynamic LDS: [W*cpw] int32 columns | [W*cpw] dw | [W*cpw] Devex weights |
// [W*cpw][TKP] window rows | [W*rw][TKP] row eta coefficients (wave-major)
template <int WAVES>
struct TabCache {
    int32_t* col;
    double* dwc;
    double* wc;
    double* wt;
    double* ur;
    __device__ TabCache(unsigned char* base, int cpw) {
        const int ns = cpw * WAVES;
        col = reinterpret_cast<int32_t*>(base);
        dwc = reinterpret_cast<double*>(base + ((4 * ns + 15) / 16) * 16);
        wc = dwc + ns;
        wt = wc + ns;
        ur = wt + (int64_t)ns * TKP;
    }
    static size_t bytes(int cpw, int rw) {
        const size_t ns = (size_t)cpw * WAVES;
        return ((4 * ns + 15) / 16) * 16 + 8 * ns * (2 + TKP) + 8 * (size_t)rw * WAVES * TKP;
    }
};

template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_tab_loop(Params P, LoopArgs La, int cpw, int rw) {
    constexpr int WAVES = BLOCK / 64;
    __shared__ TabLds<WAVES> S;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const TabCache<WAVES> C(smem, cpw);
    uint64_t* const XP = reinterpret_cast<uint64_t*>(La.xp);
    uint64_t* const XU = reinterpret_cast<uint64_t*>(La.xu);
    DevState* st = P.st;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int G = (int)gridDim.x;
    const bool wg0 = blockIdx.x == 0;
    const int64_t L = P.L, m = P.m, n = P.n;
    const int KW = P.win;
    {  // the whole grid resident, or nobody touches the state (spx_grid.h)
        __shared__ int s_arr;
        if (!grid_arrive(La.ls, &s_arr)) return;
    }

    int64_t it = st->iter;
    const int64_t it0 = it;
    const int64_t limit = st->limit;
    if (st->status != ST_RUNNING || it >= limit) return;
    int nw = st->nw;
    if (nw >= KW) return;  // the host folds first
    int64_t q = st->q;
    double aq = st->aq;
    int64_t q_prev = -1;   // the pivot before the pending one (this launch only)
    double aq_prev = 0.0;
    int64_t xb_applied = st->xb_applied;
    const int cnt = st->nb_count;
    int64_t lastv = P.nb_list[cnt - 1];  // the list's last slot (it receives every leaving column)
    int64_t dleave = st->leave;
    double dwp = st->wp;
    const int stride = G * WAVES;
    const int vid = (int)blockIdx.x * WAVES + wave;  // this wave's first list slot
    // this lane's column slot and row
    const int cs = lane < cpw ? lane : cpw - 1;
    const int ls = wave * cpw + cs;
    const bool cv = lane < cpw && vid + lane * stride < cnt;
    const int64_t rpw = (m + G - 1) / G;
    const int64_t row0 = (int64_t)blockIdx.x * rpw;
    const int64_t row1 = (row0 + rpw < m) ? row0 + rpw : m;
    const int rs = lane < rw ? lane : rw - 1;
    const int lr = wave * rw + rs;
    const int64_t irow = row0 + wave + (int64_t)rs * WAVES;
    const bool rv = lane < rw && irow < row1;
    // this workgroup's slice of a base row (Qrows staging for k_fold)
    const int64_t qsl = ((L + G - 1) / G + 1) / 2 * 2;
    const int64_t qk0 = (int64_t)blockIdx.x * qsl;
    const int64_t qk1 = (qk0 + qsl < L) ? qk0 + qsl : L;

    // ---- prologue: window scalars, column and row caches
    if (tid < KW) S.SY[tid] = (tid < nw) ? P.SY[tid] : 0.0;
    if (nw > 0 && wg0 && tid < nw - 1) P.Urows[(int64_t)(nw - 1) * KW + tid] = P.U[q * KW + tid];
    if (cv) {
        const int32_t j = P.nb_list[vid + lane * stride];
        C.col[ls] = j;
        C.dwc[ls] = P.dw[j];
        C.wc[ls] = P.devex ? P.W[j] : 1.0;
    }
    lds_barrier();
    for (int c = 0; c < cpw; ++c) {  // window rows: one coalesced row per step
        if (vid + c * stride >= cnt) break;
        const int64_t j = C.col[wave * cpw + c];
        C.wt[(int64_t)(wave * cpw + c) * TKP + lane] = (lane < nw - 1) ? P.Wt[j * KW + lane] : 0.0;
    }
    double apr = 0.0, cbr = 0.0, xbr = 0.0;
    int64_t bxr = -1;
    if (rv) {
        apr = ((it & 1) ? P.alpha1 : P.alpha0)[irow];
        cbr = P.c_B[irow];
        xbr = P.x_b[irow];
        bxr = P.b_ixs[irow];
    }
    for (int r = 0; r < rw; ++r) {  // eta coefficients: one coalesced row per step
        const int64_t i = row0 + wave + (int64_t)r * WAVES;
        if (i >= row1) break;
        C.ur[(int64_t)(wave * rw + r) * TKP + lane] = (lane < nw - 1) ? P.U[i * KW + lane] : 0.0;
    }
    lds_barrier();
    // list slots the last pivot changed, owned by this wave: re-cached at the
    // start of the next pricing phase (their window rows then are visible)
    int rc_ls0 = -1, rc_ls1 = -1;
    int64_t rc_j0 = 0, rc_j1 = 0;
    double rc_basic = 0.0;  // the leaving column's window entry for the pivot that made it leave
    // U[q][tau-1] of the pending pivot, from the ratio-test partial (its row
    // owner's store is still in flight); false at launch: every entry is in HBM
    bool uq_pad = false;
    double uq_pad_v = 0.0;
    // results of a pass that go to HBM one phase later (after the next
    // barrier 1, so no barrier's drain waits for them): this lane's row
    // (eta entry, its basic column's window entry, x_b, alpha) and, in
    // workgroup 0, the pivot's bookkeeping (v4:339-342)
    bool rp = false, rp_pend = false;
    int r_tau = 0;
    int64_t r_it = 0, r_bx = -1;
    double r_ei = 0.0, r_bv = 0.0;
    bool bk = false;
    int64_t bk_kp = 0, bk_lastv = 0, bk_p = 0, bk_leave = 0, bk_qn = 0, bk_it = 0;
    int bk_nw = 0;
    double bk_cp = 0.0, bk_sy = 0.0, bk_aq = 0.0, bk_mine = 0.0, bk_wp = 0.0;
    auto flush = [&]() {
        if (rp && rv) {
            if (rp_pend) {
                st_agent(&P.U[irow * KW + r_tau], r_ei);
                st_agent(&P.Wt[r_bx * KW + r_tau], r_bv);
            }
            P.x_b[irow] = xbr;
            ((r_it & 1) ? P.alpha0 : P.alpha1)[irow] = apr;
        }
        rp = false;
        if (bk && wg0 && tid == 0) {
            if (bk_kp != cnt - 1) {
                st_agent(&P.nb_list[bk_kp], (int32_t)bk_lastv);
                st_agent(&P.nb_pos[bk_lastv], (int32_t)bk_kp);
            }
            st_agent(&P.nb_pos[bk_p], (int32_t)-1);
            st_agent(&P.nb_list[cnt - 1], (int32_t)bk_leave);
            st_agent(&P.nb_pos[bk_leave], (int32_t)(cnt - 1));
            st_agent(&P.c_B[bk_qn], bk_cp);
            st_agent(&P.b_ixs[bk_qn], bk_p);
            P.SY[bk_nw] = bk_sy;
            st->aq = bk_aq;
            st->s_y = bk_sy;
            st->nw = bk_nw + 1;
            st->xb_applied = bk_it;
            st->p = bk_p;
            st->q = bk_qn;
            st->min_e = bk_mine;
            st->iter = bk_it + 1;
            record_pivot(P, bk_it, bk_p, bk_qn);
            if (P.devex) {
                st->leave = bk_leave;
                st->wp = bk_wp;
            }
        }
        bk = false;
    };

    for (int pass = 0; pass < La.npasses && it < limit; ++pass) {
        const bool pend = nw > 0;
        const int tau = nw - 1;
        unsigned long long* clk = (La.clock && wg0 && tid == 0) ? La.clock + 3 * (int64_t)pass : nullptr;
        if (clk) clk[0] = rtime();

        // ================= phase A: pricing, lane c <-> column slot c
        // Every load of the phase is issued before any is waited for (one
        // round trip): the T_w row entry of this lane's column, the pending
        // pivot's eta coefficients U[q][s<tau] (S.Uq), Wt[n][.] and xw[q]
        // for s_x, this workgroup's slice of the base row B_w[q,:] (Qrows,
        // stored in phase B) and the list slots the last pivot changed.
        const int64_t cj = !cv ? 0 : (ls == rc_ls0) ? rc_j0 : (ls == rc_ls1) ? rc_j1 : (int64_t)C.col[ls];
        const double tq = (pend && cv) ? P.T[cj * L + q] : 0.0;
        double uqv = 0.0, wtn = 0.0;
        if (pend && lane < tau) {
            if (tid < KW) uqv = (uq_pad && lane == tau - 1) ? uq_pad_v : ld_agent(&P.U[q * KW + lane]);
            wtn = ld_agent(&P.Wt[n * KW + lane]);
        }
        const double xwq = pend ? P.xw[q] : 0.0;
        const double qv = (pend && qk0 + tid < qk1) ? P.B0[q * L + qk0 + tid] : 0.0;
        if (rc_ls0 >= 0 || rc_ls1 >= 0) {
            double rw_v[2], rdw[2], rwc[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int lsn = h ? rc_ls1 : rc_ls0;
                const int64_t jn = h ? rc_j1 : rc_j0;
                rw_v[h] = rdw[h] = rwc[h] = 0.0;
                if (lsn < 0) continue;
                // the leaving column's entry for the last pivot: its basic-column
                // value (stored one phase later, so not yet visible)
                rw_v[h] = (h && lane == tau - 1) ? rc_basic : ((lane < tau) ? ld_agent(&P.Wt[jn * KW + lane]) : 0.0);
                if (lane == 0) {
                    rdw[h] = P.dw[jn];
                    rwc[h] = P.devex ? ld_agent(&P.W[jn]) : 1.0;
                }
            }
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int lsn = h ? rc_ls1 : rc_ls0;
                if (lsn < 0) continue;
                C.wt[(int64_t)lsn * TKP + lane] = rw_v[h];
                if (lane == 0) {
                    C.col[lsn] = (int32_t)(h ? rc_j1 : rc_j0);
                    C.dwc[lsn] = rdw[h];
                    C.wc[lsn] = rwc[h];
                }
            }
            rc_ls0 = rc_ls1 = -1;
        }
        if (tid < KW) S.Uq[tid] = uqv;
        // its coefficients into Urows (k_fold), as k_update stages them
        if (pend && wg0 && tid < tau) P.Urows[(int64_t)tau * KW + tid] = uqv;
        lds_barrier();
        // s_x = r_tau . b for phase B's x_b update (k_tab_update's formula)
        double sxw = 0.0;
        if (pend) sxw = xwq + wave_sum(lane < tau ? mul_nc(S.Uq[lane], wtn) : 0.0);
        TAB_STAMP(1);
        TabPick best{INFINITY, INT64_MAX, 0.0, 0.0, -1};
        double cw = 0.0, cwt = 0.0;  // this column's window entry and Devex weight, stored in phase B
        {
            const double dv = cv ? C.dwc[ls] : 0.0;
            const double* wrow = C.wt + (int64_t)ls * TKP;
            double e;
            tab_price_column(tq, dv, cv ? tau : -1, S.SY, S.Uq, [&](int s2) { return wrow[s2]; }, cw, e);
            TAB_STAMP(2);
            if (cv) {
                if (pend) C.wt[(int64_t)ls * TKP + tau] = cw;
                double key = e;
                if (P.devex) {  // include/simplex.h SPX_PRICING_DEVEX, as k_price
                    cwt = C.wc[ls];
                    if (pend) {
                        if (cj == dleave) cwt = fmax(dwp / (aq * aq), 1.0);
                        else {
                            const double g = cw / aq;
                            cwt = fmax(cwt, g * g * dwp);
                        }
                        C.wc[ls] = cwt;
                    }
                    key = (e < -P.eps) ? -(e * e) / cwt : INFINITY;
                }
                best.val = key;
                best.idx = cj;
            }
            // wave argmin on (key, column) by DPP (lane 63 ends with it); the
            // winner's entry, reduced cost and slot are read from its lane
            double bv = best.val;
            int64_t bj = best.idx;
            lane_argmin<64>(bv, bj);
            bv = readlane_d(bv, 63);
            bj = readlane_l(bj, 63);
            const unsigned long long wb = __ballot(cv && cj == bj);
            const int wl = wb ? __ffsll((long long)wb) - 1 : 0;
            best = TabPick{bv, bj, readlane_d(cw, wl), readlane_d(e, wl), (int64_t)vid + (int64_t)wl * stride};
        }
        TAB_STAMP(3);
        if (lane == 0) S.ppick[wave] = best;
        lds_barrier();
        if (wave == 0) {  // workgroup merge: lane w holds wave w's pick; the winning lane stores the partial
            const TabPick w = lane < WAVES ? S.ppick[lane] : TabPick{INFINITY, INT64_MAX, 0.0, 0.0, -1};
            double bv = w.val;
            int64_t bj = w.idx;
            lane_argmin<8>(bv, bj);
            bv = readlane_d(bv, 0);
            bj = readlane_l(bj, 0);
            const unsigned long long wb = __ballot(lane < WAVES && w.idx == bj && w.val == bv);
            const int wl = wb ? __ffsll((long long)wb) - 1 : 0;
            if (lane == wl) {  // no drain: phase A stores nothing another workgroup reads
                const int g = blockIdx.x;
                const uint32_t tg = tab_tag(La.epoch, pass, 0);
                st_tagged(XP, 0, G, g, tg, w.val);
                st_tagged(XP, 1, G, g, tg, w.idx);
                st_tagged(XP, 2, G, g, tg, w.w);
                st_tagged(XP, 3, G, g, tg, w.e);
                st_tagged(XP, 4, G, g, tg, w.slot);
            }
        }
        TAB_STAMP(4);
        TAB_STAMP(5);

        // ================= phase B: entering column, FTRAN + ratio test
        // Deferred writes, drained at barrier 2: phase A's column results,
        // the last pass's row results and bookkeeping, and the pending
        // pivot's base row slice for k_fold.
        // Wave 0 polls the pricing partials and reduces them (the same p in
        // every workgroup); the other waves meanwhile issue the deferred
        // stores, then read the result from LDS.
        if (cv && pend) {
            st_agent(&P.Wt[cj * KW + tau], cw);
            if (P.devex) st_agent(&P.W[cj], cwt);
        }
        if (pend && wg0 && tid == 0) st_agent(&P.Wt[n * KW + tau], sxw);
        flush();
        if (pend && qk0 + tid < qk1) P.Qrows[(int64_t)tau * L + qk0 + tid] = qv;
        if (wave == 0) {
            TabPick w{INFINITY, INT64_MAX, 0.0, 0.0, -1};
            const uint32_t tg = tab_tag(La.epoch, pass, 0);
            bool ok = true;
            for (int g0 = 0; g0 < G && ok; g0 += 64) {
                uint64_t x[2 * TAB_PP_FIELDS];
                ok = poll_tagged<TAB_PP_FIELDS>(XP, G, g0 + lane, tg, x, La.ls);
                if (ok && g0 + lane < G)
                    pick_merge(w, TabPick{tagged_field<double>(x, 0), tagged_field<int64_t>(x, 1),
                                          tagged_field<double>(x, 2), tagged_field<double>(x, 3),
                                          tagged_field<int64_t>(x, 4)});
            }
            double bv = w.val;
            int64_t bj = w.idx;
            lane_argmin<64>(bv, bj);
            bv = readlane_d(bv, 63);
            bj = readlane_l(bj, 63);
            const unsigned long long wb = __ballot(w.idx == bj && w.val == bv);
            const int wl = wb ? __ffsll((long long)wb) - 1 : 0;
            const TabPick r{bv, bj, readlane_d(w.w, wl), readlane_d(w.e, wl), readlane_l(w.slot, wl)};
            if (lane == 0) {
                S.pwin = r;
                S.fail = !ok;
            }
        }
        lds_barrier();
        if (S.fail) return;
        const TabPick pw = S.pwin;
        TAB_STAMP(0);
        TAB_STAMP(5);
        const int64_t p = pw.idx;
        const double min_e = pw.val;
        if (no_entering(P, min_e, p)) {  // OptimumFound (v4:299-302)
            if (wg0 && tid == 0) {
                st->p = p;
                st->min_e = P.devex ? pw.e : min_e;
                st->status = ST_OPTIMAL;
            }
            break;
        }
        double rei = 0.0;  // this lane's row: eta entry of the pending pivot
        double c_p = 0.0;
        {
            // the entering column's window row: entries s < tau from earlier
            // passes, entry tau from its pricer's partial; a column that left
            // at the last pivot has its entry tau-1 (its basic value) still in
            // flight: (q == q_prev) ? aq_prev : 0
            if (tid < KW) {
                double v = 0.0;
                if (tid == tau) v = pw.w;
                else if (tid < tau)
                    v = (p == lastv && tid == tau - 1 && q_prev >= 0) ? ((q == q_prev) ? aq_prev : 0.0)
                                                                      : ld_agent(&P.Wt[p * KW + tid]);
                S.Wp[tid] = v;
            }
            const bool upd_x = xb_applied < it;
            const double tcol = rv ? P.T[p * L + irow] : 0.0;
            c_p = P.c[p];
            const double s_x = upd_x ? sxw : 0.0;
            lds_barrier();
            TAB_STAMP(7);
            double th = INFINITY, tT = 0.0, a = 0.0;
            int64_t ti = INT64_MAX;
            if (rv) {
                rei = pend ? eta_entry(apr, irow, q, aq) : 0.0;
                const double* urow = C.ur + (int64_t)lr * TKP;
                a = tab_ftran_row(tcol, tau, rei, S.Wp, [&](int s2) { return urow[s2]; });
                if (pend) C.ur[(int64_t)lr * TKP + tau] = rei;
                if (upd_x) xbr = fma(s_x, rei, xbr);
                apr = a;
                th = ratio_key(P, xbr, a);
                ti = irow;
                tT = cbr * a;
                // for the deferred write
                rp = true;
                rp_pend = pend;
                r_tau = tau;
                r_it = it;
                r_ei = rei;
                r_bx = bxr;
                r_bv = (irow == q) ? aq : 0.0;  // r_tau . A_j of the basic column j of this row
            }
            TAB_STAMP(8);
            // wave merge by DPP: argmin on (theta, row) and the c_B.alpha sum;
            // alpha <= 0 counted by ballot; the winner's scalars (and its eta
            // entry, U[q][tau] for the next pricing) from its lane
            double bth = th;
            int64_t bti = ti;
            lane_argmin<64>(bth, bti);
            lane_sum<64>(tT);
            UpdPartial wp;
            wp.theta = readlane_d(bth, 63);
            wp.idx = readlane_l(bti, 63);
            wp.T = readlane_d(tT, 63);
            wp.nonpos = __popcll(__ballot(rv && !(a > P.piv_tol)));
            const unsigned long long wb = __ballot(rv && irow == wp.idx);
            const int wl = wb ? __ffsll((long long)wb) - 1 : 0;
            wp.a_w = readlane_d(a, wl);
            wp.cb_w = readlane_d(cbr, wl);
            wp.bix_w = readlane_l(bxr, wl);
            wp.pad = readlane_l(__double_as_longlong(rei), wl);
            if (lane == 0) S.ured[wave] = wp;
            drain_vmem();  // this pass's agent-scope writes, before the partial publishes them
            lds_barrier();
            if (wave == 0) {  // workgroup merge: lane w holds wave w's partial
                const UpdPartial u = lane < WAVES ? S.ured[lane] : upd_empty();
                double uth = u.theta, uT = u.T;
                int64_t uti = u.idx;
                int unp = (int)u.nonpos;
                lane_argmin<8>(uth, uti);
                lane_sum<8>(uT);
                lane_isum<8>(unp);
                uth = readlane_d(uth, 0);
                uti = readlane_l(uti, 0);
                const int64_t snp = __builtin_amdgcn_readlane(unp, 0);
                const double sT = readlane_d(uT, 0);  // (cross-lane reads stay outside the branch)
                const unsigned long long wb2 = __ballot(lane < WAVES && u.idx == uti && u.theta == uth);
                const int wl2 = wb2 ? __ffsll((long long)wb2) - 1 : 0;
                if (lane == wl2) {
                    const int g = blockIdx.x;
                    const uint32_t tg = tab_tag(La.epoch, pass, 1);
                    st_tagged(XU, 0, G, g, tg, u.theta);
                    st_tagged(XU, 1, G, g, tg, u.idx);
                    st_tagged(XU, 2, G, g, tg, snp);
                    st_tagged(XU, 3, G, g, tg, sT);
                    st_tagged(XU, 4, G, g, tg, u.a_w);
                    st_tagged(XU, 5, G, g, tg, u.cb_w);
                    st_tagged(XU, 6, G, g, tg, u.bix_w);
                    st_tagged(XU, 7, G, g, tg, u.pad);
                }
            }
        }
        TAB_STAMP(9);

        // ================= phase C: leaving row, s_y, bookkeeping (update_tail)
        {  // wave 0 polls the ratio-test partials and reduces them (DPP)
            if (wave == 0) {
                UpdPartial w = upd_empty();
                const uint32_t tg = tab_tag(La.epoch, pass, 1);
                bool ok = true;
                for (int g0 = 0; g0 < G && ok; g0 += 64) {
                    uint64_t x[2 * TAB_UP_FIELDS];
                    ok = poll_tagged<TAB_UP_FIELDS>(XU, G, g0 + lane, tg, x, La.ls);
                    if (ok && g0 + lane < G) {
                        UpdPartial v;
                        v.theta = tagged_field<double>(x, 0);
                        v.idx = tagged_field<int64_t>(x, 1);
                        v.nonpos = tagged_field<int64_t>(x, 2);
                        v.T = tagged_field<double>(x, 3);
                        v.a_w = tagged_field<double>(x, 4);
                        v.cb_w = tagged_field<double>(x, 5);
                        v.bix_w = tagged_field<int64_t>(x, 6);
                        v.pad = tagged_field<int64_t>(x, 7);
                        tup_merge(w, v);
                    }
                }
                if (clk) clk[2] = rtime();
                double bth = w.theta, sT = w.T;
                int64_t bti = w.idx;
                int np = (int)w.nonpos;
                lane_argmin<64>(bth, bti);
                lane_sum<64>(sT);
                lane_isum<64>(np);
                UpdPartial r;
                r.theta = readlane_d(bth, 63);
                r.idx = readlane_l(bti, 63);
                r.T = readlane_d(sT, 63);
                r.nonpos = __builtin_amdgcn_readlane(np, 63);
                const unsigned long long wb = __ballot(w.idx == r.idx && w.theta == r.theta);
                const int wl = wb ? __ffsll((long long)wb) - 1 : 0;
                r.a_w = readlane_d(w.a_w, wl);
                r.cb_w = readlane_d(w.cb_w, wl);
                r.bix_w = readlane_l(w.bix_w, wl);
                r.pad = readlane_l(w.pad, wl);
                if (lane == 0) {
                    S.uwin = r;
                    S.fail = !ok;
                }
            }
            lds_barrier();
            if (S.fail) return;
        }
        const UpdPartial t = S.uwin;
        TAB_STAMP(10);
        if (t.nonpos == m || t.idx < 0 || t.idx >= m) {  // Unbounded (v4:319-322)
            if (wg0 && tid == 0) {
                st->p = p;
                st->min_e = min_e;
                st->status = ST_UNBOUNDED;
            }
            break;
        }
        const int64_t qn = t.idx, leave = t.bix_w;
        const double aqn = t.a_w;
        const double s_y = y_scalar(t.T, aqn, t.cb_w, c_p);
        const int64_t kp = pw.slot;
        const double wp_new = P.devex ? ld_agent(&P.W[p]) : 0.0;
        // the bookkeeping, written one phase later (flush)
        bk = true;
        bk_kp = kp;
        bk_lastv = lastv;
        bk_p = p;
        bk_leave = leave;
        bk_qn = qn;
        bk_it = it;
        bk_nw = nw;
        bk_cp = c_p;
        bk_sy = s_y;
        bk_aq = aqn;
        bk_mine = P.devex ? pw.e : min_e;
        bk_wp = wp_new;
        if (rv && irow == qn) {  // the pivot's row: its basis entry (v4:339-342)
            bxr = p;
            cbr = c_p;
        }
        // the two list slots the pivot changed (swap-remove of p: slot kp <-
        // lastv; append of leave: slot cnt-1); their owners re-cache them at
        // the start of the next pricing phase
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int slot = h ? cnt - 1 : (int)kp;  // the list holds n - m < 2^31 entries
            if (h == 0 && kp == cnt - 1) continue;
            const int sq = slot / stride;
            if (slot - sq * stride != vid) continue;
            const int lsn = wave * cpw + sq;
            if (h) {
                rc_ls1 = lsn;
                rc_j1 = leave;
                rc_basic = pend ? ((qn == q) ? aq : 0.0) : 0.0;  // r_tau . A_leave, leave basic in row qn
            } else {
                rc_ls0 = lsn;
                rc_j0 = lastv;
            }
        }
        lastv = leave;
        // the new pending pivot's eta coefficient U[qn][tau] (the next
        // phase A loads the entries s < tau)
        uq_pad = true;
        uq_pad_v = __longlong_as_double(t.pad);
        if (tid == 0) S.SY[nw] = s_y;
        q_prev = q;
        aq_prev = aq;
        q = qn;
        aq = aqn;
        xb_applied = it;
        dleave = leave;
        dwp = wp_new;
        ++nw;
        ++it;
        TAB_STAMP(11);
        lds_barrier();
    }
    flush();
    // the pending pivot's base row slice for k_fold (the next launch's
    // prologue does not restage it)
    if (nw > 0)
        for (int64_t k = qk0 + tid; k < qk1; k += BLOCK) P.Qrows[(int64_t)(nw - 1) * L + k] = P.B0[q * L + k];
    if (wg0 && tid == 0) La.ls->passes = (int32_t)(it - it0);
}

// The window reset k_fold's last workgroup does (the pending pivot stays
// pending as tau = 0), when k_fold is skipped.
__global__ void k_tab_reset(Params P, int min_nw) {
    DevState* st = P.st;
    const int nw = st->nw;
    if (nw < min_nw || nw < 2) return;
    P.SY[0] = P.SY[nw - 1];
    st->nw = 1;
}

// B_w from T_w's slack block for readbacks (P.tab_slack): B_w[r][i] =
// T_w[r, ns + i], a 64 x 64 tile per workgroup transposed through LDS.
__global__ __launch_bounds__(256) void k_tab_binv(Params P) {
    __shared__ double tile[64][65];
    const int64_t m = P.m, L = P.L, ns = P.n - P.m;
    const int64_t r0 = (int64_t)blockIdx.x * 64, i0 = (int64_t)blockIdx.y * 64;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    for (int k = ty; k < 64; k += 4) {  // column i0 + k of the block, rows r0 + tx
        const int64_t i = i0 + k, r = r0 + tx;
        tile[k][tx] = (i < m && r < m) ? P.T[(ns + i) * L + r] : 0.0;
    }
    __syncthreads();
    for (int k = ty; k < 64; k += 4) {  // row r0 + k of B_w, columns i0 + tx
        const int64_t r = r0 + k, i = i0 + tx;
        if (r < m && i < m) P.B0[r * L + i] = tile[tx][k];
    }
}

}  // namespace

hipError_t launch_tab_binv(const Params& P, hipStream_t s) {
    if (!P.tab || !P.tab_slack) return hipSuccess;
    const unsigned g = (unsigned)((P.m + 63) / 64);
    hipLaunchKernelGGL(k_tab_binv, dim3(g, g), dim3(256), 0, s, P);
    return hipGetLastError();
}

hipError_t launch_tab_fold(const Params& P, int min_nw, int cus, hipStream_t s) {
    if (!P.tab) return hipSuccess;
    hipError_t e = hipMemsetAsync(P.tab_cnt, 0, sizeof(int32_t), s);
    if (e != hipSuccess) return e;
    const unsigned ga = (unsigned)((P.n + 255) / 256);
    switch (P.win) {
        case 8: hipLaunchKernelGGL(k_tab_active<8>, dim3(ga), dim3(256), 0, s, P, min_nw); break;
        case 16: hipLaunchKernelGGL(k_tab_active<16>, dim3(ga), dim3(256), 0, s, P, min_nw); break;
        case 32: hipLaunchKernelGGL(k_tab_active<32>, dim3(ga), dim3(256), 0, s, P, min_nw); break;
        case 64: hipLaunchKernelGGL(k_tab_active<64>, dim3(ga), dim3(256), 0, s, P, min_nw); break;
        default: return hipErrorInvalidValue;
    }
    // 2 workgroups per CU (LDS: 68 KiB each), all resident; each takes an equal
    // share of the (column group, row block) tasks of the active list
    const dim3 grid((unsigned)(2 * (cus > 0 ? cus : 1)));
    switch (P.win) {
        case 8: hipLaunchKernelGGL(k_tab_fold<8>, grid, dim3(TF_BLOCK), 0, s, P, min_nw); break;
        case 16: hipLaunchKernelGGL(k_tab_fold<16>, grid, dim3(TF_BLOCK), 0, s, P, min_nw); break;
        case 32: hipLaunchKernelGGL(k_tab_fold<32>, grid, dim3(TF_BLOCK), 0, s, P, min_nw); break;
        case 64: hipLaunchKernelGGL(k_tab_fold<64>, grid, dim3(TF_BLOCK), 0, s, P, min_nw); break;
        default: return hipErrorInvalidValue;
    }
    if (P.tab_slack) hipLaunchKernelGGL(k_tab_reset, dim3(1), dim3(1), 0, s, P, min_nw);  // k_fold is skipped
    return hipGetLastError();
}

hipError_t launch_tab_build(const Params& P, hipStream_t s) {
    if (!P.tab) return hipSuccess;
    const dim3 grid((unsigned)((P.m + 63) / 64), (unsigned)((P.n + 63) / 64));
    hipLaunchKernelGGL(k_tab_build, grid, dim3(256), 0, s, P);
    return hipGetLastError();
}

constexpr int TAB_BLOCK = 512;

hipError_t tab_loop_prepare(const Params& P, int cus, int grid_hint, LoopCfg& c) {
    c.ok = false;
    c.block = TAB_BLOCK;
    c.lds_r = false;
    c.lds_bytes = 0;
    if (!P.tab || P.win > TKW) return hipSuccess;
    constexpr int W = TAB_BLOCK / 64;
    const int64_t cols = P.ns;  // one rank: the non-basic list keeps n - m entries
    // the fewest workgroups (cheapest grid barrier: measured 1.3 us at 64,
    // 3.6 us at 256, tools/barrier_bench.hip) whose caches fit: at most one
    // column slot and one row per lane, LDS <= 150 KiB
    auto fits = [&](int g, int& cpw, int& rw) {
        const int64_t cp = (cols + (int64_t)g * W - 1) / ((int64_t)g * W);
        const int64_t r = ((P.m + g - 1) / g + W - 1) / W;
        cpw = (int)std::max<int64_t>(cp, 1);
        rw = (int)std::max<int64_t>(r, 1);
        const int64_t qsl = ((P.L + g - 1) / g + 1) / 2 * 2;  // Qrows slice: one element per thread
        return cp <= 64 && r <= 64 && qsl <= TAB_BLOCK && g <= TAB_BLOCK && TabCache<W>::bytes(cpw, rw) <= 150 * 1024;
    };
    int best = 0, cpw = 0, rw = 0;
    if (grid_hint > 0) {
        if (grid_hint <= cus && fits(grid_hint, cpw, rw)) best = grid_hint;
    } else {
        for (int g : {32, 48, 64, 96, 128, 192, 256, cus}) {
            if (g <= cus && fits(g, cpw, rw)) {
                best = g;
                break;
            }
        }
    }
    if (!best) return hipSuccess;
    c.grid = best;
    c.cpw = cpw;
    c.rw = rw;
    c.lds_bytes = TabCache<W>::bytes(cpw, rw);
    int dev = 0, coop = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    e = hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, dev);
    if (e != hipSuccess) return e;
    if (!coop) return hipSuccess;
    const void* fn = reinterpret_cast<const void*>(&k_tab_loop<TAB_BLOCK>);
    e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)c.lds_bytes);
    if (e != hipSuccess) return e;
    int per_cu = 0;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_tab_loop<TAB_BLOCK>, TAB_BLOCK, c.lds_bytes);
    if (e != hipSuccess) return e;
    c.ok = per_cu >= 1;
    return hipSuccess;
}

void tab_loop_partial_bytes(const LoopCfg& c, size_t* xp, size_t* xu) {
    *xp = 16 * TAB_PP_FIELDS * (size_t)c.grid;
    *xu = 16 * TAB_UP_FIELDS * (size_t)c.grid;
}

hipError_t launch_tab_loop(const Params& P, const LoopArgs& a, const LoopCfg& c, hipStream_t s) {
    int cpw = c.cpw, rw = c.rw;
    void* args[] = {const_cast<Params*>(&P), const_cast<LoopArgs*>(&a), &cpw, &rw};
    // plain launch of a co-resident grid (c.grid <= CUs, per_cu >= 1): the
    // barriers and hand-offs are our own, see launch_loop
    return hipLaunchKernel(reinterpret_cast<const void*>(&k_tab_loop<TAB_BLOCK>), dim3(loop_grid_launched(c.grid, a.call_launch)),
                           dim3(c.block), args, (size_t)c.lds_bytes, s);
}

}  // namespace spx

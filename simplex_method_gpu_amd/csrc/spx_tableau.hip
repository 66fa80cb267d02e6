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
// k_tab_build rebuilds T_w = B_w A after a reinversion or a warm start.
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

// Workgroup = 4 waves; wave w owns TJ x 16 columns of T_w (its Wt fragments,
// the MFMA A operand, lane: Wt[j0 + cl][4 s + kr], stay in registers) and
// walks its row range 16 rows at a time: the U fragment (B operand, lane:
// U[i + cl][4 s + kr], an L2 hit: U is m x KW) and the TJ accumulator tiles
// of T_w (lane: T_w[i + cl, j0 + 16 jt + kr + 4 r]) of the next row block are
// loaded before this block's ceil(nf/4) x TJ v_mfma_f64_16x16x4f64.  T_w is
// read and written once per fold.
template <int KW, int TJ>
__global__ __launch_bounds__(256) void k_tab_fold(Params P, int min_nw) {
    const DevState* st = P.st;
    const int nw = st->nw;
    if (nw < min_nw || nw < 2) return;
    const int nf = nw - 1;
    constexpr int KS = KW / 4;
    const int ks = (nf + 3) / 4;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int cl = lane & 15, kr = lane >> 4;
    const int64_t m = P.m, n = P.n, L = P.L;
    const double* __restrict__ U = P.U;
    const double* __restrict__ Wt = P.Wt;
    double* __restrict__ T = P.T;
    const int64_t cb = (int64_t)blockIdx.y * (4 * 16 * TJ);  // this workgroup's columns

    if (blockIdx.x == 0) {  // dw[j] += sum_{t<nf} SY[t] Wt[j][t], fixed t order
        for (int64_t j = cb + tid; j < cb + 4 * 16 * TJ && j < n; j += 256) {
            double d = 0.0;
            for (int t = 0; t < nf; ++t) d = fma(P.SY[t], Wt[j * KW + t], d);
            P.dw[j] += d;
        }
    }
    const int64_t j0 = cb + (int64_t)wave * 16 * TJ;
    const int64_t per = ((m + gridDim.x - 1) / gridDim.x + 15) / 16 * 16;
    const int64_t i_lo = (int64_t)blockIdx.x * per;
    const int64_t i_hi = (i_lo + per < m) ? i_lo + per : m;
    if (j0 >= n || i_lo >= i_hi) return;

    double wf[TJ][KS];
#pragma unroll
    for (int jt = 0; jt < TJ; ++jt) {
        const int64_t j = j0 + 16 * jt + cl;
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const int t = 4 * s + kr;
            wf[jt][s] = (j < n && t < nf) ? Wt[j * KW + t] : 0.0;
        }
    }
    bool cok[TJ][4];
#pragma unroll
    for (int jt = 0; jt < TJ; ++jt)
#pragma unroll
        for (int r = 0; r < 4; ++r) cok[jt][r] = j0 + 16 * jt + kr + 4 * r < n;
    auto load = [&](int64_t i0, double (&uf)[KS], dbl4 (&acc)[TJ]) {
        const int64_t i = i0 + cl;
        const bool iok = i < i_hi;
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const int t = 4 * s + kr;
            uf[s] = (iok && t < nf) ? U[i * KW + t] : 0.0;
        }
#pragma unroll
        for (int jt = 0; jt < TJ; ++jt)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                acc[jt][r] = (iok && cok[jt][r]) ? T[(j0 + 16 * jt + kr + 4 * r) * L + i] : 0.0;
    };
    double uf[KS];
    dbl4 acc[TJ];
    load(i_lo, uf, acc);
    for (int64_t i0 = i_lo; i0 < i_hi; i0 += 16) {
        double un[KS];
        dbl4 an[TJ];
        const bool more = i0 + 16 < i_hi;
        if (more) load(i0 + 16, un, an);
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            if (s < ks) {
#pragma unroll
                for (int jt = 0; jt < TJ; ++jt)
                    acc[jt] = __builtin_amdgcn_mfma_f64_16x16x4f64(wf[jt][s], uf[s], acc[jt], 0, 0, 0);
            }
        }
        const int64_t i = i0 + cl;
        if (i < i_hi) {
#pragma unroll
            for (int jt = 0; jt < TJ; ++jt)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    if (cok[jt][r]) T[(j0 + 16 * jt + kr + 4 * r) * L + i] = acc[jt][r];
        }
        if (more) {
#pragma unroll
            for (int s = 0; s < KS; ++s) uf[s] = un[s];
#pragma unroll
            for (int jt = 0; jt < TJ; ++jt) acc[jt] = an[jt];
        }
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
// Persistent tableau loop: whole passes in ONE cooperative launch, two grid
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
//   A  lane c prices column c: T_w[q, j] (one gather per wave, with the
//      re-cache of list slots the last pivot changed) and the window sums
//      from LDS; workgroup argmin -> partial WITH the candidate's window
//      row.                                                    -> barrier 1
//   B  every workgroup loads all pricing partials and rows in one round
//      trip (same p everywhere, Wt[p][.] with it); lane r: alpha_i from
//      T_w[i,p] and its LDS row; x_b; ratio test -> partial WITH the
//      candidate's eta row U[i][.].                            -> barrier 2
//   C  every workgroup loads all ratio partials and rows in one round trip
//      (q, s_y, and U[q][.] for the next pricing); workgroup 0 writes the
//      bookkeeping; owners note the two list slots the pivot changed; the
//      new pending base row B_w[q,:] goes to Qrows for k_fold, one slice
//      per workgroup.
// Global copies of everything cached (Wt, U, W, x_b, alpha) are written as
// they change, so the two-kernel passes, the folds and readbacks see the
// same state.
// ---------------------------------------------------------------------------
constexpr int TKW = 64;
constexpr int TKP = TKW + 1;  // LDS row pitch (doubles): lane-per-row reads hit distinct banks
#ifndef SPX_TAB_CLK
#define SPX_TAB_CLK 0  // diagnostic stamp placement: 0 = phases A / B / C
#endif

struct alignas(16) TabPP {  // pricing partial + the candidate's window row
    double val;
    int64_t idx;
    double w;
    double e;
    int64_t slot;
    int64_t pad;
    double row[TKW];
};
struct alignas(16) TabUP {  // ratio-test partial + the candidate's eta row
    UpdPartial h;
    double row[TKW];
};

struct TabPick {  // merged pricing candidate and the partial it came from
    double val;
    int64_t idx;
    double w, e;
    int64_t slot;
    int32_t g;
};
__device__ __forceinline__ void pick_merge(TabPick& a, const TabPick& b) {
    if (argmin_better(b.val, b.idx, a.val, a.idx)) a = b;
}
__device__ __forceinline__ TabPick pick_shfl_xor(const TabPick& v, int off) {
    TabPick o;
    o.val = __shfl_xor(v.val, off, 64);
    o.idx = __shfl_xor(v.idx, off, 64);
    o.w = __shfl_xor(v.w, off, 64);
    o.e = __shfl_xor(v.e, off, 64);
    o.slot = __shfl_xor(v.slot, off, 64);
    o.g = __shfl_xor(v.g, off, 64);
    return o;
}
// ratio-test merge carrying the source partial (UpdPartial::pad) with the winner
__device__ __forceinline__ void tup_merge(UpdPartial& a, const UpdPartial& b) {
    const bool take = argmin_better(b.theta, b.idx, a.theta, a.idx);
    upd_merge(a, b);
    if (take) a.pad = b.pad;
}
__device__ __forceinline__ UpdPartial tup_shfl_xor(const UpdPartial& v, int off) {
    UpdPartial o = upd_shfl_xor(v, off);
    o.pad = __shfl_xor(v.pad, off, 64);
    return o;
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

// TPR: partial-row doubles per loading thread (64 / (BLOCK / G) at most)
template <int BLOCK, int TPR>
__global__ __launch_bounds__(BLOCK) void k_tab_loop(Params P, LoopArgs La, int cpw, int rw) {
    constexpr int WAVES = BLOCK / 64;
    __shared__ TabLds<WAVES> S;
    __shared__ int s_ok;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const TabCache<WAVES> C(smem, cpw);
    TabPP* const XP = reinterpret_cast<TabPP*>(La.xp);
    TabUP* const XU = reinterpret_cast<TabUP*>(La.xu);
    DevState* st = P.st;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int G = (int)gridDim.x;
    const bool wg0 = blockIdx.x == 0;
    const int64_t L = P.L, m = P.m, n = P.n;
    const int KW = P.win;

    int64_t it = st->iter;
    const int64_t it0 = it;
    const int64_t limit = st->limit;
    if (st->status != ST_RUNNING || it >= limit) return;
    int nw = st->nw;
    if (nw >= KW) return;  // the host folds first
    int64_t q = st->q;
    double aq = st->aq;
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
    // partial loading: tpp threads per partial, each a slice of its row
    const int tpp = BLOCK / G;
    const int pg = tid / tpp, psub = tid - pg * tpp;
    const bool pok = pg < G;
    const int per = (TKW + tpp - 1) / tpp;
    // this workgroup's slice of a base row (Qrows staging for k_fold)
    const int64_t qsl = ((L + G - 1) / G + 1) / 2 * 2;
    const int64_t qk0 = (int64_t)blockIdx.x * qsl;
    const int64_t qk1 = (qk0 + qsl < L) ? qk0 + qsl : L;

    // ---- prologue: window scalars, column and row caches
    if (tid < KW) {
        S.SY[tid] = (tid < nw) ? P.SY[tid] : 0.0;
        S.Uq[tid] = (nw > 0 && tid < nw - 1) ? P.U[q * KW + tid] : 0.0;
    }
    if (nw > 0) {  // the pending pivot's base row (B_w changed at the last fold)
        for (int64_t k = qk0 + tid; k < qk1; k += BLOCK) P.Qrows[(int64_t)(nw - 1) * L + k] = P.B0[q * L + k];
        if (wg0 && tid < nw - 1) P.Urows[(int64_t)(nw - 1) * KW + tid] = P.U[q * KW + tid];
    }
    if (cv) {
        const int32_t j = P.nb_list[vid + lane * stride];
        C.col[ls] = j;
        C.dwc[ls] = P.dw[j];
        C.wc[ls] = P.devex ? P.W[j] : 1.0;
    }
    __syncthreads();
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
    __syncthreads();
    uint32_t target = 0;
    // list slots the last pivot changed, owned by this wave: re-cached at the
    // start of the next pricing phase (their window rows then are visible)
    int rc_ls0 = -1, rc_ls1 = -1;
    int64_t rc_j0 = 0, rc_j1 = 0;

    for (int pass = 0; pass < La.npasses && it < limit; ++pass) {
        const bool pend = nw > 0;
        const int tau = nw - 1;
        unsigned long long* clk = (La.clock && wg0 && tid == 0) ? La.clock + 3 * (int64_t)pass : nullptr;
        if (clk) clk[0] = rtime();

        // ================= phase A: pricing, lane c <-> column slot c
        // (issued together: the re-cache loads, T_w[q, j] of every column,
        // and the x_b update's s_x = r_tau . b for phase B)
        if (rc_ls0 >= 0 || rc_ls1 >= 0) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int lsn = h ? rc_ls1 : rc_ls0;
                if (lsn < 0) continue;
                const int64_t jn = h ? rc_j1 : rc_j0;
                C.wt[(int64_t)lsn * TKP + lane] = (lane < tau) ? ld_agent(&P.Wt[jn * KW + lane]) : 0.0;
                if (lane == 0) {
                    C.col[lsn] = (int32_t)jn;
                    C.dwc[lsn] = P.dw[jn];
                    C.wc[lsn] = P.devex ? ld_agent(&P.W[jn]) : 1.0;
                }
            }
            rc_ls0 = rc_ls1 = -1;
        }
        double sxw = 0.0;
        if (pend) {
            sxw = lane < tau ? S.Uq[lane] * ld_agent(&P.Wt[n * KW + lane]) : 0.0;
            sxw = P.xw[q] + wave_sum(sxw);
            if (wg0 && tid == 0) st_agent(&P.Wt[n * KW + tau], sxw);
        }
        TabPick best{INFINITY, INT64_MAX, 0.0, 0.0, -1, (int32_t)blockIdx.x};
        {
            const int64_t j = cv ? (int64_t)C.col[ls] : 0;
            const double tq = (pend && cv) ? P.T[j * L + q] : 0.0;
            const double dv = cv ? C.dwc[ls] : 0.0;
            const double* wrow = C.wt + (int64_t)ls * TKP;
            double w, e;
            tab_price_column(tq, dv, cv ? tau : -1, S.SY, S.Uq, [&](int s2) { return wrow[s2]; }, w, e);
#if SPX_TAB_CLK == 1  // diagnostic: {pass start, column done, barrier 1 done}
            if (clk) clk[1] = rtime();
#endif
            if (cv) {
                if (pend) {
                    C.wt[(int64_t)ls * TKP + tau] = w;
                    st_agent(&P.Wt[j * KW + tau], w);
                }
                double key = e;
                if (P.devex) {  // include/simplex.h SPX_PRICING_DEVEX, as k_price
                    double wt = C.wc[ls];
                    if (pend) {
                        if (j == dleave) wt = fmax(dwp / (aq * aq), 1.0);
                        else {
                            const double g = w / aq;
                            wt = fmax(wt, g * g * dwp);
                        }
                        C.wc[ls] = wt;
                        st_agent(&P.W[j], wt);
                    }
                    key = (e < -P.eps) ? -(e * e) / wt : INFINITY;
                }
                best = TabPick{key, j, w, e, (int64_t)vid + (int64_t)lane * stride, (int32_t)(wave * 64 + lane)};
            }
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) pick_merge(best, pick_shfl_xor(best, off));
        }
        if (lane == 0) S.ppick[wave] = best;
        __syncthreads();
        {
            TabPick w = S.ppick[0];
            for (int i = 1; i < WAVES; ++i) pick_merge(w, S.ppick[i]);
            // the winning lane's wave copies its window row into the partial
            TabPP* d = &XP[blockIdx.x];
            if (w.idx != INT64_MAX && wave == (w.g >> 6)) {
                const int wls = wave * cpw + (w.g & 63);
                st_agent(&d->row[lane], C.wt[(int64_t)wls * TKP + lane]);
            }
            if (tid == 0) {
                st_agent(&d->val, w.val);
                st_agent(&d->idx, w.idx);
                st_agent(&d->w, w.w);
                st_agent(&d->e, w.e);
                st_agent(&d->slot, w.slot);
            }
        }
        target += (uint32_t)G;
        if (!grid_sync(La.ls, target, &s_ok)) return;
#if SPX_TAB_CLK != 2
        if (clk) clk[SPX_TAB_CLK == 1 ? 2 : 1] = rtime();
#endif

        // ================= phase B: entering column (all partials and rows
        // in one round trip), FTRAN + ratio test
        {
            TabPick w{INFINITY, INT64_MAX, 0.0, 0.0, -1, 0};
            double rowv[TPR];
            if (pok) {
                const TabPP* d = &XP[pg];
                if (psub == 0) w = TabPick{ld_agent(&d->val), ld_agent(&d->idx), ld_agent(&d->w), ld_agent(&d->e),
                                           ld_agent(&d->slot), pg};
#pragma unroll
                for (int k = 0; k < TPR; ++k)
                    if (k < per && psub * per + k < TKW) rowv[k] = ld_agent(&d->row[psub * per + k]);
            }
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) pick_merge(w, pick_shfl_xor(w, off));
            if (lane == 0) S.ppick[wave] = w;
            __syncthreads();
            TabPick t = S.ppick[0];
            for (int i = 1; i < WAVES; ++i) pick_merge(t, S.ppick[i]);
            if (pok && pg == t.g && t.idx != INT64_MAX) {
#pragma unroll
                for (int k = 0; k < TPR; ++k)
                    if (k < per && psub * per + k < TKW) S.Wp[psub * per + k] = rowv[k];
            }
            if (tid == 0) S.pwin = t;
            __syncthreads();
        }
        const TabPick pw = S.pwin;
        const int64_t p = pw.idx;
        const double min_e = pw.val;
#if SPX_TAB_CLK == 2  // diagnostic: {pass start, barrier 1 done, p and Wt[p] known}
        if (clk) clk[1] = rtime();
#endif
        if (no_entering(P, min_e, p)) {  // OptimumFound (v4:299-302)
            if (wg0 && tid == 0) {
                st->p = p;
                st->min_e = P.devex ? pw.e : min_e;
                st->status = ST_OPTIMAL;
            }
            break;
        }
        // the winner's own window entry Wt[p][tau] (the row copy may predate it)
        if (tid == 0 && pend) S.Wp[tau] = pw.w;
        {
            double* a_new = (it & 1) ? P.alpha0 : P.alpha1;
            const bool upd_x = xb_applied < it;
            const double tcol = rv ? P.T[p * L + irow] : 0.0;
            const double s_x = upd_x ? sxw : 0.0;
            __syncthreads();
            UpdPartial wp = upd_empty();
            if (rv) {
                const double ei = pend ? eta_entry(apr, irow, q, aq) : 0.0;
                const double* urow = C.ur + (int64_t)lr * TKP;
                const double a = tab_ftran_row(tcol, tau, ei, S.Wp, [&](int s2) { return urow[s2]; });
                if (pend) {
                    C.ur[(int64_t)lr * TKP + tau] = ei;
                    st_agent(&P.U[irow * KW + tau], ei);
                    st_agent(&P.Wt[bxr * KW + tau], (irow == q) ? aq : 0.0);
                }
                if (upd_x) {
                    xbr = fma(s_x, ei, xbr);
                    P.x_b[irow] = xbr;
                }
                apr = a;
                a_new[irow] = a;
                wp.theta = ratio_key(P, xbr, a);
                wp.idx = irow;
                wp.nonpos = !(a > P.piv_tol);
                wp.T = cbr * a;
                wp.a_w = a;
                wp.cb_w = cbr;
                wp.bix_w = bxr;
                wp.pad = wave * 64 + lane;
            }
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const UpdPartial o = tup_shfl_xor(wp, off);
                UpdPartial lo = (lane & off) ? o : wp;
                const UpdPartial hi = (lane & off) ? wp : o;
                tup_merge(lo, hi);
                wp = lo;
            }
            if (lane == 0) S.ured[wave] = wp;
            __syncthreads();
            UpdPartial w = S.ured[0];
            for (int i = 1; i < WAVES; ++i) tup_merge(w, S.ured[i]);
            TabUP* d = &XU[blockIdx.x];
            if (w.idx >= row0 && w.idx < row1 && wave == (int)(w.pad >> 6)) {
                const int wlr = wave * rw + (int)(w.pad & 63);
                st_agent(&d->row[lane], C.ur[(int64_t)wlr * TKP + lane]);
            }
            if (tid == 0) {
                st_agent(&d->h.theta, w.theta);
                st_agent(&d->h.idx, w.idx);
                st_agent(&d->h.nonpos, w.nonpos);
                st_agent(&d->h.T, w.T);
                st_agent(&d->h.a_w, w.a_w);
                st_agent(&d->h.cb_w, w.cb_w);
                st_agent(&d->h.bix_w, w.bix_w);
            }
        }
        target += (uint32_t)G;
        if (!grid_sync(La.ls, target, &s_ok)) return;
#if SPX_TAB_CLK != 1
        if (clk) clk[2] = rtime();
#endif

        // ================= phase C: leaving row (all partials and eta rows in
        // one round trip), s_y, bookkeeping (update_tail)
        {
            UpdPartial w = upd_empty();
            double rowv[TPR];
            if (pok) {
                const TabUP* d = &XU[pg];
                if (psub == 0) {
                    w.theta = ld_agent(&d->h.theta);
                    w.idx = ld_agent(&d->h.idx);
                    w.nonpos = ld_agent(&d->h.nonpos);
                    w.T = ld_agent(&d->h.T);
                    w.a_w = ld_agent(&d->h.a_w);
                    w.cb_w = ld_agent(&d->h.cb_w);
                    w.bix_w = ld_agent(&d->h.bix_w);
                    w.pad = pg;
                }
#pragma unroll
                for (int k = 0; k < TPR; ++k)
                    if (k < per && psub * per + k < TKW) rowv[k] = ld_agent(&d->row[psub * per + k]);
            }
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const UpdPartial o = tup_shfl_xor(w, off);
                UpdPartial lo = (lane & off) ? o : w;
                const UpdPartial hi = (lane & off) ? w : o;
                tup_merge(lo, hi);
                w = lo;
            }
            if (lane == 0) S.ured[wave] = w;
            __syncthreads();
            UpdPartial t = S.ured[0];
            for (int k2 = 1; k2 < WAVES; ++k2) tup_merge(t, S.ured[k2]);
            // U[q][0..tau] of the new pending pivot, for the next pricing
            if (pok && pg == (int)t.pad && t.idx >= 0 && t.idx < m) {
#pragma unroll
                for (int k = 0; k < TPR; ++k)
                    if (k < per && psub * per + k < TKW) S.Uq[psub * per + k] = rowv[k];
            }
            if (tid == 0) S.uwin = t;
            __syncthreads();
        }
        const UpdPartial t = S.uwin;
        if (t.nonpos == m || t.idx < 0 || t.idx >= m) {  // Unbounded (v4:319-322)
            if (wg0 && tid == 0) {
                st->p = p;
                st->min_e = min_e;
                st->status = ST_UNBOUNDED;
            }
            break;
        }
        const int64_t qn = t.idx, leave = t.bix_w;
        const double aqn = t.a_w, c_p = P.c[p];
        const double s_y = y_scalar(t.T, aqn, t.cb_w, c_p);
        const int64_t kp = pw.slot;
        const double wp_new = P.devex ? ld_agent(&P.W[p]) : 0.0;
        if (wg0 && tid == 0) {
            if (kp != cnt - 1) {
                st_agent(&P.nb_list[kp], (int32_t)lastv);
                st_agent(&P.nb_pos[lastv], (int32_t)kp);
            }
            st_agent(&P.nb_pos[p], (int32_t)-1);
            st_agent(&P.nb_list[cnt - 1], (int32_t)leave);
            st_agent(&P.nb_pos[leave], (int32_t)(cnt - 1));
            st_agent(&P.c_B[qn], c_p);
            st_agent(&P.b_ixs[qn], p);
            P.SY[nw] = s_y;
            st->aq = aqn;
            st->s_y = s_y;
            st->nw = nw + 1;
            st->xb_applied = it;
            st->p = p;
            st->q = qn;
            st->min_e = P.devex ? pw.e : min_e;
            st->iter = it + 1;
            if (P.devex) {
                st->leave = leave;
                st->wp = wp_new;
            }
        }
        if (wg0 && tid < nw) P.Urows[(int64_t)nw * KW + tid] = S.Uq[tid];
        if (rv && irow == qn) {  // the pivot's row: its basis entry (v4:339-342)
            bxr = p;
            cbr = c_p;
        }
        // the two list slots the pivot changed (swap-remove of p: slot kp <-
        // lastv; append of leave: slot cnt-1); their owners re-cache them at
        // the start of the next pricing phase
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int64_t slot = h ? (int64_t)cnt - 1 : kp;
            if (h == 0 && kp == cnt - 1) continue;
            if ((int)(slot % stride) != vid) continue;
            const int lsn = wave * cpw + (int)(slot / stride);
            if (h) {
                rc_ls1 = lsn;
                rc_j1 = leave;
            } else {
                rc_ls0 = lsn;
                rc_j0 = lastv;
            }
        }
        lastv = leave;
        // the new pending pivot (tau' = nw): its base row into Qrows (this
        // workgroup's slice)
        for (int64_t k = qk0 + tid; k < qk1; k += BLOCK) P.Qrows[(int64_t)nw * L + k] = P.B0[qn * L + k];
        if (tid == 0) S.SY[nw] = s_y;
        q = qn;
        aq = aqn;
        xb_applied = it;
        dleave = leave;
        dwp = wp_new;
        ++nw;
        ++it;
        __syncthreads();
    }
    if (wg0 && tid == 0) La.ls->passes = (int32_t)(it - it0);
}

}  // namespace

hipError_t launch_tab_fold(const Params& P, int min_nw, int cus, hipStream_t s) {
    if (!P.tab) return hipSuccess;
    constexpr int TJ = 2;
    const int64_t gy = (P.n + 64 * TJ - 1) / (64 * TJ);
    // rows split so that the grid has about 2 workgroups per CU (8 waves)
    int64_t gx = (2 * (int64_t)cus + gy - 1) / gy;
    const int64_t maxx = (P.m + 15) / 16;
    if (gx > maxx) gx = maxx;
    if (gx < 1) gx = 1;
    const dim3 grid((unsigned)gx, (unsigned)gy);
    switch (P.win) {
        case 8: hipLaunchKernelGGL((k_tab_fold<8, TJ>), grid, dim3(256), 0, s, P, min_nw); break;
        case 16: hipLaunchKernelGGL((k_tab_fold<16, TJ>), grid, dim3(256), 0, s, P, min_nw); break;
        case 32: hipLaunchKernelGGL((k_tab_fold<32, TJ>), grid, dim3(256), 0, s, P, min_nw); break;
        case 64: hipLaunchKernelGGL((k_tab_fold<64, TJ>), grid, dim3(256), 0, s, P, min_nw); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_tab_build(const Params& P, hipStream_t s) {
    if (!P.tab) return hipSuccess;
    const dim3 grid((unsigned)((P.m + 63) / 64), (unsigned)((P.n + 63) / 64));
    hipLaunchKernelGGL(k_tab_build, grid, dim3(256), 0, s, P);
    return hipGetLastError();
}

constexpr int TAB_BLOCK = 512;

// the instantiation whose per-thread partial-row slice covers G partials
static const void* tab_loop_fn(int g) {
    const int per = (TKW + TAB_BLOCK / g - 1) / (TAB_BLOCK / g);
    if (per <= 8) return reinterpret_cast<const void*>(&k_tab_loop<TAB_BLOCK, 8>);
    if (per <= 16) return reinterpret_cast<const void*>(&k_tab_loop<TAB_BLOCK, 16>);
    return reinterpret_cast<const void*>(&k_tab_loop<TAB_BLOCK, 32>);
}

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
        return cp <= 64 && r <= 64 && g <= TAB_BLOCK / 2 && TabCache<W>::bytes(cpw, rw) <= 150 * 1024;
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
    const void* fn = tab_loop_fn(best);
    e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)c.lds_bytes);
    if (e != hipSuccess) return e;
    int per_cu = 0;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, TAB_BLOCK, c.lds_bytes);
    if (e != hipSuccess) return e;
    c.ok = per_cu >= 1;
    return hipSuccess;
}

void tab_loop_partial_bytes(const LoopCfg& c, size_t* xp, size_t* xu) {
    *xp = sizeof(TabPP) * (size_t)c.grid;
    *xu = sizeof(TabUP) * (size_t)c.grid;
}

hipError_t launch_tab_loop(const Params& P, const LoopArgs& a, const LoopCfg& c, hipStream_t s) {
    int cpw = c.cpw, rw = c.rw;
    void* args[] = {const_cast<Params*>(&P), const_cast<LoopArgs*>(&a), &cpw, &rw};
    return hipLaunchCooperativeKernel(tab_loop_fn(c.grid), dim3(c.grid), dim3(c.block), args, (unsigned)c.lds_bytes,
                                      s);
}

}  // namespace spx

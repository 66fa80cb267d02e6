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

#include "spx_common.h"
#include "spx_fold.h"
#include "spx_grid.h"
#include "spx_loop.h"
#include "spx_tableau.h"

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
// Persistent tableau loop: whole passes in ONE cooperative launch (one
// workgroup per CU), two grid barriers per pass, as k_loop (spx_loop.h) does
// for the eta window — but a tableau pass moves a few MB, not 537 MB, so its
// kernel boundaries, not its bytes, are what a two-kernel pass pays for.
//   A  prices the workgroup's share of the non-basic list (k_price WM 3, term
//      for term: one wave per column, lane s holding Wt[j][s]).  -> barrier 1
//   B  every workgroup reduces the pricing partials (same order, same p),
//      then alpha_i = T_w[i,p] + sum_tau U[i][tau] Wt[p][tau] for its rows,
//      the pending eta column into U, x_b, ratio test (k_update, tableau
//      branch, term for term).                                 -> barrier 2
//   C  every workgroup reduces the ratio-test partials (q, s_y); workgroup 0
//      writes the bookkeeping; the new pending base row B_w[q,:] goes to
//      Qrows for k_fold, one slice per workgroup.
// The last pivot's non-basic-list change is applied as a local patch until
// workgroup 0's writes are visible (after the next barrier).
// ---------------------------------------------------------------------------
constexpr int TKW = 64;

template <int WAVES>
struct TabLds {
    double SY[TKW];
    double Uq[TKW];
    PricePartial pred[WAVES];
    UpdPartial ured[WAVES];
    PricePartial pwin;
    UpdPartial uwin;
    int64_t kp, lastv;
};

__device__ __forceinline__ void tprice_merge(PricePartial& a, const PricePartial& b) {
    if (argmin_better(b.val, b.idx, a.val, a.idx)) a = b;
}

template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_tab_loop(Params P, LoopArgs La) {
    constexpr int WAVES = BLOCK / 64;
    constexpr int TPC = 4;  // columns per wave in flight (k_price WM 3)
    __shared__ TabLds<WAVES> S;
    __shared__ int s_ok;
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
    int64_t dleave = st->leave;
    double dwp = st->wp;
    // this workgroup's slice of a base row (Qrows staging for k_fold)
    const int64_t qsl = ((L + G - 1) / G + 1) / 2 * 2;
    const int64_t qk0 = (int64_t)blockIdx.x * qsl;
    const int64_t qk1 = (qk0 + qsl < L) ? qk0 + qsl : L;
    if (tid < KW) {
        S.SY[tid] = (tid < nw) ? P.SY[tid] : 0.0;
        S.Uq[tid] = (nw > 0 && tid < nw - 1) ? ld_agent(&P.U[q * KW + tid]) : 0.0;
    }
    if (nw > 0) {  // the pending pivot's base row (B_w changed at the last fold)
        for (int64_t k = qk0 + tid; k < qk1; k += BLOCK) P.Qrows[(int64_t)(nw - 1) * L + k] = P.B0[q * L + k];
        if (wg0 && tid < nw - 1) P.Urows[(int64_t)(nw - 1) * KW + tid] = ld_agent(&P.U[q * KW + tid]);
    }
    __syncthreads();
    int pk1 = -1, pk2 = -1;
    int64_t pv1 = 0, pv2 = 0;
    auto list_at = [&](int idx) -> int64_t {
        return (idx == pk1) ? pv1 : ((idx == pk2) ? pv2 : (int64_t)ld_agent(&P.nb_list[idx]));
    };
    uint32_t target = 0;
    const int64_t rpw = (m + G - 1) / G;
    const int64_t row0 = (int64_t)blockIdx.x * rpw;
    const int64_t row1 = (row0 + rpw < m) ? row0 + rpw : m;
    const int stride = G * WAVES;
    const int idx0 = (int)blockIdx.x * WAVES + wave;

    for (int pass = 0; pass < La.npasses && it < limit; ++pass) {
        const bool pend = nw > 0;
        const int tau = nw - 1;
        unsigned long long* clk = (La.clock && wg0 && tid == 0) ? La.clock + 3 * (int64_t)pass : nullptr;
        if (clk) clk[0] = rtime();

        // ================= phase A: pricing (k_price, WM 3)
        double uq = 0.0, syl = 0.0, syp = 0.0;
        if (pend) {
            if (lane < tau) {
                uq = S.Uq[lane];
                syl = S.SY[lane];
            }
            syp = S.SY[tau];
        }
        double best = INFINITY, bw = 0.0, be = 0.0;
        int64_t bj = INT64_MAX;
        for (int idx = idx0; idx < cnt; idx += stride * TPC) {
            int64_t jj[TPC];
            double wv[TPC], tq[TPC], dv[TPC], sa[TPC], wn[TPC];
#pragma unroll
            for (int c = 0; c < TPC; ++c) {
                const int ic = idx + c * stride;
                jj[c] = ic < cnt ? list_at(ic) : -1;
            }
#pragma unroll
            for (int c = 0; c < TPC; ++c) {
                const int64_t j = jj[c] < 0 ? 0 : jj[c];
                wv[c] = (pend && lane < tau) ? ld_agent(&P.Wt[j * KW + lane]) : 0.0;
                tq[c] = pend ? P.T[j * L + q] : 0.0;
                dv[c] = P.dw[j];
                sa[c] = syl * wv[c];
                wn[c] = uq * wv[c];
            }
            if (pend) {
#pragma unroll
                for (int off = 32; off > 0; off >>= 1)
#pragma unroll
                    for (int c = 0; c < TPC; ++c) {
                        const double ta = __shfl_xor(sa[c], off, 64);
                        const double tb = __shfl_xor(wn[c], off, 64);
                        sa[c] += ta;
                        wn[c] += tb;
                    }
            }
#pragma unroll
            for (int c = 0; c < TPC; ++c) {
                if (jj[c] < 0) continue;
                const int64_t j = jj[c];
                const double w = tq[c] + wn[c];
                if (pend && lane == 0) st_agent(&P.Wt[j * KW + tau], w);
                const double e = pend ? fma(syp, w, dv[c] + sa[c]) : dv[c];
                double key = e;
                if (P.devex) {  // include/simplex.h SPX_PRICING_DEVEX, as k_price
                    double wt = ld_agent(&P.W[j]);
                    if (pend) {
                        if (j == dleave) wt = fmax(dwp / (aq * aq), 1.0);
                        else {
                            const double g = w / aq;
                            wt = fmax(wt, g * g * dwp);
                        }
                        if (lane == 0) st_agent(&P.W[j], wt);
                    }
                    key = (e < -P.eps) ? -(e * e) / wt : INFINITY;
                }
                if (argmin_better(key, j, best, bj)) {
                    best = key;
                    bj = j;
                    bw = w;
                    be = e;
                }
            }
        }
        if (lane == 0) S.pred[wave] = PricePartial{best, bj, bw, be};
        __syncthreads();
        if (tid == 0) {
            PricePartial w = S.pred[0];
            for (int i = 1; i < WAVES; ++i) tprice_merge(w, S.pred[i]);
            PricePartial* d = &La.pp[blockIdx.x];
            st_agent(&d->val, w.val);
            st_agent(&d->idx, w.idx);
            st_agent(&d->w, w.w);
            st_agent(&d->pad, w.pad);
        }
        target += (uint32_t)G;
        if (!grid_sync(La.ls, target, &s_ok)) return;
        if (clk) clk[1] = rtime();

        // ================= phase B: entering column, FTRAN + ratio test
        {
            PricePartial w{INFINITY, INT64_MAX, 0.0, 0.0};
            for (int g = tid; g < G; g += BLOCK) {
                const PricePartial* d = &La.pp[g];
                PricePartial v{ld_agent(&d->val), ld_agent(&d->idx), ld_agent(&d->w), ld_agent(&d->pad)};
                tprice_merge(w, v);
            }
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) {
                PricePartial o{__shfl_xor(w.val, off, 64), __shfl_xor(w.idx, off, 64), __shfl_xor(w.w, off, 64),
                               __shfl_xor(w.pad, off, 64)};
                tprice_merge(w, o);
            }
            if (lane == 0) S.pred[wave] = w;
            __syncthreads();
            if (tid == 0) {
                PricePartial t = S.pred[0];
                for (int i = 1; i < WAVES; ++i) tprice_merge(t, S.pred[i]);
                S.pwin = t;
                if (!no_entering(P, t.val, t.idx)) {
                    S.kp = ld_agent(&P.nb_pos[t.idx]);
                    S.lastv = ld_agent(&P.nb_list[cnt - 1]);
                }
            }
            __syncthreads();
        }
        const int64_t p = S.pwin.idx;
        const double min_e = S.pwin.val;
        if (no_entering(P, min_e, p)) {  // OptimumFound (v4:299-302)
            if (wg0 && tid == 0) {
                st->p = p;
                st->min_e = P.devex ? S.pwin.pad : min_e;
                st->status = ST_OPTIMAL;
            }
            break;
        }
        {
            const int par = (int)(it & 1);
            const double* a_prev = par ? P.alpha1 : P.alpha0;
            double* a_new = par ? P.alpha0 : P.alpha1;
            const bool upd_x = xb_applied < it;
            const double wl = lane < nw ? ld_agent(&P.Wt[p * KW + lane]) : 0.0;
            double sxw = 0.0;
            if (pend) {
                sxw = lane < tau ? ld_agent(&P.U[q * KW + lane]) * ld_agent(&P.Wt[n * KW + lane]) : 0.0;
                sxw = P.xw[q] + wave_sum(sxw);
                if (wg0 && tid == 0) st_agent(&P.Wt[n * KW + tau], sxw);
            }
            const double s_x = upd_x ? sxw : 0.0;
            UpdPartial wp = upd_empty();
            for (int64_t i0 = row0 + wave; i0 < row1; i0 += 2 * WAVES) {
                const int64_t i1 = i0 + WAVES;
                const bool two = i1 < row1;
                double acc[2], cu[2], ei[2], cb[2], xb[2];
                int64_t bix[2];
#pragma unroll
                for (int r = 0; r < 2; ++r) {
                    const int64_t i = r ? (two ? i1 : i0) : i0;
                    acc[r] = lane == 0 ? P.T[p * L + i] : 0.0;
                    ei[r] = pend ? eta_entry(ld_agent(&a_prev[i]), i, q, aq) : 0.0;
                    bix[r] = ld_agent(&P.b_ixs[i]);
                    cb[r] = ld_agent(&P.c_B[i]);
                    xb[r] = P.x_b[i];
                    cu[r] = lane < tau ? ld_agent(&P.U[i * KW + lane]) : (lane == tau ? ei[r] : 0.0);
                    acc[r] = fma(cu[r], wl, acc[r]);
                }
#pragma unroll
                for (int off = 32; off > 0; off >>= 1) {
                    const double t0 = __shfl_xor(acc[0], off, 64);
                    const double t1 = __shfl_xor(acc[1], off, 64);
                    acc[0] += t0;
                    acc[1] += t1;
                }
#pragma unroll
                for (int r = 0; r < 2; ++r) {
                    if (r && !two) break;
                    const int64_t i = r ? i1 : i0;
                    const double a = acc[r];
                    if (pend && lane == 0) {
                        st_agent(&P.Wt[bix[r] * KW + tau], (i == q) ? aq : 0.0);
                        st_agent(&P.U[i * KW + tau], ei[r]);
                    }
                    double x = xb[r];
                    if (upd_x) x = fma(s_x, ei[r], x);
                    if (lane == 0) {
                        st_agent(&a_new[i], a);
                        if (upd_x) P.x_b[i] = x;
                    }
                    const double th = ratio_key(P, x, a);
                    wp.nonpos += !(a > P.piv_tol);
                    wp.T = fma(cb[r], a, wp.T);
                    if (argmin_better(th, i, wp.theta, wp.idx)) {
                        wp.theta = th;
                        wp.idx = i;
                        wp.a_w = a;
                        wp.cb_w = cb[r];
                        wp.bix_w = bix[r];
                    }
                }
            }
            if (lane == 0) S.ured[wave] = wp;
            __syncthreads();
            if (tid == 0) {
                UpdPartial w = S.ured[0];
                for (int i = 1; i < WAVES; ++i) upd_merge(w, S.ured[i]);
                UpdPartial* d = &La.up[blockIdx.x];
                st_agent(&d->theta, w.theta);
                st_agent(&d->idx, w.idx);
                st_agent(&d->nonpos, w.nonpos);
                st_agent(&d->T, w.T);
                st_agent(&d->a_w, w.a_w);
                st_agent(&d->cb_w, w.cb_w);
                st_agent(&d->bix_w, w.bix_w);
            }
        }
        target += (uint32_t)G;
        if (!grid_sync(La.ls, target, &s_ok)) return;
        if (clk) clk[2] = rtime();

        // ================= phase C: leaving row, s_y, bookkeeping (update_tail)
        {
            UpdPartial w = upd_empty();
            for (int g = tid; g < G; g += BLOCK) {
                const UpdPartial* d = &La.up[g];
                UpdPartial v;
                v.theta = ld_agent(&d->theta);
                v.idx = ld_agent(&d->idx);
                v.nonpos = ld_agent(&d->nonpos);
                v.T = ld_agent(&d->T);
                v.a_w = ld_agent(&d->a_w);
                v.cb_w = ld_agent(&d->cb_w);
                v.bix_w = ld_agent(&d->bix_w);
                v.pad = 0;
                upd_merge(w, v);
            }
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) {
                const UpdPartial o = upd_shfl_xor(w, off);
                UpdPartial lo = (lane & off) ? o : w;
                const UpdPartial hi = (lane & off) ? w : o;
                upd_merge(lo, hi);
                w = lo;
            }
            if (lane == 0) S.ured[wave] = w;
            __syncthreads();
            if (tid == 0) {
                UpdPartial t = S.ured[0];
                for (int k2 = 1; k2 < WAVES; ++k2) upd_merge(t, S.ured[k2]);
                S.uwin = t;
            }
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
        const int64_t kp = S.kp, lastv = S.lastv;
        pk1 = (kp != cnt - 1) ? (int)kp : -1;
        pv1 = lastv;
        pk2 = cnt - 1;
        pv2 = leave;
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
            st->min_e = P.devex ? S.pwin.pad : min_e;
            st->iter = it + 1;
            if (P.devex) {
                st->leave = leave;
                st->wp = wp_new;
            }
        }
        // the new pending pivot (tau' = nw): its base row into Qrows (this
        // workgroup's slice) and its U coefficients; LDS copies for pricing
        for (int64_t k = qk0 + tid; k < qk1; k += BLOCK) P.Qrows[(int64_t)nw * L + k] = P.B0[qn * L + k];
        if (tid < nw) {
            const double u = ld_agent(&P.U[qn * KW + tid]);
            S.Uq[tid] = u;
            if (wg0) P.Urows[(int64_t)nw * KW + tid] = u;
        }
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

hipError_t tab_loop_prepare(const Params& P, int cus, LoopCfg& c) {
    c.ok = false;
    c.block = 512;
    c.grid = cus;
    c.lds_r = false;
    c.lds_bytes = 0;
    if (!P.tab || P.win > TKW) return hipSuccess;
    int dev = 0, coop = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    e = hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, dev);
    if (e != hipSuccess) return e;
    if (!coop) return hipSuccess;
    int per_cu = 0;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_tab_loop<512>, 512, 0);
    if (e != hipSuccess) return e;
    c.ok = per_cu >= 1;
    return hipSuccess;
}

hipError_t launch_tab_loop(const Params& P, const LoopArgs& a, const LoopCfg& c, hipStream_t s) {
    void* args[] = {const_cast<Params*>(&P), const_cast<LoopArgs*>(&a)};
    return hipLaunchCooperativeKernel(reinterpret_cast<const void*>(&k_tab_loop<512>), dim3(c.grid), dim3(c.block),
                                      args, 0, s);
}

}  // namespace spx

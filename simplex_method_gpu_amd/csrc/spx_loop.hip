// spx_loop.hip — the persistent eta-window loop kernel (see spx_loop.h).
//
// Arithmetic is that of k_price / k_update in window mode (spx_kernels.hip),
// term for term and in the same per-lane order, so pivot paths match the
// two-kernel loop and the oracle; only the ratio test's T sum (s_y) is
// grouped by this launch's geometry.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdlib.h>

#include "spx_common.h"
#include "spx_loop.h"
#include "spx_grid.h"

namespace spx {

namespace {

constexpr int KWMAX = 64;

template <int WAVES>
struct LoopLds {  // the small shared region after y_w (and the base row)
    double SY[KWMAX];
    double Uq[KWMAX];
    PricePartial pred[WAVES];
    UpdPartial ured[WAVES];
    PricePartial pwin;  // the merged entering candidate
    UpdPartial uwin;    // the merged leaving candidate
    int64_t kp, lastv;  // list slots read in phase B for the pivot's list change
};

__device__ __forceinline__ void price_merge(PricePartial& a, const PricePartial& b) {
    if (argmin_better(b.val, b.idx, a.val, a.idx)) a = b;
}

// Dot-product kernels of one pricing column: the first CH dbl2 chunks per
// lane come from pre[] (loaded ahead), the rest streamed; per-lane sums in
// increasing k (the order k_price uses, so the bits match).
constexpr int CH = 8;
#ifndef SPX_LOOP_CPRE
#define SPX_LOOP_CPRE 0  // first pricing column of a pass loaded ahead (launch start, phase C): measured no gain
#endif

template <bool PEND>
__device__ __forceinline__ void price_column(const dbl2* __restrict__ col, const dbl2* Y, const dbl2* Rw, int64_t L2,
                                             int lane, const dbl2 (&pre)[CH], bool have, double& a0, double& a1,
                                             double& b0, double& b1) {
    int64_t k = lane;
    if (have) {
#pragma unroll
        for (int u = 0; u < CH; ++u) {
            const dbl2 w = Y[lane + u * 64];
            a0 = fma(pre[u].x, w.x, a0);
            a1 = fma(pre[u].y, w.y, a1);
            if constexpr (PEND) {
                const dbl2 r = Rw[lane + u * 64];
                b0 = fma(pre[u].x, r.x, b0);
                b1 = fma(pre[u].y, r.y, b1);
            }
        }
        k += CH * 64;
    }
#ifndef SPX_LOOP_PIPE
#define SPX_LOOP_PIPE 1  // two 8-chunk batches of a column in flight (as k_price)
#endif
    if (SPX_LOOP_PIPE && (L2 & 511) == 0 && L2 > 8 * 64) {
        // the next batch requested before the current one is consumed; the
        // same fma order as the loop below
        int64_t kb = have ? 8 * 64 : 0;
        dbl2 vc[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) vc[u] = ld2<SPX_NT_A>(&col[kb + lane + u * 64]);
        auto consume = [&](int64_t kq) {
#pragma unroll
            for (int h = 0; h < 8; h += 4) {
                dbl2 w[4], r[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    w[u] = Y[kq + lane + (h + u) * 64];
                    if constexpr (PEND) r[u] = Rw[kq + lane + (h + u) * 64];
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    a0 = fma(vc[h + u].x, w[u].x, a0);
                    a1 = fma(vc[h + u].y, w[u].y, a1);
                    if constexpr (PEND) {
                        b0 = fma(vc[h + u].x, r[u].x, b0);
                        b1 = fma(vc[h + u].y, r[u].y, b1);
                    }
                }
            }
        };
        for (; kb + 8 * 64 < L2; kb += 8 * 64) {
            dbl2 vn[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) vn[u] = ld2<SPX_NT_A>(&col[kb + 8 * 64 + lane + u * 64]);
            consume(kb);
#pragma unroll
            for (int u = 0; u < 8; ++u) vc[u] = vn[u];
        }
        consume(kb);
        return;
    }
    for (; k + 7 * 64 < L2; k += 8 * 64) {
        dbl2 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = ld2<SPX_NT_A>(&col[k + u * 64]);
#pragma unroll
        for (int h = 0; h < 8; h += 4) {
            dbl2 w[4], r[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                w[u] = Y[k + (h + u) * 64];
                if constexpr (PEND) r[u] = Rw[k + (h + u) * 64];
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                a0 = fma(v[h + u].x, w[u].x, a0);
                a1 = fma(v[h + u].y, w[u].y, a1);
                if constexpr (PEND) {
                    b0 = fma(v[h + u].x, r[u].x, b0);
                    b1 = fma(v[h + u].y, r[u].y, b1);
                }
            }
        }
    }
    for (; k < L2; k += 64) {
        const dbl2 v = ld2<SPX_NT_A>(&col[k]);
        const dbl2 w = Y[k];
        a0 = fma(v.x, w.x, a0);
        a1 = fma(v.y, w.y, a1);
        if constexpr (PEND) {
            const dbl2 r = Rw[k];
            b0 = fma(v.x, r.x, b0);
            b1 = fma(v.y, r.y, b1);
        }
    }
}

// FTRAN of two rows at once (acc0: row pointer s0, acc1: s1 or none), U dbl2
// chunks each per round trip; the first U chunks of each row may come from
// pf0/pf1 (loaded ahead of the barrier).  Per-row order as k_update.
#ifndef SPX_LOOP_FU
#define SPX_LOOP_FU 4  // 8 spills registers with the barrier-crossing prefetch
#endif
constexpr int FU = SPX_LOOP_FU;

__device__ __forceinline__ void ftran_rows2(const dbl2* __restrict__ ap, const dbl2* __restrict__ s0,
                                            const dbl2* __restrict__ s1, int64_t L2, int lane, const dbl2 (&pf0)[FU],
                                            const dbl2 (&pf1)[FU], bool have, double& acc0, double& acc1) {
    int64_t k = lane;
    if (have && FU * 64 <= L2) {
        dbl2 av[FU];
#pragma unroll
        for (int t = 0; t < FU; ++t) av[t] = ap[k + t * 64];
#pragma unroll
        for (int t = 0; t < FU; ++t) {
            acc0 = fma(pf0[t].x, av[t].x, acc0);
            acc0 = fma(pf0[t].y, av[t].y, acc0);
            if (s1) {
                acc1 = fma(pf1[t].x, av[t].x, acc1);
                acc1 = fma(pf1[t].y, av[t].y, acc1);
            }
        }
        k += FU * 64;
    }
    for (; k + (FU - 1) * 64 < L2; k += FU * 64) {
        dbl2 av[FU], b0[FU], b1[FU];
#pragma unroll
        for (int t = 0; t < FU; ++t) {
            av[t] = ap[k + t * 64];
            b0[t] = ld2<SPX_NT_BLOAD>(&s0[k + t * 64]);
            if (s1) b1[t] = ld2<SPX_NT_BLOAD>(&s1[k + t * 64]);
        }
#pragma unroll
        for (int t = 0; t < FU; ++t) {
            acc0 = fma(b0[t].x, av[t].x, acc0);
            acc0 = fma(b0[t].y, av[t].y, acc0);
            if (s1) {
                acc1 = fma(b1[t].x, av[t].x, acc1);
                acc1 = fma(b1[t].y, av[t].y, acc1);
            }
        }
    }
    for (; k < L2; k += 64) {
        const dbl2 av = ap[k];
        const dbl2 v0 = s0[k];
        acc0 = fma(v0.x, av.x, acc0);
        acc0 = fma(v0.y, av.y, acc0);
        if (s1) {
            const dbl2 v1 = s1[k];
            acc1 = fma(v1.x, av.x, acc1);
            acc1 = fma(v1.y, av.y, acc1);
        }
    }
}

template <int BLOCK, bool LDS_R>
__global__ __launch_bounds__(BLOCK) void k_loop(Params P, LoopArgs La) {
    constexpr int WAVES = BLOCK / 64;
    using Sh = LoopLds<WAVES>;
    DevState* st = P.st;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int G = (int)gridDim.x;
    const bool wg0 = blockIdx.x == 0;
    const int64_t L = P.L, L2 = L >> 1, m = P.m, n = P.n;
    const int KW = P.win;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    double* ys = reinterpret_cast<double*>(smem);
    double* rs = ys + (LDS_R ? L : 0);
    Sh& S = *reinterpret_cast<Sh*>(smem + (LDS_R ? 2 : 1) * L * 8);
    __shared__ int s_ok;
    // the whole grid resident, or nobody touches the state (spx_grid.h)
    if (!grid_arrive(La.ls, &s_ok)) return;

    // ---- launch prologue: the state every workgroup keeps (uniform)
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
    const double* yw = st->y_buf ? P.y1 : P.y0;
    const double* Bw = P.B0;
    const int stride = G * WAVES;
    const int idx0 = (int)blockIdx.x * WAVES + wave;
    // first pricing column's chunks in flight during the LDS fill
    dbl2 pre[CH];
    bool have = SPX_LOOP_CPRE && idx0 < cnt && L2 >= CH * 64;
    if (have) {
        const dbl2* c0 = reinterpret_cast<const dbl2*>(P.A + (int64_t)ld_agent(&P.nb_list[idx0]) * L);
#pragma unroll
        for (int u = 0; u < CH; ++u) pre[u] = ld2<SPX_NT_A>(&c0[lane + u * 64]);
    }
    {
        const dbl2* yin = reinterpret_cast<const dbl2*>(yw);
        const dbl2* rin = reinterpret_cast<const dbl2*>(Bw + (nw > 0 ? q : 0) * L);
        dbl2* yl = reinterpret_cast<dbl2*>(ys);
        dbl2* rl = reinterpret_cast<dbl2*>(rs);
        for (int64_t k = tid; k < L2; k += BLOCK) {
            yl[k] = yin[k];
            if (LDS_R && nw > 0) rl[k] = rin[k];
        }
        if (tid < KW) {
            S.SY[tid] = (tid < nw) ? P.SY[tid] : 0.0;
            S.Uq[tid] = (nw > 0 && tid < nw - 1) ? ld_agent(&P.U[q * KW + tid]) : 0.0;
        }
        // the pending pivot's base row and coefficients for k_fold (after a
        // fold B_w changed, so the row is re-staged, as k_price does)
        if (wg0 && nw > 0) {
            dbl2* qo = reinterpret_cast<dbl2*>(P.Qrows + (int64_t)(nw - 1) * L);
            for (int64_t k = tid; k < L2; k += BLOCK) qo[k] = rin[k];
            if (tid < nw - 1) P.Urows[(int64_t)(nw - 1) * KW + tid] = ld_agent(&P.U[q * KW + tid]);
        }
    }
    __syncthreads();
    // the last pivot's change of the non-basic list, applied locally (slot ->
    // column) until workgroup 0's global writes are known visible
    int pk1 = -1, pk2 = -1;
    int64_t pv1 = 0, pv2 = 0;
    auto list_at = [&](int idx) -> int64_t {
        return (idx == pk1) ? pv1 : ((idx == pk2) ? pv2 : (int64_t)ld_agent(&P.nb_list[idx]));
    };
    uint32_t target = 0;
    const int64_t rpw = (m + G - 1) / G;  // FTRAN rows per workgroup: row0 + wave + r * WAVES
    const int64_t row0 = (int64_t)blockIdx.x * rpw;
    const int64_t row1 = (row0 + rpw < m) ? row0 + rpw : m;
    const dbl2* srcB = reinterpret_cast<const dbl2*>(Bw);

    // nw < KW bounds every pass as well (uniform across the grid): the window
    // never overflows whatever npasses the host asked for
    for (int pass = 0; pass < La.npasses && it < limit && nw < KW; ++pass) {
        const bool pend = nw > 0;
        const int tau = nw - 1;
        unsigned long long* clk = (La.clock && wg0 && tid == 0) ? La.clock + 3 * (int64_t)pass : nullptr;
        if (clk) clk[0] = rtime();

        // ================= phase A: pricing (k_price, window mode)
        double uq = 0.0, syl = 0.0, syp = 0.0;
        if (pend) {
            if (lane < tau) {
                uq = S.Uq[lane];
                syl = S.SY[lane];
            }
            syp = S.SY[tau];
        }
        const dbl2* Y = reinterpret_cast<const dbl2*>(ys);
        const dbl2* Rw = LDS_R ? reinterpret_cast<const dbl2*>(rs) : reinterpret_cast<const dbl2*>(Bw + q * L);
        double best = INFINITY, bw = 0.0, be = 0.0;
        int64_t bj = INT64_MAX;
        int64_t jn = (idx0 < cnt) ? list_at(idx0) : 0;
        for (int idx = idx0; idx < cnt; idx += stride) {
            const int64_t j = jn;
            const dbl2* __restrict__ col = reinterpret_cast<const dbl2*>(P.A + j * L);
            double wv = 0.0;
            if (pend && lane < tau) wv = ld_agent(&P.Wt[j * KW + lane]);
            double a0 = 0.0, a1 = 0.0, b0 = 0.0, b1 = 0.0;
            if (pend) price_column<true>(col, Y, Rw, L2, lane, pre, have, a0, a1, b0, b1);
            else price_column<false>(col, Y, Rw, L2, lane, pre, have, a0, a1, b0, b1);
            // the next column's first chunks in flight during this reduction
            const int nidx = idx + stride;
#ifndef SPX_LOOP_NPRE
#define SPX_LOOP_NPRE 0  // next column loaded during the reduction: measured slower (C3 +2 us)
#endif
            have = SPX_LOOP_NPRE && nidx < cnt && L2 >= CH * 64;
            if (have) {
                jn = list_at(nidx);
                const dbl2* cn = reinterpret_cast<const dbl2*>(P.A + jn * L);
#pragma unroll
                for (int u = 0; u < CH; ++u) pre[u] = ld2<SPX_NT_A>(&cn[lane + u * 64]);
            } else if (nidx < cnt) {
                jn = list_at(nidx);
            }
            double e, wn = 0.0;
            if (pend) {
                // r_tau . A_j = B_w[q,:] . A_j + sum_s U[q][s] Wt[j][s]
                double sa = fma(syl, wv, a0 + a1);
                wn = fma(uq, wv, b0 + b1);
                wave_sum2(sa, wn);
                if (lane == 0) st_agent(&P.Wt[j * KW + tau], wn);
                e = fma(syp, wn, sa) - P.c[j];
            } else {
                e = wave_sum(a0 + a1) - P.c[j];
            }
            double key = e;
            if (P.devex) {  // include/simplex.h SPX_PRICING_DEVEX, as k_price
                double w = ld_agent(&P.W[j]);
                if (pend) {
                    if (j == dleave) w = fmax(dwp / (aq * aq), 1.0);
                    else {
                        const double g = wn / aq;
                        w = fmax(w, g * g * dwp);
                    }
                    if (lane == 0) st_agent(&P.W[j], w);
                }
                key = (e < -P.eps) ? -(e * e) / w : INFINITY;
            }
            if (argmin_better(key, j, best, bj)) {
                best = key;
                bj = j;
                bw = wn;
                be = e;
            }
        }
        if (lane == 0) S.pred[wave] = PricePartial{best, bj, bw, be};
        __syncthreads();
        if (tid == 0) {
            PricePartial w = S.pred[0];
            for (int i = 1; i < WAVES; ++i) price_merge(w, S.pred[i]);
            PricePartial* d = &La.pp[blockIdx.x];
            st_agent(&d->val, w.val);
            st_agent(&d->idx, w.idx);
            st_agent(&d->w, w.w);
            st_agent(&d->pad, w.pad);
        }
        // this wave's first two FTRAN rows: their first chunks in flight across
        // the barrier (B_w rows do not depend on the entering column)
        const int64_t fr0 = row0 + wave, fr1 = row0 + wave + WAVES;
        dbl2 pf0[FU], pf1[FU];
#ifndef SPX_LOOP_FPRE
#define SPX_LOOP_FPRE 1
#endif
        const bool fpre = SPX_LOOP_FPRE && !P.bc && fr0 < row1 && FU * 64 <= L2;
        if (fpre) {
#pragma unroll
            for (int t = 0; t < FU; ++t) {
                pf0[t] = ld2<SPX_NT_BLOAD>(&srcB[fr0 * L2 + lane + t * 64]);
                if (fr1 < row1) pf1[t] = ld2<SPX_NT_BLOAD>(&srcB[fr1 * L2 + lane + t * 64]);
            }
        }
        target += (uint32_t)G;
        if (!grid_sync(La.ls, target, &s_ok)) return;
        if (clk) clk[1] = rtime();

        // ================= phase B: entering column, FTRAN + ratio test (k_update, window mode)
        {
            PricePartial w{INFINITY, INT64_MAX, 0.0, 0.0};
            for (int g = tid; g < G; g += BLOCK) {
                const PricePartial* d = &La.pp[g];
                PricePartial v{ld_agent(&d->val), ld_agent(&d->idx), ld_agent(&d->w), ld_agent(&d->pad)};
                price_merge(w, v);
            }
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) {
                PricePartial o{__shfl_xor(w.val, off, 64), __shfl_xor(w.idx, off, 64), __shfl_xor(w.w, off, 64),
                               __shfl_xor(w.pad, off, 64)};
                price_merge(w, o);
            }
            if (lane == 0) S.pred[wave] = w;
            __syncthreads();
            if (tid == 0) {
                PricePartial t = S.pred[0];
                for (int i = 1; i < WAVES; ++i) price_merge(t, S.pred[i]);
                S.pwin = t;
                if (!no_entering(P, t.val, t.idx)) {  // the list slots the pivot will change
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
            const dbl2* __restrict__ ap = reinterpret_cast<const dbl2*>(P.A + p * L);
            const bool upd_x = xb_applied < it;
            const double wl = lane < nw ? ld_agent(&P.Wt[p * KW + lane]) : 0.0;
            double sxw = 0.0;
            if (pend) {
                sxw = lane < tau ? mul_nc(ld_agent(&P.U[q * KW + lane]), ld_agent(&P.Wt[n * KW + lane])) : 0.0;
                sxw = P.xw[q] + wave_sum(sxw);
                if (wg0 && tid == 0) st_agent(&P.Wt[n * KW + tau], sxw);
            }
            const double s_x = upd_x ? sxw : 0.0;
            // compact FTRAN operand (Params::bc, spx_kernels.hip k_update BC):
            // A_p on the column list in LDS when it fits (else gathered per
            // chunk), the same per-lane order, so the same bits as k_update
            const int Sb = P.bc ? P.bc_n[0] : 0;
            const bool apl = P.bc && Sb <= P.bc_lds;
            double* apc = reinterpret_cast<double*>(smem + (LDS_R ? 2 : 1) * L * 8 + ((sizeof(Sh) + 15) / 16) * 16);
            const double* apd = P.A + p * L;
            if (apl) {
                for (int c = tid; c < Sb; c += BLOCK) apc[c] = apd[P.rlist[c]];
                __syncthreads();
            }
            auto compact_row = [&](int64_t i) -> double {
                double a = (lane == 0 && P.rmap[i] < 0) ? apd[i] : 0.0;
                const dbl2* brow = reinterpret_cast<const dbl2*>(bc_buf(P, P.bc_n[2]) + i * (int64_t)P.bc_n[1]);
                const int S2 = (Sb + 1) >> 1;
                for (int k0 = 0; k0 < S2; k0 += 8 * 64) {
                    dbl2 v[8], w[8];
#pragma unroll
                    for (int t = 0; t < 8; ++t) {
                        const int k2 = k0 + lane + 64 * t;
                        v[t] = brow[k2 < S2 ? k2 : 0];
                        if (apl) {
                            w[t] = reinterpret_cast<const dbl2*>(apc)[k2 < S2 ? k2 : 0];
                        } else {
                            const int c0 = 2 * (k2 < S2 ? k2 : 0);
                            w[t].x = apd[P.rlist[c0]];
                            w[t].y = c0 + 1 < Sb ? apd[P.rlist[c0 + 1]] : 0.0;
                        }
                    }
#pragma unroll
                    for (int t = 0; t < 8; ++t) {
                        const int k2 = k0 + lane + 64 * t;
                        if (2 * k2 < Sb) a = fma(v[t].x, w[t].x, a);
                        if (2 * k2 + 1 < Sb) a = fma(v[t].y, w[t].y, a);
                    }
                }
                return a;
            };
            UpdPartial wp = upd_empty();
            for (int64_t i0 = row0 + wave; i0 < row1; i0 += 2 * WAVES) {
                const int64_t i1 = i0 + WAVES;
                const bool two = i1 < row1;
                double acc[2] = {0.0, 0.0};
                if (P.bc) {
                    acc[0] = compact_row(i0);
                    if (two) acc[1] = compact_row(i1);
                } else if (i0 == fr0)  // the prefetched pair (the first)
                    ftran_rows2(ap, srcB + i0 * L2, two ? srcB + i1 * L2 : nullptr, L2, lane, pf0, pf1, fpre,
                                acc[0], acc[1]);
                else
                    ftran_rows2(ap, srcB + i0 * L2, two ? srcB + i1 * L2 : nullptr, L2, lane, pf0, pf1, false,
                                acc[0], acc[1]);
#pragma unroll
                for (int r = 0; r < 2; ++r) {
                    const int64_t i = r ? i1 : i0;
                    if (r && !two) break;
                    const double ei = pend ? eta_entry(ld_agent(&a_prev[i]), i, q, aq) : 0.0;
                    const int64_t bix = ld_agent(&P.b_ixs[i]);
                    const double cb = ld_agent(&P.c_B[i]);
                    double xb = P.x_b[i];
                    if (pend && lane == 0) st_agent(&P.Wt[bix * KW + tau], (i == q) ? aq : 0.0);
                    const double cu = lane < tau ? ld_agent(&P.U[i * KW + lane]) : (lane == tau ? ei : 0.0);
                    const double a = wave_sum(fma(cu, wl, acc[r]));
                    if (pend && lane == 0) st_agent(&P.U[i * KW + tau], ei);
                    if (upd_x) xb = fma(s_x, ei, xb);
                    if (lane == 0) {
                        st_agent(&a_new[i], a);
                        if (upd_x) P.x_b[i] = xb;
                    }
                    const double th = ratio_key(P, xb, a);
                    wp.nonpos += !(a > P.piv_tol);
                    wp.T = fma(cb, a, wp.T);
                    if (argmin_better(th, i, wp.theta, wp.idx)) {
                        wp.theta = th;
                        wp.idx = i;
                        wp.a_w = a;
                        wp.cb_w = cb;
                        wp.bix_w = bix;
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
        // the list change (pivot_bookkeeping's swap-remove of p + append of leave)
        pk1 = (kp != cnt - 1) ? (int)kp : -1;
        pv1 = lastv;
        pk2 = cnt - 1;
        pv2 = leave;
        // the next pass's first column in flight during the base-row fill
        have = SPX_LOOP_CPRE && idx0 < cnt && L2 >= CH * 64 && it + 1 < limit;
        if (have) {
            const dbl2* c0 = reinterpret_cast<const dbl2*>(P.A + list_at(idx0) * L);
#pragma unroll
            for (int u = 0; u < CH; ++u) pre[u] = ld2<SPX_NT_A>(&c0[lane + u * 64]);
        }
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
            if (P.rleft) st_agent(&P.rleft[qn], 1);  // (as pivot_bookkeeping: the compact operand's list)
            P.SY[nw] = s_y;
            st->aq = aqn;
            st->s_y = s_y;
            st->nw = nw + 1;
            st->xb_applied = it;
            st->p = p;
            st->q = qn;
            st->min_e = P.devex ? S.pwin.pad : min_e;
            st->iter = it + 1;
            record_pivot(P, it, p, qn);
            if (P.devex) {
                st->leave = leave;
                st->wp = wp_new;
            }
        }
        // the new pending pivot (tau' = nw): base row and its U coefficients;
        // workgroup 0 also keeps them in Qrows / Urows for k_fold
        {
            const dbl2* rin = reinterpret_cast<const dbl2*>(Bw + qn * L);
            dbl2* rl = reinterpret_cast<dbl2*>(rs);
            dbl2* qo = reinterpret_cast<dbl2*>(P.Qrows + (int64_t)nw * L);
            for (int64_t k = tid; k < L2; k += BLOCK) {
                const dbl2 v = rin[k];
                if (LDS_R) rl[k] = v;
                if (wg0) qo[k] = v;
            }
            if (tid < nw) {
                const double u = ld_agent(&P.U[qn * KW + tid]);
                S.Uq[tid] = u;
                if (wg0) P.Urows[(int64_t)nw * KW + tid] = u;
            }
            if (tid == 0) S.SY[nw] = s_y;
        }
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

template <int BLOCK, bool LR>
static hipError_t prepare_t(const LoopCfg& c, int* per_cu) {
    const void* fn = reinterpret_cast<const void*>(&k_loop<BLOCK, LR>);
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)c.lds_bytes);
    if (e != hipSuccess) return e;
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(per_cu, k_loop<BLOCK, LR>, BLOCK, c.lds_bytes);
}

template <int BLOCK, bool LR>
static const void* fn_t() {
    return reinterpret_cast<const void*>(&k_loop<BLOCK, LR>);
}

hipError_t loop_prepare(const Params& P, int cus, LoopCfg& c, bool want_bc) {
    c.ok = false;
    c.block = 512;  // 8 waves per CU: 256 VGPRs per lane for the prefetch registers (1024 spilled)
    c.grid = cus;
    const size_t ybytes = (size_t)P.L * 8;
    const size_t small = sizeof(LoopLds<16>) + 16;
    const size_t cap = 150 * 1024;
    c.lds_r = 2 * ybytes + small <= cap;
    if (!c.lds_r && ybytes + small > cap) return hipSuccess;  // y_w alone does not fit
    c.lds_bytes = (c.lds_r ? 2 : 1) * ybytes + small;
    if (want_bc) {  // compact FTRAN operand: A_p on the column list, what is left up to cap
        const size_t room = cap - c.lds_bytes;
        c.bc_lds = (int)std::min<size_t>((size_t)P.L, room / 8 / 64 * 64);
        c.lds_bytes += (size_t)c.bc_lds * 8;
    }
    int dev = 0, coop = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    e = hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, dev);
    if (e != hipSuccess) return e;
    if (!coop) return hipSuccess;
    int per_cu = 0;
    e = c.lds_r ? prepare_t<512, true>(c, &per_cu) : prepare_t<512, false>(c, &per_cu);
    if (e != hipSuccess) return e;
    c.ok = per_cu >= 1;
    return hipSuccess;
}

hipError_t launch_loop(const Params& P, const LoopArgs& a, const LoopCfg& c, hipStream_t s) {
    void* args[] = {const_cast<Params*>(&P), const_cast<LoopArgs*>(&a)};
    const void* fn = c.lds_r ? fn_t<512, true>() : fn_t<512, false>();
    // a plain launch: the grid (one workgroup per CU, per_cu >= 1 checked in
    // loop_prepare) is co-resident without the cooperative launch's check,
    // and the grid barrier is our own (spx_grid.h), so no cooperative queue
    // (MI355X_MICROARCH.md coop-launch: +15-19 us host wall per launch).  The
    // round-1 cooperative launch is gone for good: a process that had made one
    // faulted in the HIP runtime's exit teardown under rocprofv3
    // (profiles/r03_coop_exit_segv.txt), so no switch brings it back.
    return hipLaunchKernel(fn, dim3(loop_grid_launched(c.grid, a.call_launch)), dim3(c.block), args,
                           (size_t)c.lds_bytes, s);
}

// SPX_LOOP_OVERSUB=1 (tests): launch 4,096 more workgroups than the
// co-resident grid -- more than any GPU holds at once (at most 32 waves per
// CU) -- so the entry check (grid_arrive) must fail and the host fall back to
// two-kernel passes.  SPX_LOOP_OVERSUB=2: only the first launch of a call, so
// the later launches of that call would have a resident grid (the sticky
// failure of grid_arrive must still send them home).
int loop_grid_launched(int grid, int call_launch) {
    const char* v = std::getenv("SPX_LOOP_OVERSUB");
    const bool over = v && (v[0] == '1' || (v[0] == '2' && call_launch == 0));
    return over ? grid + 4096 : grid;
}

}  // namespace spx

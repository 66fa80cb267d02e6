// spx_tabdev.h — per-lane arithmetic of the window tableau,
// shared by the two-kernel passes (k_price WM 3 and k_tab_update,
// spx_kernels.hip) and the persistent tableau loop (k_tab_loop,
// spx_tableau.hip), so every path produces the same bits for a column or a
// row.  One lane owns one column (pricing) or one row (FTRAN); the window
// sums run in pivot order s = 0, 1, ... inside the lane, so no cross-lane
// reduction is needed until the argmin.
#pragma once
#include <hip/hip_runtime.h>

#include "spx_common.h"

namespace spx {

// Pricing of one non-basic column j for the pending window pivot tau
// (tau < 0: nothing pending):
//   w   = r_tau . A_j = T_w[q_tau, j] + sum_{s<tau} U[q_tau][s] Wt[j][s]
//   e_j = dw[j] + sum_{s<tau} SY[s] Wt[j][s] + SY[tau] w
// (e_j = y.A_j - c_j of v4:288-290 with y = y_w + sum_s SY[s] r_s and
// dw = y_w A - c).  tq = T_w[q_tau, j]; dv = dw[j]; sy, uq = SY[.] and
// U[q_tau][.]; wt(s) = Wt[j][s].
template <class F>
__device__ __forceinline__ void tab_price_column(double tq, double dv, int tau, const double* sy, const double* uq,
                                                 F wt, double& w, double& e) {
    double sa = 0.0, wn = 0.0;
    int s = 0;
    for (; s + 4 <= tau; s += 4) {
        double v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = wt(s + u);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            sa = fma(sy[s + u], v[u], sa);
            wn = fma(uq[s + u], v[u], wn);
        }
    }
    for (; s < tau; ++s) {
        const double v = wt(s);
        sa = fma(sy[s], v, sa);
        wn = fma(uq[s], v, wn);
    }
    w = tq + wn;
    e = (tau >= 0) ? fma(sy[tau], w, dv + sa) : dv;
}

// FTRAN of one row i (v4:306-308 with B^-1 = B_w + sum_s eta_s r_s^T):
//   alpha_i = T_w[i, p] + sum_{s<tau} U[i][s] Wt[p][s] + eta_tau[i] Wt[p][tau]
// t = T_w[i, p]; ei = eta_tau[i] (compute_E_q of the pending pivot,
// v4:210-215, not yet in U); wp = Wt[p][.]; u(s) = U[i][s].
template <class F>
__device__ __forceinline__ double tab_ftran_row(double t, int tau, double ei, const double* wp, F u) {
    double acc = t;
    int s = 0;
    for (; s + 4 <= tau; s += 4) {
        double v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = u(s + k);
#pragma unroll
        for (int k = 0; k < 4; ++k) acc = fma(v[k], wp[s + k], acc);
    }
    for (; s < tau; ++s) acc = fma(u(s), wp[s], acc);
    if (tau >= 0) acc = fma(ei, wp[tau], acc);
    return acc;
}

// Wave argmin of a pricing candidate (value, then smallest index), carrying
// w and e; every lane ends with the wave's winner.
__device__ __forceinline__ void wave_price_min(double& key, int64_t& j, double& w, double& e) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const double k2 = __shfl_xor(key, off, 64);
        const int64_t j2 = __shfl_xor(j, off, 64);
        const double w2 = __shfl_xor(w, off, 64);
        const double e2 = __shfl_xor(e, off, 64);
        if (argmin_better(k2, j2, key, j)) {
            key = k2;
            j = j2;
            w = w2;
            e = e2;
        }
    }
}

// Wave merge of ratio-test partials in a fixed role order (lower lane's value
// first), as reduce_update_partials; every lane ends with the merged partial.
__device__ __forceinline__ UpdPartial wave_upd_merge(UpdPartial w) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const UpdPartial o = upd_shfl_xor(w, off);
        UpdPartial lo = (lane & off) ? o : w;
        const UpdPartial hi = (lane & off) ? w : o;
        upd_merge(lo, hi);
        w = lo;
    }
    return w;
}

}  // namespace spx

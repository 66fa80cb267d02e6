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
#include "spx_tableau.h"

namespace spx {

namespace {

// One workgroup: 4 waves x 64 rows of T_w, and a chunk of columns.  Each wave
// keeps its U fragments (B operand, lane: U[i0 + 16 ib + cl][4 s + kr]) in
// registers for the whole chunk and walks it 16 columns at a time: Wt
// fragment (A operand, lane: Wt[j0 + cl][4 s + kr]) from L2, the 16 x 64
// T_w block as 4 accumulator tiles (lane: T_w[i0 + 16 ib + cl, j0 + kr + 4 r]),
// ceil(nf/4) v_mfma_f64_16x16x4f64 steps per tile, stored back.  The next
// block's T_w loads are issued before this block's MFMAs.
template <int KW>
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
    const int64_t per = ((n + gridDim.y - 1) / gridDim.y + 15) / 16 * 16;
    const int64_t c0 = (int64_t)blockIdx.y * per;
    const int64_t c1 = (c0 + per < n) ? c0 + per : n;
    const double* __restrict__ U = P.U;
    const double* __restrict__ Wt = P.Wt;
    double* __restrict__ T = P.T;

    if (blockIdx.x == 0) {  // dw[j] += sum_{t<nf} SY[t] Wt[j][t], fixed t order
        for (int64_t j = c0 + tid; j < c1; j += 256) {
            double d = 0.0;
            for (int t = 0; t < nf; ++t) d = fma(P.SY[t], Wt[j * KW + t], d);
            P.dw[j] += d;
        }
    }
    const int64_t i0 = ((int64_t)blockIdx.x * 4 + wave) * 64;
    if (i0 >= m || c0 >= c1) return;
    double uf[4][KS];
#pragma unroll
    for (int ib = 0; ib < 4; ++ib) {
        const int64_t i = i0 + 16 * ib + cl;
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const int t = 4 * s + kr;
            uf[ib][s] = (i < m && t < nf) ? U[i * KW + t] : 0.0;
        }
    }
    bool rok[4];
#pragma unroll
    for (int ib = 0; ib < 4; ++ib) rok[ib] = i0 + 16 * ib + cl < m;
    auto load_block = [&](int64_t j0, dbl4 (&acc)[4]) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int64_t j = j0 + kr + 4 * r;
            const bool jok = j < c1;
#pragma unroll
            for (int ib = 0; ib < 4; ++ib)
                acc[ib][r] = (jok && rok[ib]) ? T[j * L + i0 + 16 * ib + cl] : 0.0;
        }
    };
    dbl4 cur[4];
    load_block(c0, cur);
    for (int64_t j0 = c0; j0 < c1; j0 += 16) {
        double wf[KS];
        const int64_t jw = j0 + cl;
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const int t = 4 * s + kr;
            wf[s] = (jw < c1 && t < nf) ? Wt[jw * KW + t] : 0.0;
        }
        dbl4 nxt[4];
        const bool more = j0 + 16 < c1;
        if (more) load_block(j0 + 16, nxt);
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            if (s < ks) {
#pragma unroll
                for (int ib = 0; ib < 4; ++ib)
                    cur[ib] = __builtin_amdgcn_mfma_f64_16x16x4f64(wf[s], uf[ib][s], cur[ib], 0, 0, 0);
            }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int64_t j = j0 + kr + 4 * r;
            if (j < c1) {
#pragma unroll
                for (int ib = 0; ib < 4; ++ib)
                    if (rok[ib]) T[j * L + i0 + 16 * ib + cl] = cur[ib][r];
            }
        }
        if (more) {
#pragma unroll
            for (int ib = 0; ib < 4; ++ib) cur[ib] = nxt[ib];
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

}  // namespace

hipError_t launch_tab_fold(const Params& P, int min_nw, int cus, hipStream_t s) {
    if (!P.tab) return hipSuccess;
    const int64_t gx = (P.m + 255) / 256;
    // about 8 workgroups per CU over the whole T_w (2 resident per CU at the
    // fragment register budget), each chunk a whole number of 16-column blocks
    int64_t gy = ((int64_t)8 * cus + gx - 1) / gx;
    const int64_t maxy = (P.n + 15) / 16;
    if (gy > maxy) gy = maxy;
    if (gy < 1) gy = 1;
    const dim3 grid((unsigned)gx, (unsigned)gy);
    switch (P.win) {
        case 8: hipLaunchKernelGGL(k_tab_fold<8>, grid, dim3(256), 0, s, P, min_nw); break;
        case 16: hipLaunchKernelGGL(k_tab_fold<16>, grid, dim3(256), 0, s, P, min_nw); break;
        case 32: hipLaunchKernelGGL(k_tab_fold<32>, grid, dim3(256), 0, s, P, min_nw); break;
        case 64: hipLaunchKernelGGL(k_tab_fold<64>, grid, dim3(256), 0, s, P, min_nw); break;
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

}  // namespace spx

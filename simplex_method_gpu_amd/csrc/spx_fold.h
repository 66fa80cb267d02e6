// spx_fold.h — device helpers shared by the eta-window fold (k_fold,
// spx_kernels.hip) and the basis reinversion (spx_reinv.hip): a rank-nf
// update B += U R of a 64-column stripe of a row-major matrix with fp64 MFMA
// tiles (v_mfma_f64_16x16x4f64), R rebuilt from base rows and coefficients.
//
// Workgroup shape (tools/fold_bench.hip, MI355X, m = 4096, KW = 64: 168 ->
// 80 us, bit-identical):
//   1. the coefficients are staged transposed into LDS (fold_stage_N);
//   2. wave 0 rebuilds R right-looking (fold_rebuild_R);
//   3. every wave walks its 16-row tiles (fold_tiles), R fragments read from
//      LDS per k-step rather than held in 128 VGPRs, the next tile's loads
//      issued before this tile's MFMAs.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace spx {

typedef double dbl4 __attribute__((ext_vector_type(4)));

template <int KW>
constexpr int FOLD_NP = KW + 2;  // LDS pitch of the staged coefficients

// All threads: NT[s][t] = Urows[t][s] on the strict lower nf x nf triangle, 0
// elsewhere (so rows t >= nf of R rebuild to exact zeros).  Pitch KW + 2 keeps
// the transposing stores off one bank and the rows 16-byte aligned (the
// rebuild's uniform reads pair up into ds_read_b128).
template <int KW>
__device__ __forceinline__ void fold_stage_N(const double* Urows, int nf, double (&NT)[KW][FOLD_NP<KW>]) {
    for (int k = threadIdx.x; k < KW * KW; k += blockDim.x) {
        const int t = k / KW, s = k % KW;
        NT[s][t] = (t < nf && s < t) ? Urows[k] : 0.0;
    }
}

// Wave 0 of a fold workgroup, after fold_stage_N and a barrier: r_t for the
// 64-column stripe at c0 (one column per lane), r_t = Qrows[t] + sum_{s<t}
// Urows[t][s] r_s, into Rl and R.  Right-looking: once r_s is final every later
// r_t takes its s term, so each r_t still sums s = 0, 1, .. in order (the bits
// of the left-looking recurrence) but the 63 accumulators are independent
// instead of one 2016-deep fma chain.
template <int KW>
__device__ __forceinline__ void fold_rebuild_R(const double* Qrows, const double (&NT)[KW][FOLD_NP<KW>], int nf, int64_t L,
                                               int64_t c0, double (&Rl)[KW][64], double (&R)[KW]) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int t = 0; t < KW; ++t) R[t] = (t < nf) ? Qrows[(int64_t)t * L + c0 + lane] : 0.0;
#pragma unroll
    for (int s = 0; s < KW; ++s) {
        Rl[s][lane] = R[s];
#pragma unroll
        for (int t = s + 1; t < KW; ++t) R[t] = fma(NT[s][t], R[s], R[t]);
    }
}

// The 16-row x 64-column tile of B at rows r0.. (rows >= i1 read as 0), in the
// MFMA accumulator layout: lane holds rows r0 + kr + 4 r, column 16 jb + cl.
__device__ __forceinline__ void fold_tile_load(const double* B, int64_t L, int64_t c0, int64_t r0, int64_t i1,
                                               dbl4 (&t)[4]) {
    const int lane = threadIdx.x & 63;
    const int kr = lane >> 4, cl = lane & 15;
#pragma unroll
    for (int jb = 0; jb < 4; ++jb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int64_t i = r0 + kr + 4 * r;
            t[jb][r] = (i < i1) ? B[i * L + c0 + 16 * jb + cl] : 0.0;
        }
}

// B[i0:i1, c0:c0+64] += U[i0:i1, 0:nf] R[0:nf, stripe] with 16x16 fp64 MFMA
// tiles (the B tile is the accumulator); U is m x KW row-major.  Wave w takes
// tiles i0 + 16 w, i0 + 16 (w + nwaves), ..  Call after a barrier that
// published Rl.
template <int KW>
__device__ __forceinline__ void fold_tiles(double* B, const double* U, int nf, int64_t L, int64_t c0, int64_t i0,
                                           int64_t i1, const double (&Rl)[KW][64]) {
    constexpr int KS = KW / 4;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nwaves = blockDim.x >> 6;
    const int kr = lane >> 4, cl = lane & 15;
    const int ks = (nf + 3) / 4;
    dbl4 nxt[4];
    if (i0 + 16 * wave < i1) fold_tile_load(B, L, c0, i0 + 16 * wave, i1, nxt);
    for (int64_t r0 = i0 + 16 * wave; r0 < i1; r0 += 16 * nwaves) {
        dbl4 acc[4];
#pragma unroll
        for (int jb = 0; jb < 4; ++jb) acc[jb] = nxt[jb];
        const int64_t rn = r0 + 16 * nwaves;
        if (rn < i1) fold_tile_load(B, L, c0, rn, i1, nxt);
        // U fragment (A operand): lane holds U[r0 + cl][4 s + kr]
        const int64_t ia = r0 + cl;
        double af[KS];
#pragma unroll
        for (int s2 = 0; s2 < KS; ++s2) {
            const int t = 4 * s2 + kr;
            af[s2] = (ia < i1 && t < nf) ? U[ia * KW + t] : 0.0;
        }
        // R fragment (B operand) from LDS: R[4 s + kr][16 jb + cl]
#pragma unroll
        for (int s2 = 0; s2 < KS; ++s2) {
            if (s2 < ks) {
#pragma unroll
                for (int jb = 0; jb < 4; ++jb)
                    acc[jb] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[s2], Rl[4 * s2 + kr][16 * jb + cl], acc[jb], 0,
                                                                   0, 0);
            }
        }
#pragma unroll
        for (int jb = 0; jb < 4; ++jb)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int64_t i = r0 + kr + 4 * r;
                if (i < i1) B[i * L + c0 + 16 * jb + cl] = acc[jb][r];
            }
    }
}

// Row ranges of a fold grid: gridDim.y ranges of whole 16-row tiles.
__device__ __forceinline__ void fold_rows(int64_t m, int64_t& i0, int64_t& i1) {
    const int64_t per = ((m + gridDim.y - 1) / gridDim.y + 15) / 16 * 16;
    i0 = (int64_t)blockIdx.y * per;
    i1 = (i0 + per < m) ? i0 + per : m;
}

// Host: the row split of a fold grid over nx stripes — about 2 workgroups per
// CU (65 KiB of LDS each), at least one 16-row tile per wave.
inline int64_t fold_grid_y(int64_t m, int nx, int cus) {
    int64_t ny = ((int64_t)2 * cus + nx - 1) / nx;
    const int64_t maxy = (m + 63) / 64;
    if (ny > maxy) ny = maxy;
    if (ny < 1) ny = 1;
    return ny;
}

}  // namespace spx

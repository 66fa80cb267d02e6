// spx_fold.h — device helpers shared by the eta-window fold (k_fold,
// spx_kernels.hip) and the basis reinversion (spx_reinv.hip): a rank-nf
// update B += U R of a 64-column stripe of a row-major matrix with fp64 MFMA
// tiles (v_mfma_f64_16x16x4f64), R rebuilt from base rows and coefficients.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace spx {

typedef double dbl4 __attribute__((ext_vector_type(4)));

// Wave 0 of a fold workgroup: r_t for the 64-column stripe at c0 (one column
// per lane), r_t = Qrows[t] + sum_{s<t} Urows[t][s] r_s, into Rl and R.
template <int KW>
__device__ __forceinline__ void fold_rebuild_R(const double* Qrows, const double* Urows, int nf, int64_t L,
                                               int64_t c0, double (&Rl)[KW][64], double (&R)[KW]) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int t = 0; t < KW; ++t) {
        double v = 0.0;
        if (t < nf) {
            v = Qrows[(int64_t)t * L + c0 + lane];
#pragma unroll
            for (int s2 = 0; s2 < t; ++s2) v = fma(Urows[t * KW + s2], R[s2], v);
        }
        R[t] = v;
        Rl[t][lane] = v;
    }
}

// B[i0:i1, c0:c0+64] += U[i0:i1, 0:nf] R[0:nf, stripe] with 16x16 fp64 MFMA
// tiles (the B tile is the accumulator); U is m x KW row-major.  Call after a
// barrier that published Rl.
template <int KW>
__device__ __forceinline__ void fold_tiles(double* B, const double* U, int nf, int64_t L, int64_t c0, int64_t i0,
                                           int64_t i1, const double (&Rl)[KW][64]) {
    constexpr int KS = KW / 4;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nwaves = blockDim.x >> 6;
    // R fragments (B operand): lane holds R[4s + (lane>>4)][16 jb + (lane&15)]
    const int kr = lane >> 4, cl = lane & 15;
    double bf[KS][4];
#pragma unroll
    for (int s2 = 0; s2 < KS; ++s2)
#pragma unroll
        for (int jb = 0; jb < 4; ++jb) bf[s2][jb] = Rl[4 * s2 + kr][16 * jb + cl];
    const int ks = (nf + 3) / 4;
    for (int64_t r0 = i0 + 16 * wave; r0 < i1; r0 += 16 * nwaves) {
        // U fragment (A operand): lane holds U[r0 + (lane&15)][4s + (lane>>4)]
        const int64_t ia = r0 + cl;
        double af[KS];
#pragma unroll
        for (int s2 = 0; s2 < KS; ++s2) {
            const int t = 4 * s2 + kr;
            af[s2] = (ia < i1 && t < nf) ? U[ia * KW + t] : 0.0;
        }
        // B tile as the accumulator: lane holds rows r0 + kr + 4 r, column 16 jb + cl
        dbl4 acc[4];
#pragma unroll
        for (int jb = 0; jb < 4; ++jb)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int64_t i = r0 + kr + 4 * r;
                acc[jb][r] = (i < i1) ? B[i * L + c0 + 16 * jb + cl] : 0.0;
            }
#pragma unroll
        for (int s2 = 0; s2 < KS; ++s2) {
            if (s2 < ks) {
#pragma unroll
                for (int jb = 0; jb < 4; ++jb)
                    acc[jb] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[s2], bf[s2][jb], acc[jb], 0, 0, 0);
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

}  // namespace spx

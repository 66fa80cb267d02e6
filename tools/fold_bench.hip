// fold_bench.hip — the eta-window fold B += U R (m x m row-major B, U m x 64,
// R rebuilt per 64-column stripe from base rows Q and coefficients N) in
// isolation: where its time goes (rebuild vs MFMA tiles) and tile variants.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -Isimplex_method_gpu_amd/csrc -o /tmp/fb tools/fold_bench.hip
//   /tmp/fb [m=4096]
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "spx_fold.h"

using namespace spx;

#define CK(x)                                                                             \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                                 \
        }                                                                                 \
    } while (0)

constexpr int KW = 64;

// the pre-change helpers (left-looking rebuild, R fragments in registers)
template <int KW>
__device__ __forceinline__ void old_rebuild_R(const double* Qrows, const double* Urows, int nf, long L, long c0,
                                              double (&Rl)[KW][64], double (&R)[KW]) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int t = 0; t < KW; ++t) {
        double v = 0.0;
        if (t < nf) {
            v = Qrows[(long)t * L + c0 + lane];
#pragma unroll
            for (int s2 = 0; s2 < t; ++s2) v = fma(Urows[t * KW + s2], R[s2], v);
        }
        R[t] = v;
        Rl[t][lane] = v;
    }
}
template <int KW>
__device__ __forceinline__ void old_tiles(double* B, const double* U, int nf, long L, long c0, long i0, long i1,
                                          const double (&Rl)[KW][64]) {
    constexpr int KS = KW / 4;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nwaves = blockDim.x >> 6;
    const int kr = lane >> 4, cl = lane & 15;
    double bf[KS][4];
#pragma unroll
    for (int s2 = 0; s2 < KS; ++s2)
#pragma unroll
        for (int jb = 0; jb < 4; ++jb) bf[s2][jb] = Rl[4 * s2 + kr][16 * jb + cl];
    const int ks = (nf + 3) / 4;
    for (long r0 = i0 + 16 * wave; r0 < i1; r0 += 16 * nwaves) {
        const long ia = r0 + cl;
        double af[KS];
#pragma unroll
        for (int s2 = 0; s2 < KS; ++s2) {
            const int t = 4 * s2 + kr;
            af[s2] = (ia < i1 && t < nf) ? U[ia * KW + t] : 0.0;
        }
        dbl4 acc[4];
#pragma unroll
        for (int jb = 0; jb < 4; ++jb)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const long i = r0 + kr + 4 * r;
                acc[jb][r] = (i < i1) ? B[i * L + c0 + 16 * jb + cl] : 0.0;
            }
#pragma unroll
        for (int s2 = 0; s2 < KS; ++s2)
            if (s2 < ks)
#pragma unroll
                for (int jb = 0; jb < 4; ++jb)
                    acc[jb] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[s2], bf[s2][jb], acc[jb], 0, 0, 0);
#pragma unroll
        for (int jb = 0; jb < 4; ++jb)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const long i = r0 + kr + 4 * r;
                if (i < i1) B[i * L + c0 + 16 * jb + cl] = acc[jb][r];
            }
    }
}

// K0: the previous k_fold body (wave 0 rebuilds R left-looking, R fragments in registers)
__global__ __launch_bounds__(256) void k0_cur(double* B, const double* U, const double* Q, const double* N, int nf,
                                              long m, long L, double* sink) {
    __shared__ double Rl[KW][64];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const long c0 = (long)blockIdx.x * 64;
    if (wave == 0) {
        double R[KW];
        old_rebuild_R<KW>(Q, N, nf, L, c0, Rl, R);
    }
    __syncthreads();
    const long per = ((m + gridDim.y - 1) / gridDim.y + 15) / 16 * 16;
    const long i0 = (long)blockIdx.y * per;
    const long i1 = (i0 + per < m) ? i0 + per : m;
    old_tiles<KW>(B, U, nf, L, c0, i0, i1, Rl);
}

// K5: the shipped k_fold structure (spx_fold.h); Y = wave 0's y_w term, XW =
// wave 1's xw rows (spread over every workgroup), as in k_fold
template <bool Y, bool XW>
__global__ __launch_bounds__(256) void k5_ship(double* B, const double* U, const double* Q, const double* N, int nf,
                                               long m, long L, double* sink) {
    __shared__ double Rl[KW][64];
    __shared__ double NT[KW][FOLD_NP<KW>];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const long c0 = (long)blockIdx.x * 64;
    int64_t i0, i1;
    fold_rows(m, i0, i1);
    fold_stage_N<KW>(N, nf, NT);
    __syncthreads();
    if (wave == 0) {
        double R[KW];
        fold_rebuild_R<KW>(Q, NT, nf, L, c0, Rl, R);
        if (Y && blockIdx.y == 0) {
            double d = 0.0;
#pragma unroll
            for (int t = 0; t < KW; ++t)
                if (t < nf) d = fma(U[t], R[t], d);
            sink[c0 + lane] += d;
        }
    } else if (XW && wave == 1) {
        const int64_t nwg = (int64_t)gridDim.x * gridDim.y;
        const int64_t rpw = (m + nwg - 1) / nwg;
        const int64_t r0 = ((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * rpw;
        const int64_t r1 = (r0 + rpw < m) ? r0 + rpw : m;
        for (int64_t i = r0 + lane; i < r1; i += 64) {
            double d = 0.0;
#pragma unroll
            for (int t = 0; t < KW; ++t)
                if (t < nf) d = fma(U[i * KW + t], Q[t], d);
            sink[L + i] += d;
        }
    }
    __syncthreads();
    fold_tiles<KW>(B, U, nf, L, c0, i0, i1, Rl);
}

// K3 tiles: B fragments read from LDS per k-step (few VGPRs), the next tile's
// B loads issued before this tile's MFMAs
template <int KWT>
__device__ __forceinline__ void tiles_lds(double* B, const double* U, int nf, long L, long c0, long i0, long i1,
                                          const double (&Rl)[KWT][64]) {
    constexpr int KS = KWT / 4;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nwaves = blockDim.x >> 6;
    const int kr = lane >> 4, cl = lane & 15;
    const int ks = (nf + 3) / 4;
    long r0 = i0 + 16 * wave;
    if (r0 >= i1) return;
    dbl4 nxt[4];
    auto load_tile = [&](long rr, dbl4(&t)[4]) {
#pragma unroll
        for (int jb = 0; jb < 4; ++jb)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const long i = rr + kr + 4 * r;
                t[jb][r] = (i < i1) ? B[i * L + c0 + 16 * jb + cl] : 0.0;
            }
    };
    load_tile(r0, nxt);
    for (; r0 < i1; r0 += 16 * nwaves) {
        dbl4 acc[4];
#pragma unroll
        for (int jb = 0; jb < 4; ++jb) acc[jb] = nxt[jb];
        const long rn = r0 + 16 * nwaves;
        if (rn < i1) load_tile(rn, nxt);
        const long ia = r0 + cl;
        double af[KS];
#pragma unroll
        for (int s2 = 0; s2 < KS; ++s2) {
            const int t = 4 * s2 + kr;
            af[s2] = (ia < i1 && t < nf) ? U[ia * KWT + t] : 0.0;
        }
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
                const long i = r0 + kr + 4 * r;
                if (i < i1) B[i * L + c0 + 16 * jb + cl] = acc[jb][r];
            }
    }
}

template <int BLK>
__global__ __launch_bounds__(BLK) void k3_tiles(double* B, const double* U, const double* Rg, int nf, long m, long L,
                                                double* sink) {
    __shared__ double Rl[KW][64];
    const long c0 = (long)blockIdx.x * 64;
    for (int k = threadIdx.x; k < KW * 64; k += BLK) Rl[k >> 6][k & 63] = Rg[(long)(k >> 6) * L + c0 + (k & 63)];
    __syncthreads();
    const long per = ((m + gridDim.y - 1) / gridDim.y + 15) / 16 * 16;
    const long i0 = (long)blockIdx.y * per;
    const long i1 = (i0 + per < m) ? i0 + per : m;
    tiles_lds<KW>(B, U, nf, L, c0, i0, i1, Rl);
}

// R = Q + N R per column (one lane per column), the whole width: R for every
// stripe once instead of once per row-range workgroup
__global__ __launch_bounds__(64) void k_rglobal(const double* Q, const double* N, int nf, long L, double* Rg) {
    const long j = (long)blockIdx.x * 64 + threadIdx.x;
    double R[KW];
#pragma unroll
    for (int t = 0; t < KW; ++t) {
        double v = 0.0;
        if (t < nf) {
            v = Q[(long)t * L + j];
#pragma unroll
            for (int s = 0; s < t; ++s) v = fma(N[t * KW + s], R[s], v);
        }
        R[t] = v;
        Rg[(long)t * L + j] = v;
    }
}


// K4: the candidate k_fold: every wave's first B tile in flight first; N
// staged transposed in LDS (zero outside the strict lower nf x nf triangle);
// wave 0 rebuilds R right-looking (after r_s is final, every later r_t takes
// its s term: the same fma order per t as fold_rebuild_R, 63 independent
// accumulators instead of one 2016-deep chain); then tiles_lds.
template <int BLK>
__global__ __launch_bounds__(BLK) void k4_fold(double* B, const double* U, const double* Q, const double* N, int nf,
                                               long m, long L, double* sink) {
    __shared__ double Rl[KW][64];
    __shared__ double NT[KW][KW];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const long c0 = (long)blockIdx.x * 64;
    for (int k = tid; k < KW * KW; k += BLK) {
        const int t = k / KW, s2 = k % KW;
        NT[s2][t] = (t < nf && s2 < t) ? N[k] : 0.0;
    }
    __syncthreads();
    if (wave == 0) {
        double R[KW];
#pragma unroll
        for (int t = 0; t < KW; ++t) R[t] = (t < nf) ? Q[(long)t * L + c0 + lane] : 0.0;
#pragma unroll
        for (int s2 = 0; s2 < KW; ++s2) {
            Rl[s2][lane] = R[s2];
#pragma unroll
            for (int t = s2 + 1; t < KW; ++t) R[t] = fma(NT[s2][t], R[s2], R[t]);
        }
    }
    __syncthreads();
    const long per = ((m + gridDim.y - 1) / gridDim.y + 15) / 16 * 16;
    const long i0 = (long)blockIdx.y * per;
    const long i1 = (i0 + per < m) ? i0 + per : m;
    tiles_lds<KW>(B, U, nf, L, c0, i0, i1, Rl);
}

// MFMA f64 issue rate: 8 independent 16x16x4 accumulators per wave
__global__ __launch_bounds__(256) void k_mfma_peak(double* out, int iters) {
    dbl4 acc[8];
    for (int j = 0; j < 8; ++j) acc[j] = dbl4{0.0, 0.0, 0.0, 0.0};
    double a = 1e-3 * threadIdx.x, b = 2e-3;
    for (int i = 0; i < iters; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[j], 0, 0, 0);
    double s = 0.0;
    for (int j = 0; j < 8; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
    if (s == 12345.0) out[0] = s;
}

// VALU f64 fma issue rate: 16 independent chains per lane
__global__ __launch_bounds__(256) void k_valu_peak(double* out, int iters) {
    double acc[16];
    for (int j = 0; j < 16; ++j) acc[j] = 1e-3 * j;
    const double a = 1.0000001, b = 1e-9 * threadIdx.x;
    for (int i = 0; i < iters; ++i)
#pragma unroll
        for (int j = 0; j < 16; ++j) acc[j] = fma(acc[j], a, b);
    double s = 0.0;
    for (int j = 0; j < 16; ++j) s += acc[j];
    if (s == 12345.0) out[0] = s;
}

// ---------------------------------------------------------------------------
// Window-tableau fold T_w += U Wt^T (T_w column-major L x n).  The MFMA kernel
// as shipped in spx_tableau.hip (copied verbatim below, Params -> TPar), and
// the VALU candidate.
// ---------------------------------------------------------------------------
typedef double dbl2 __attribute__((ext_vector_type(2)));
struct FakeSt { int nw; };
struct TPar {
    FakeSt* st;
    long m, n, L;
    double *U, *Wt, *T, *SY, *dw;
};
constexpr int TF_RB = 64;  // rows per block
constexpr int TF_UP = 68;  // LDS pitch of a staged eta row (doubles): 16-B aligned, spreads banks

template <int KW>
__global__ __launch_bounds__(256) void k_tab_fold_mfma(TPar P, int min_nw) {
    const FakeSt* st = P.st;
    const int nw = st->nw;
    if (nw < min_nw || nw < 2) return;
    const int nf = nw - 1;
    constexpr int KS = KW / 4;
    constexpr int KW2 = KW / 2;             // dbl2 per eta row
    constexpr int UPT = TF_RB * KW2 / 256;  // dbl2 staged per thread per block
    __shared__ __attribute__((aligned(16))) double Ub[2][TF_RB * TF_UP];
    const int ks = (nf + 3) / 4;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int cl = lane & 15, kr = lane >> 4;
    const int64_t m = P.m, n = P.n, L = P.L;
    const double* __restrict__ U = P.U;
    const double* __restrict__ Wt = P.Wt;
    double* __restrict__ T = P.T;
    const int64_t cb = (int64_t)blockIdx.y * 64;  // this workgroup's columns

    if (blockIdx.x == 0 && tid < 64 && cb + tid < n) {  // dw[j] += sum_{t<nf} SY[t] Wt[j][t]
        const int64_t j = cb + tid;
        double d = 0.0;
        for (int t = 0; t < nf; ++t) d = fma(P.SY[t], Wt[j * KW + t], d);
        P.dw[j] += d;
    }
    const int64_t per = ((m + gridDim.x - 1) / gridDim.x + TF_RB - 1) / TF_RB * TF_RB;
    const int64_t i_lo = (int64_t)blockIdx.x * per;
    const int64_t i_hi = (i_lo + per < m) ? i_lo + per : m;
    if (cb >= n || i_lo >= i_hi) return;  // uniform per workgroup
    const int64_t j0 = cb + 16 * wave;

    double wf[KS];
#pragma unroll
    for (int s = 0; s < KS; ++s) {
        const int t = 4 * s + kr;
        wf[s] = (j0 + cl < n && t < nf) ? Wt[(j0 + cl) * KW + t] : 0.0;
    }
    bool jok[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) jok[r] = j0 + kr + 4 * r < n;

    auto stage_load = [&](int64_t i0, dbl2 (&ur)[UPT]) {
#pragma unroll
        for (int k = 0; k < UPT; ++k) {
            const int pce = tid + 256 * k;
            const int64_t i = i0 + pce / KW2;
            ur[k] = (i < i_hi) ? reinterpret_cast<const dbl2*>(U)[i0 * KW2 + pce] : dbl2{0.0, 0.0};
        }
    };
    auto stage_write = [&](int buf, const dbl2 (&ur)[UPT]) {
#pragma unroll
        for (int k = 0; k < UPT; ++k) {
            const int pce = tid + 256 * k;
            *reinterpret_cast<dbl2*>(&Ub[buf][(pce / KW2) * TF_UP + 2 * (pce % KW2)]) = ur[k];
        }
    };
    auto tile_load = [&](int64_t i0, dbl4 (&acc)[4]) {
#pragma unroll
        for (int it = 0; it < 4; ++it) {
            const int64_t i = i0 + 16 * it + cl;
#pragma unroll
            for (int r = 0; r < 4; ++r)
                acc[it][r] = (jok[r] && i < i_hi) ? T[(j0 + kr + 4 * r) * L + i] : 0.0;
        }
    };

    dbl2 ur[UPT];
    dbl4 acc[4];
    stage_load(i_lo, ur);
    tile_load(i_lo, acc);
    stage_write(0, ur);
    __syncthreads();
    int buf = 0;
    for (int64_t i0 = i_lo; i0 < i_hi; i0 += TF_RB, buf ^= 1) {
        const bool more = i0 + TF_RB < i_hi;
        dbl4 nxt[4];
        if (more) {
            stage_load(i0 + TF_RB, ur);
            tile_load(i0 + TF_RB, nxt);
        }
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
            if (i < i_hi) {
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    if (jok[r]) T[(j0 + kr + 4 * r) * L + i] = acc[it][r];
            }
        }
        if (more) {
            stage_write(buf ^ 1, ur);
#pragma unroll
            for (int it = 0; it < 4; ++it) acc[it] = nxt[it];
        }
        __syncthreads();
    }
}


// VALU candidate: one lane per row (a wave owns 64 rows, its U row segment in
// 2 x nf VGPRs), columns walked G at a time, Wt[j][t] as scalar operands, an
// fma chain t = 0, 1, .. per element; next group's T in flight.
template <int KW, int G, bool FULL>
__global__ __launch_bounds__(256) void k_tab_fold_valu(TPar P, int nf, int cpw) {
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const long m = P.m, L = P.L;
    const int n = (int)P.n;
    const long i = ((long)blockIdx.x * 4 + wave) * 64 + lane;
    const bool ok = i < m;
    const long ic = ok ? i : m - 1;  // rows past m compute on row m-1 and store nothing
    constexpr int TN = FULL ? KW - 1 : KW;
    double u[TN];
#pragma unroll
    for (int t = 0; t < TN; ++t) u[t] = (FULL || t < nf) ? P.U[ic * KW + t] : 0.0;
    const int j0 = (int)blockIdx.y * cpw;
    const int j1 = (j0 + cpw < n) ? j0 + cpw : n;
    if (j0 >= j1) return;
    // Wt through the constant address space: uniform loads become s_load
    // (scalar operands of the fmas), not VGPR-resident vector loads
    typedef const __attribute__((address_space(4))) double* cptr;
    const cptr Wt = (cptr)P.Wt;
    double* __restrict__ T = P.T;
    auto col = [&](int j) { return (j < n) ? j : n - 1; };
    double nx[G];
#pragma unroll
    for (int c = 0; c < G; ++c) nx[c] = T[(long)col(j0 + c) * L + ic];
    for (int jj = j0; jj < j1; jj += G) {
        const int j = __builtin_amdgcn_readfirstlane(jj);
        double acc[G];
#pragma unroll
        for (int c = 0; c < G; ++c) acc[c] = nx[c];
        if (j + G < j1) {
#pragma unroll
            for (int c = 0; c < G; ++c) nx[c] = T[(long)col(j + G + c) * L + ic];
        }
        // t in chunks of TC, the next chunk's Wt scalars loaded before this
        // chunk's fmas; sched_barrier keeps the compiler from hoisting every
        // load of the column group (G x 63 doubles) into SGPRs at once
        constexpr int TC = 4;
        constexpr int NCH = (TN + TC - 1) / TC;
        double wc[G][TC], wn[G][TC];
#pragma unroll
        for (int c = 0; c < G; ++c)
#pragma unroll
            for (int k = 0; k < TC; ++k) wc[c][k] = Wt[(long)col(j + c) * KW + k];
#pragma unroll
        for (int ch = 0; ch < NCH; ++ch) {
            if (ch + 1 < NCH) {
#pragma unroll
                for (int c = 0; c < G; ++c)
#pragma unroll
                    for (int k = 0; k < TC; ++k) wn[c][k] = Wt[(long)col(j + c) * KW + (ch + 1) * TC + k];
            }
#pragma unroll
            for (int k = 0; k < TC; ++k) {
                const int t = ch * TC + k;
                if (t < TN && (FULL || t < nf)) {
#pragma unroll
                    for (int c = 0; c < G; ++c) acc[c] = fma(u[t], wc[c][k], acc[c]);
                }
            }
#pragma unroll
            for (int c = 0; c < G; ++c)
#pragma unroll
                for (int k = 0; k < TC; ++k) wc[c][k] = wn[c][k];
            asm volatile("" ::: "memory");
        }
        if (ok) {
#pragma unroll
            for (int c = 0; c < G; ++c)
                if (j + c < j1) T[(long)(j + c) * L + i] = acc[c];
        }
    }
}

// Variants of the shipped tableau fold: WAVES waves per workgroup (16 columns
// each, so 16 WAVES columns per workgroup), NBUF LDS buffers of staged U rows,
// PF = next block's T tiles in flight during this block's MFMAs.
template <int KW, int WAVES, int NBUF, bool PF, int UP = TF_UP>
__global__ __launch_bounds__(64 * WAVES) void k_tab_fold_v(TPar P, int min_nw) {
    constexpr int BLK = 64 * WAVES;
    const FakeSt* st = P.st;
    const int nw = st->nw;
    if (nw < min_nw || nw < 2) return;
    const int nf = nw - 1;
    constexpr int KS = KW / 4;
    constexpr int KW2 = KW / 2;
    constexpr int UPT = TF_RB * KW2 / BLK;
    __shared__ __attribute__((aligned(16))) double Ub[NBUF][TF_RB * UP];
    const int ks = (nf + 3) / 4;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int cl = lane & 15, kr = lane >> 4;
    const int64_t m = P.m, n = P.n, L = P.L;
    const double* __restrict__ U = P.U;
    const double* __restrict__ Wt = P.Wt;
    double* __restrict__ T = P.T;
    const int64_t cb = (int64_t)blockIdx.y * 16 * WAVES;
    const int64_t per = ((m + gridDim.x - 1) / gridDim.x + TF_RB - 1) / TF_RB * TF_RB;
    const int64_t i_lo = (int64_t)blockIdx.x * per;
    const int64_t i_hi = (i_lo + per < m) ? i_lo + per : m;
    if (cb >= n || i_lo >= i_hi) return;
    const int64_t j0 = cb + 16 * wave;
    double wf[KS];
#pragma unroll
    for (int s = 0; s < KS; ++s) {
        const int t = 4 * s + kr;
        wf[s] = (j0 + cl < n && t < nf) ? Wt[(j0 + cl) * KW + t] : 0.0;
    }
    bool jok[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) jok[r] = j0 + kr + 4 * r < n;
    auto stage_load = [&](int64_t i0, dbl2(&ur)[UPT]) {
#pragma unroll
        for (int k = 0; k < UPT; ++k) {
            const int pce = tid + BLK * k;
            const int64_t i = i0 + pce / KW2;
            ur[k] = (i < i_hi) ? reinterpret_cast<const dbl2*>(U)[i0 * KW2 + pce] : dbl2{0.0, 0.0};
        }
    };
    auto stage_write = [&](int buf, const dbl2(&ur)[UPT]) {
#pragma unroll
        for (int k = 0; k < UPT; ++k) {
            const int pce = tid + BLK * k;
            *reinterpret_cast<dbl2*>(&Ub[buf][(pce / KW2) * UP + 2 * (pce % KW2)]) = ur[k];
        }
    };
    auto tile_load = [&](int64_t i0, dbl4(&acc)[4]) {
#pragma unroll
        for (int it = 0; it < 4; ++it) {
            const int64_t i = i0 + 16 * it + cl;
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[it][r] = (jok[r] && i < i_hi) ? T[(j0 + kr + 4 * r) * L + i] : 0.0;
        }
    };
    dbl2 ur[UPT];
    dbl4 acc[4];
    stage_load(i_lo, ur);
    tile_load(i_lo, acc);
    stage_write(0, ur);
    __syncthreads();
    int buf = 0;
    for (int64_t i0 = i_lo; i0 < i_hi; i0 += TF_RB) {
        const bool more = i0 + TF_RB < i_hi;
        dbl4 nxt[4];
        if (more) {
            stage_load(i0 + TF_RB, ur);
            if (PF) tile_load(i0 + TF_RB, nxt);
        }
        const double* ub = Ub[buf];
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            if (s < ks) {
#pragma unroll
                for (int it = 0; it < 4; ++it) {
                    const double bv = ub[(16 * it + cl) * UP + 4 * s + kr];
                    acc[it] = __builtin_amdgcn_mfma_f64_16x16x4f64(wf[s], bv, acc[it], 0, 0, 0);
                }
            }
        }
#pragma unroll
        for (int it = 0; it < 4; ++it) {
            const int64_t i = i0 + 16 * it + cl;
            if (i < i_hi) {
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    if (jok[r]) T[(j0 + kr + 4 * r) * L + i] = acc[it][r];
            }
        }
        if (more) {
            if (NBUF == 1) __syncthreads();  // every wave is done reading Ub[0]
            stage_write(NBUF == 1 ? 0 : (buf ^ 1), ur);
            if (PF) {
#pragma unroll
                for (int it = 0; it < 4; ++it) acc[it] = nxt[it];
            } else {
                tile_load(i0 + TF_RB, acc);
            }
        }
        if (NBUF == 2) buf ^= 1;
        __syncthreads();
    }
}

__global__ __launch_bounds__(256) void k_flush_mall(const double* f, long n, double* sink) {
    double a = 0.0;
    for (long k = (long)blockIdx.x * 256 + threadIdx.x; k < n; k += (long)gridDim.x * 256) a += f[k];
    if (a == 1.0) sink[0] = a;
}

static double rnd(unsigned long long& s) {
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    return (double)(s >> 11) * (1.0 / 9007199254740992.0);
}

int main(int argc, char** argv) {
    const long m = argc > 1 ? atol(argv[1]) : 4096;
    const long L = m;
    const int nf = KW - 1;
    std::vector<double> hB(m * L), hU(m * KW), hQ(KW * L), hN(KW * KW, 0.0);
    unsigned long long s = 1;
    for (auto& v : hB) v = rnd(s);
    for (auto& v : hU) v = 1e-3 * (rnd(s) - 0.5);
    for (auto& v : hQ) v = rnd(s) - 0.5;
    for (int t = 0; t < KW; ++t)
        for (int u = 0; u < t; ++u) hN[t * KW + u] = 0.1 * (rnd(s) - 0.5);
    double *B, *B2, *U, *Q, *N, *Rg, *sink;
    CK(hipMalloc(&B, m * L * 8));
    CK(hipMalloc(&B2, m * L * 8));
    CK(hipMalloc(&U, m * KW * 8));
    CK(hipMalloc(&Q, KW * L * 8));
    CK(hipMalloc(&N, KW * KW * 8));
    CK(hipMalloc(&Rg, KW * L * 8));
    CK(hipMalloc(&sink, 2 * L * 8));
    CK(hipMemset(sink, 0, 2 * L * 8));
    CK(hipMemcpy(B, hB.data(), m * L * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(B2, hB.data(), m * L * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(U, hU.data(), m * KW * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(Q, hQ.data(), KW * L * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(N, hN.data(), KW * KW * 8, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int nx = (int)(L / 64);
    // each launch timed alone after a 512 MB stream has evicted the fold's
    // operands from the 256 MB MALL (the loop's folds follow the A stream)
    double* flush;
    const long nflush = 64l << 20;
    CK(hipMalloc(&flush, nflush * 8));
    CK(hipMemset(flush, 0, nflush * 8));
    auto timeit = [&](const char* name, auto fn) {
        for (int i = 0; i < 2; ++i) fn();
        CK(hipDeviceSynchronize());
        const int reps = 10;
        double us = 0.0;
        for (int r = 0; r < reps; ++r) {
            hipLaunchKernelGGL(k_flush_mall, dim3(2048), dim3(256), 0, 0, flush, nflush, sink);
            CK(hipEventRecord(e0));
            fn();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            us += 1e3 * ms / reps;
        }
        std::printf("{\"kernel\": \"%s\", \"us\": %.2f, \"GBps\": %.0f, \"TFs\": %.2f}\n", name, us,
                    16.0 * m * L / (us * 1e3), 2.0 * m * L * nf / (us * 1e6));
        std::fflush(stdout);
    };
    hipLaunchKernelGGL(k_rglobal, dim3(nx), dim3(64), 0, 0, Q, N, nf, L, Rg);
    CK(hipDeviceSynchronize());
    timeit("rglobal (R for all stripes, 64-lane WGs)",
           [&] { hipLaunchKernelGGL(k_rglobal, dim3(nx), dim3(64), 0, 0, Q, N, nf, L, Rg); });
    {
        const int it = 2048;
        auto t0 = [&] { hipLaunchKernelGGL(k_mfma_peak, dim3(2048), dim3(256), 0, 0, sink, it); };
        for (int i = 0; i < 2; ++i) t0();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        t0();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        std::printf("{\"kernel\": \"mfma f64 16x16x4 peak\", \"TFs\": %.2f}\n",
                    2048.0 * 4 * it * 8 * 2048 / (ms * 1e9));
        auto t1 = [&] { hipLaunchKernelGGL(k_valu_peak, dim3(2048), dim3(256), 0, 0, sink, it); };
        for (int i = 0; i < 2; ++i) t1();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        t1();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        std::printf("{\"kernel\": \"valu f64 fma peak\", \"TFs\": %.2f}\n",
                    2048.0 * 256 * it * 16 * 2 / (ms * 1e9));
    }
    for (int ny : {4, 8, 16}) {
        char nm[128];
        std::snprintf(nm, sizeof nm, "k4 fold 256 ny=%d", ny);
        timeit(nm, [&] { hipLaunchKernelGGL(k4_fold<256>, dim3(nx, ny), dim3(256), 0, 0, B, U, Q, N, nf, m, L, sink); });
        std::snprintf(nm, sizeof nm, "k5 ship Y+XW ny=%d", ny);
        timeit(nm, [&] { hipLaunchKernelGGL((k5_ship<true, true>), dim3(nx, ny), dim3(256), 0, 0, B, U, Q, N, nf, m, L, sink); });
        std::snprintf(nm, sizeof nm, "k5 ship bare ny=%d", ny);
        timeit(nm, [&] { hipLaunchKernelGGL((k5_ship<false, false>), dim3(nx, ny), dim3(256), 0, 0, B, U, Q, N, nf, m, L, sink); });
        std::snprintf(nm, sizeof nm, "k0 previous ny=%d", ny);
        timeit(nm, [&] { hipLaunchKernelGGL(k0_cur, dim3(nx, ny), dim3(256), 0, 0, B, U, Q, N, nf, m, L, sink); });
    }

    // ---- tableau fold: n = 4 m columns
    {
        const long n = 4 * m;
        double *T, *Wt, *SY, *dw;
        CK(hipMalloc(&T, L * n * 8));
        CK(hipMalloc(&Wt, n * KW * 8));
        CK(hipMalloc(&SY, KW * 8));
        CK(hipMalloc(&dw, n * 8));
        FakeSt* fst;
        CK(hipMalloc(&fst, sizeof(FakeSt)));
        FakeSt h{KW};
        CK(hipMemcpy(fst, &h, sizeof h, hipMemcpyHostToDevice));
        std::vector<double> hT(L * n), hW(n * KW);
        for (auto& v : hT) v = rnd(s);
        for (auto& v : hW) v = rnd(s) - 0.5;
        CK(hipMemcpy(T, hT.data(), L * n * 8, hipMemcpyHostToDevice));
        CK(hipMemcpy(Wt, hW.data(), n * KW * 8, hipMemcpyHostToDevice));
        CK(hipMemcpy(SY, hU.data(), KW * 8, hipMemcpyHostToDevice));
        CK(hipMemset(dw, 0, n * 8));
        TPar P{fst, m, n, L, U, Wt, T, SY, dw};
        auto tf = [&](const char* name, auto fn) {
            for (int i = 0; i < 2; ++i) fn();
            CK(hipDeviceSynchronize());
            const int reps = 6;
            double us = 0.0;
            for (int r = 0; r < reps; ++r) {
                hipLaunchKernelGGL(k_flush_mall, dim3(2048), dim3(256), 0, 0, flush, nflush, sink);
                CK(hipEventRecord(e0));
                fn();
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                us += 1e3 * ms / reps;
            }
            std::printf("{\"kernel\": \"%s\", \"us\": %.2f, \"GBps\": %.0f, \"TFs\": %.2f}\n", name, us,
                        16.0 * m * n / (us * 1e3), 2.0 * m * n * nf / (us * 1e6));
            std::fflush(stdout);
        };
        const long gy = (n + 63) / 64;
        long gx = (2 * 256 + gy - 1) / gy;
        tf("tab fold mfma (shipped)", [&] { hipLaunchKernelGGL(k_tab_fold_mfma<KW>, dim3(gx, gy), dim3(256), 0, 0, P, 2); });
        auto tv = [&](const char* name, auto kern, int waves, int per_cu) {
            const long gyv = (n + 16 * waves - 1) / (16 * waves);
            long gxv = ((long)per_cu * 256 + gyv - 1) / gyv;
            const long maxx = (m + 63) / 64;
            if (gxv > maxx) gxv = maxx;
            tf(name, [&] { hipLaunchKernelGGL(kern, dim3(gxv, gyv), dim3(64 * waves), 0, 0, P, 2); });
        };
        tv("tv W8 B2 noPF 2/CU UP68 (=shipped)", k_tab_fold_v<KW, 8, 2, false, 68>, 8, 2);
        tv("tv W8 B2 noPF 2/CU UP66", k_tab_fold_v<KW, 8, 2, false, 66>, 8, 2);
        tv("tv W8 B2 noPF 2/CU UP70", k_tab_fold_v<KW, 8, 2, false, 70>, 8, 2);
        tv("tv W8 B2 PF 2/CU UP66", k_tab_fold_v<KW, 8, 2, true, 66>, 8, 2);
        tv("tv W4 B2 noPF 4/CU UP66", k_tab_fold_v<KW, 4, 2, false, 66>, 4, 4);
        // the two folds of a tableau window: one after the other, or side by
        // side on two streams (they share no written data once the window reset
        // is left to a later kernel)
        {
            hipStream_t s1, s2;
            CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
            CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
            hipEvent_t ef, ej1, ej2;
            CK(hipEventCreateWithFlags(&ef, hipEventDisableTiming));
            CK(hipEventCreateWithFlags(&ej1, hipEventDisableTiming));
            CK(hipEventCreateWithFlags(&ej2, hipEventDisableTiming));
            auto tabl = [&](hipStream_t st, int per_cu) {
                const long gyv = (n + 127) / 128;
                long gxv = ((long)per_cu * 256 + gyv - 1) / gyv;
                hipLaunchKernelGGL((k_tab_fold_v<KW, 8, 2, false, 68>), dim3(gxv, gyv), dim3(512), 0, st, P, 2);
            };
            auto foldl = [&](hipStream_t st, int ny) {
                hipLaunchKernelGGL((k5_ship<true, true>), dim3(nx, ny), dim3(256), 0, st, B, U, Q, N, nf, m, L, sink);
            };
            tf("pair sequential (tab 2/CU, fold ny=8)", [&] { tabl(0, 2); foldl(0, 8); });
            auto conc = [&](int tpc, int ny) {
                CK(hipEventRecord(ef, 0));
                CK(hipStreamWaitEvent(s1, ef, 0));
                CK(hipStreamWaitEvent(s2, ef, 0));
                foldl(s2, ny);
                tabl(s1, tpc);
                CK(hipEventRecord(ej1, s1));
                CK(hipEventRecord(ej2, s2));
                CK(hipStreamWaitEvent(0, ej1, 0));
                CK(hipStreamWaitEvent(0, ej2, 0));
            };
            tf("pair concurrent (tab 2/CU, fold ny=8)", [&] { conc(2, 8); });
            tf("pair concurrent (tab 1/CU, fold ny=4)", [&] { conc(1, 4); });
            tf("pair concurrent (tab 2/CU, fold ny=4)", [&] { conc(2, 4); });
            tf("pair concurrent (tab 4/CU, fold ny=8)", [&] { conc(4, 8); });
        }
        CK(hipFree(T));
    }
    std::vector<double> o1(m * L), o2(m * L);
    double md;
    long nd;
    // k4 (whole candidate fold) against k0 (shipped fold): bit-identical expected
    CK(hipMemcpy(B, hB.data(), m * L * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(B2, hB.data(), m * L * 8, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k0_cur, dim3(nx, 16), dim3(256), 0, 0, B, U, Q, N, nf, m, L, sink);
    hipLaunchKernelGGL((k5_ship<false, false>), dim3(nx, 8), dim3(256), 0, 0, B2, U, Q, N, nf, m, L, sink);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(o1.data(), B, m * L * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(o2.data(), B2, m * L * 8, hipMemcpyDeviceToHost));
    md = 0.0;
    nd = 0;
    for (long k = 0; k < m * L; ++k) {
        const double d = std::fabs(o1[k] - o2[k]);
        if (d > md) md = d;
        nd += (o1[k] != o2[k]);
    }
    std::printf("{\"check\": \"k4 vs k0\", \"max_abs_diff\": %.3e, \"n_diff\": %ld}\n", md, nd);
    return 0;
}

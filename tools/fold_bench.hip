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
    auto timeit = [&](const char* name, auto fn) {
        for (int i = 0; i < 3; ++i) fn();
        CK(hipDeviceSynchronize());
        const int reps = 20;
        CK(hipEventRecord(e0));
        for (int i = 0; i < reps; ++i) fn();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = 1e3 * ms / reps;
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

// fold2_bench.hip — the eta-window fold B += U R in isolation (m x m
// row-major B, U m x 64, R rebuilt per 64-column stripe from base rows Q and
// coefficients N): the round-1 fold (one wave rebuilds R; B tiles moved as
// 8-byte accesses; U fragments loaded after the next tile's B prefetch)
// against spx_fold.h (first tiles in flight over the rebuild, 4-wave quad
// rebuild, column-mapped 16-byte B tiles, U fragments prefetched), plus the
// memory-only probes that found the 8-byte pattern's cost.  MALL flushed
// before every timed launch (the loop's folds follow the A stream).
// (The round-1 experiments, tools/fold_bench.hip, are in git history.)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -Isimplex_method_gpu_amd/csrc -o tools/fold2_bench tools/fold2_bench.hip
//   tools/fold2_bench [m=4096]
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

// ---- the round-1 fold (reference for timing and bits)
__device__ __forceinline__ void prev_rebuild(const double* Qrows, const double (&NT)[KW][FOLD_NP<KW>], int nf, long L,
                                             long c0, double (&Rl)[KW][64]) {
    const int lane = threadIdx.x & 63;
    double R[KW];
#pragma unroll
    for (int t = 0; t < KW; ++t) R[t] = (t < nf) ? Qrows[(long)t * L + c0 + lane] : 0.0;
#pragma unroll
    for (int s = 0; s < KW; ++s) {
        Rl[s][lane] = R[s];
#pragma unroll
        for (int t = s + 1; t < KW; ++t) R[t] = fma(NT[s][t], R[s], R[t]);
    }
}
__device__ __forceinline__ void prev_tile_load(const double* B, long L, long c0, long r0, long i1, dbl4 (&t)[4]) {
    const int lane = threadIdx.x & 63;
    const int kr = lane >> 4, cl = lane & 15;
#pragma unroll
    for (int jb = 0; jb < 4; ++jb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const long i = r0 + kr + 4 * r;
            t[jb][r] = (i < i1) ? B[i * L + c0 + 16 * jb + cl] : 0.0;
        }
}
__device__ __forceinline__ void prev_tiles(double* B, const double* U, int nf, long L, long c0, long i0, long i1,
                                           const double (&Rl)[KW][64]) {
    constexpr int KS = KW / 4;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int kr = lane >> 4, cl = lane & 15;
    const int ks = (nf + 3) / 4;
    dbl4 nxt[4];
    if (i0 + 16 * wave < i1) prev_tile_load(B, L, c0, i0 + 16 * wave, i1, nxt);
    for (long r0 = i0 + 16 * wave; r0 < i1; r0 += 64) {
        dbl4 acc[4];
#pragma unroll
        for (int jb = 0; jb < 4; ++jb) acc[jb] = nxt[jb];
        if (r0 + 64 < i1) prev_tile_load(B, L, c0, r0 + 64, i1, nxt);
        const long ia = r0 + cl;
        double af[KS];
#pragma unroll
        for (int s2 = 0; s2 < KS; ++s2) {
            const int t = 4 * s2 + kr;
            af[s2] = (ia < i1 && t < nf) ? U[ia * KW + t] : 0.0;
        }
#pragma unroll
        for (int s2 = 0; s2 < KS; ++s2)
            if (s2 < ks)
#pragma unroll
                for (int jb = 0; jb < 4; ++jb)
                    acc[jb] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[s2], Rl[4 * s2 + kr][16 * jb + cl], acc[jb], 0,
                                                                   0, 0);
#pragma unroll
        for (int jb = 0; jb < 4; ++jb)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const long i = r0 + kr + 4 * r;
                if (i < i1) B[i * L + c0 + 16 * jb + cl] = acc[jb][r];
            }
    }
}

// MODE 0: round-1 fold; 1: shipped (spx_fold.h); 2: shipped rebuild only;
// 3: shipped tiles only (R = 0)
template <int MODE, int BLK = FOLD_THREADS, int MINB = 1>
__global__ __launch_bounds__(BLK, MINB) void k_fold_v(double* B, const double* U, const double* Q, const double* N,
                                                      int nf, long m, long L, double* sink) {
    __shared__ double Rl[KW][FOLD_RP];
    __shared__ double NT[KW][FOLD_NP<KW>];
    const int tid = threadIdx.x;
    const long c0 = (long)blockIdx.x * 64;
    int64_t i0, i1;
    fold_rows(m, i0, i1);
    if (MODE == 0) {
        double (&R64)[KW][64] = *reinterpret_cast<double (*)[KW][64]>(&Rl);
        fold_stage_N<KW>(N, nf, NT);
        __syncthreads();
        if ((tid >> 6) == 0) prev_rebuild(Q, NT, nf, L, c0, R64);
        __syncthreads();
        prev_tiles(B, U, nf, L, c0, i0, i1, R64);
        return;
    }
    FoldTilePre<KW> pre;
    if (MODE == 1) fold_tile_first<KW>(B, U, nf, L, c0, i0, i1, pre);
    if (MODE != 3 && MODE != 5) {
        fold_stage_N<KW>(N, nf, NT);
        __syncthreads();
        const long long t0 = wall_clock64();
        if (tid < 256) fold_rebuild_R4<KW, FOLD_RP>(Q, NT, nf, L, c0, Rl);
        if (MODE == 2 && tid == 0) sink[L + blockIdx.x + gridDim.x * blockIdx.y] = (double)(wall_clock64() - t0);
    } else {
        for (int k = tid; k < KW * FOLD_RP; k += BLK) (&Rl[0][0])[k] = 0.0;
    }
    __syncthreads();
    if (MODE == 1) fold_tiles<KW, FOLD_RP>(B, U, nf, L, c0, i0, i1, Rl, pre, true);
    if (MODE == 3) fold_tiles<KW, FOLD_RP>(B, U, nf, L, c0, i0, i1, Rl, pre, false);
    if (MODE == 5) fold_tiles<KW, FOLD_RP, false>(B, U, nf, L, c0, i0, i1, Rl, pre, false);
    if (MODE == 2 && Rl[tid & 63][tid >> 6] == 12345.0) sink[0] = 1.0;
}

// memory-only probes over the fold's footprint (B read + written in place):
// 12 = the round-1 tile pattern (8 B per lane, 4 rows x 128 B per
// instruction), 15 = the column-mapped tile (16 B per lane, 4 rows x 256 B)
template <int MODEP>
__global__ __launch_bounds__(256) void k_memprobe(double* B, long m, long L) {
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const long c0 = (long)blockIdx.x * 64;
    int64_t i0, i1;
    fold_rows(m, i0, i1);
    for (long r0 = i0 + 16 * wave; r0 < i1; r0 += 64) {
        dbl4 t[4];
        if (MODEP == 12) prev_tile_load(B, L, c0, r0, i1, t);
        else fold_tile_load(B, L, c0, r0, i1, t);
#pragma unroll
        for (int jb = 0; jb < 4; ++jb) t[jb] *= 1.0000001;
        if (MODEP == 12) {
            const int lane = threadIdx.x & 63, kr = lane >> 4, cl = lane & 15;
#pragma unroll
            for (int jb = 0; jb < 4; ++jb)
#pragma unroll
                for (int r = 0; r < 4; ++r) B[(r0 + kr + 4 * r) * L + c0 + 16 * jb + cl] = t[jb][r];
        } else {
            fold_tile_store(B, L, c0, r0, i1, t);
        }
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
    double *B, *B2, *U, *Q, *N, *sink, *flush;
    CK(hipMalloc(&B, m * L * 8));
    CK(hipMalloc(&B2, m * L * 8));
    CK(hipMalloc(&U, m * KW * 8));
    CK(hipMalloc(&Q, KW * L * 8));
    CK(hipMalloc(&N, KW * KW * 8));
    CK(hipMalloc(&sink, 2 * L * 8));
    CK(hipMemset(sink, 0, 2 * L * 8));
    CK(hipMemcpy(B, hB.data(), m * L * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(U, hU.data(), m * KW * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(Q, hQ.data(), KW * L * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(N, hN.data(), KW * KW * 8, hipMemcpyHostToDevice));
    const long nflush = 64l << 20;
    CK(hipMalloc(&flush, nflush * 8));
    CK(hipMemset(flush, 0, nflush * 8));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int nx = (int)(L / 64);
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
    for (int ny : {4, 8}) {
        char nm[128];
#define RUN(MODE, LABEL)                                                                                \
    std::snprintf(nm, sizeof nm, "%s ny=%d", LABEL, ny);                                                \
    timeit(nm, [&] {                                                                                    \
        hipLaunchKernelGGL(k_fold_v<MODE>, dim3(nx, ny), dim3(MODE ? FOLD_THREADS : 256), 0, 0, B, U, Q, N, nf, m, L, sink); \
    });
        RUN(0, "round-1 fold");
        RUN(1, "shipped fold (spx_fold.h)");
        RUN(2, "shipped rebuild only");
        {
            std::vector<double> h(nx * ny);
            CK(hipMemcpy(h.data(), sink + L, nx * ny * 8, hipMemcpyDeviceToHost));
            double a = 0.0, mx = 0.0;
            for (double v : h) a += v / (nx * ny), mx = v > mx ? v : mx;
            int khz = 0;
            CK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
            std::printf("{\"kernel\": \"rebuild loop wave 0 (wall clock) ny=%d\", \"avg_us\": %.2f, \"max_us\": %.2f}\n", ny,
                        a / khz * 1e3, mx / khz * 1e3);
        }
        RUN(3, "shipped tiles only");
        RUN(5, "tiles only, U fragments not loaded");
        std::snprintf(nm, sizeof nm, "shipped fold, 4-wave workgroups ny=%d", ny);
        timeit(nm, [&] { hipLaunchKernelGGL((k_fold_v<1, 256, 1>), dim3(nx, ny), dim3(256), 0, 0, B, U, Q, N, nf, m, L, sink); });
        std::snprintf(nm, sizeof nm, "memprobe round-1 tile pattern (8 B/lane) ny=%d", ny);
        timeit(nm, [&] { hipLaunchKernelGGL(k_memprobe<12>, dim3(nx, ny), dim3(256), 0, 0, B2, m, L); });
        std::snprintf(nm, sizeof nm, "memprobe column-mapped tile (16 B/lane) ny=%d", ny);
        timeit(nm, [&] { hipLaunchKernelGGL(k_memprobe<15>, dim3(nx, ny), dim3(256), 0, 0, B2, m, L); });
    }
    // bits: the round-1 fold against the shipped one, same input
    std::vector<double> o1(m * L), o2(m * L);
    CK(hipMemcpy(B, hB.data(), m * L * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(B2, hB.data(), m * L * 8, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_fold_v<0>, dim3(nx, 8), dim3(256), 0, 0, B, U, Q, N, nf, m, L, sink);
    hipLaunchKernelGGL(k_fold_v<1>, dim3(nx, 4), dim3(FOLD_THREADS), 0, 0, B2, U, Q, N, nf, m, L, sink);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(o1.data(), B, m * L * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(o2.data(), B2, m * L * 8, hipMemcpyDeviceToHost));
    double md = 0.0;
    long nd = 0;
    for (long k = 0; k < m * L; ++k) {
        const double d = std::fabs(o1[k] - o2[k]);
        if (d > md) md = d;
        nd += (o1[k] != o2[k]);
    }
    std::printf("{\"check\": \"round-1 vs shipped fold\", \"max_abs_diff\": %.3e, \"n_diff\": %ld}\n", md, nd);
    return 0;
}

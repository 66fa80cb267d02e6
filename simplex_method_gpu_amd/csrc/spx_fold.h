// spx_fold.h — device helpers shared by the eta-window fold (k_fold,
// spx_kernels.hip) and the basis reinversion (spx_reinv.hip): a rank-nf
// update B += U R of a 64-column stripe of a row-major matrix with fp64 MFMA
// tiles (v_mfma_f64_16x16x4f64), R rebuilt from base rows and coefficients.
//
// Workgroup shape (FOLD_THREADS = 512, one per CU; tools/fold2_bench.hip,
// MI355X, m = 4096, KW = 64, MALL flushed: 95 -> 76 us, bit-identical):
//   0. every wave's first tile (B rows and U fragment) is loaded before
//      anything else, so HBM is busy during the rebuild (fold_tile_first);
//   1. the coefficients are staged transposed into LDS (fold_stage_N);
//   2. waves 0-3 rebuild R right-looking, a quad of lanes per column
//      (fold_rebuild_R4);
//   3. every wave walks its 16-row tiles (fold_tiles), R fragments read from
//      LDS per k-step, the next tile's U fragment and B rows loaded after
//      this tile's operands.
//
// Column map.  The MFMA accumulator of block jb holds, in lane (kr, cl), rows
// kr + 4 r (r = 0..3) and one column per cl.  Block jb, column cl stands for
// stripe column fold_col(jb, cl) = 32 (jb >> 1) + 2 cl + (jb & 1), so a lane's
// blocks 2h and 2h + 1 are two adjacent columns: the B tile moves as 16-byte
// loads and stores of 16 lanes x 16 B = 256 contiguous bytes per row (6.5
// TB/s on the fold's footprint) instead of 8-byte accesses of 128 B per row
// (1.9-3.0 TB/s).  R is stored in Rl in the same permuted order
// (fold_slot), and only the N dimension is permuted, so every sum keeps its
// order and the bits do not change.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace spx {

typedef double dbl4 __attribute__((ext_vector_type(4)));
typedef double fdbl2 __attribute__((ext_vector_type(2)));

template <int KW>
constexpr int FOLD_NP = KW + 2;  // LDS pitch of the staged coefficients
constexpr int FOLD_THREADS_H = 512;  // = FOLD_THREADS (below): threads of a fold workgroup
// LDS pitch of Rl: 72 doubles put the four k-rows of an MFMA operand read on
// different banks (fold2_bench: -2 % against 64)
constexpr int FOLD_RP = 72;

// stripe column of MFMA block jb, accumulator column cl, and its inverse
__host__ __device__ constexpr int fold_col(int jb, int cl) { return 32 * (jb >> 1) + 2 * cl + (jb & 1); }
__host__ __device__ constexpr int fold_slot(int c) { return 16 * (2 * (c >> 5) + (c & 1)) + ((c >> 1) & 15); }

// All threads: NT[s][t] = Urows[t][s] on the strict lower nf x nf triangle, 0
// elsewhere (so rows t >= nf of R rebuild to exact zeros).  Pitch KW + 2 keeps
// the transposing stores off one bank and the rows 16-byte aligned.
template <int KW>
__device__ __forceinline__ void fold_stage_N(const double* Urows, int nf, double (&NT)[KW][FOLD_NP<KW>]) {
    for (int k = threadIdx.x; k < KW * KW; k += blockDim.x) {
        const int t = k / KW, s = k % KW;
        NT[s][t] = (t < nf && s < t) ? Urows[k] : 0.0;
    }
}

// The rebuild's operands, requested before the first tiles (vmcnt retires in
// issue order, so loads issued behind the tile prefetch would wait for it):
// the coefficients Urows (thread-strided) and, per lane of waves 0-3, the base
// rows of R for its column (rows 4 u + g).  Unconditional loads with clamped
// indices, so the compiler's waits count exactly; zeroed where unused when
// consumed.
template <int KW>
struct FoldRPre {
    static constexpr int NPT = (KW * KW + FOLD_THREADS_H - 1) / FOLD_THREADS_H;
    double n[NPT];
    double q[KW / 4];
};
template <int KW>
__device__ __forceinline__ void fold_r_load(const double* Urows, const double* Qrows, int64_t L, int64_t c0,
                                            FoldRPre<KW>& r) {
    const int tid = threadIdx.x, lane = tid & 63;
#pragma unroll
    for (int j = 0; j < FoldRPre<KW>::NPT; ++j) {
        const int k = tid + j * FOLD_THREADS_H;
        r.n[j] = Urows[k < KW * KW ? k : KW * KW - 1];
    }
    const int g = lane & 3;
    const int col = (16 * (tid >> 6) + (lane >> 2)) & 63;
#pragma unroll
    for (int u = 0; u < KW / 4; ++u) r.q[u] = Qrows[(int64_t)(4 * u + g) * L + c0 + col];
}
// fold_stage_N from the preloaded coefficients
template <int KW>
__device__ __forceinline__ void fold_stage_N_pre(const FoldRPre<KW>& r, int nf, double (&NT)[KW][FOLD_NP<KW>]) {
#pragma unroll
    for (int j = 0; j < FoldRPre<KW>::NPT; ++j) {
        const int k = threadIdx.x + j * FOLD_THREADS_H;
        // (no range test when the threads tile KW x KW exactly: a guarded
        // store let the compiler sink the load into the guard and wait there)
        if ((KW * KW) % FOLD_THREADS_H == 0 || k < KW * KW) {
            const int t = k / KW, s = k % KW;
            NT[s][t] = (t < nf && s < t) ? r.n[j] : 0.0;
        }
    }
}

// DPP quad_perm of a double (both halves)
template <int CTRL>
__device__ __forceinline__ double quad_dpp(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp((int)b, (int)b, CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp((int)(b >> 32), (int)(b >> 32), CTRL, 0xF, 0xF, false);
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}

// Waves 0-3 of a fold workgroup (threadIdx.x < 256), after fold_stage_N
// and a barrier: r_t = Qrows[t] + sum_{s<t} Urows[t][s] r_s for the 64-column
// stripe at c0, into Rl (columns in fold_slot order).  Lane 4 jj + g of wave
// w owns stripe column 16 w + jj and rows t = g, g + 4, ..  Right-looking:
// once r_s is final every later r_t takes its s term, so each r_t sums s = 0,
// 1, .. in order (the bits of the left-looking recurrence); a step's 63 - s
// updates are spread over the quad's 4 lanes and the owner of row s hands r_s
// to its quad by DPP.  (One wave doing 64 columns alone was bound by its LDS
// operand latency: ~28 us of a C3 fold; this form 21-24 us with the loads.)
template <int KW, int RP>
__device__ __forceinline__ void fold_rebuild_R4(const double* Qrows, const double (&NT)[KW][FOLD_NP<KW>], int nf,
                                                int64_t L, int64_t c0, double (&Rl)[KW][RP],
                                                const FoldRPre<KW>* pre = nullptr) {
    constexpr int TG = KW / 4;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int g = lane & 3;
    const int col = 16 * wave + (lane >> 2);
    const int slot = fold_slot(col);
    double R[TG];  // R[u]: row 4 u + g
#pragma unroll
    for (int u = 0; u < TG; ++u) {
        const int t = 4 * u + g;
        R[u] = (t < nf) ? (pre ? pre->q[u] : Qrows[(int64_t)t * L + c0 + col]) : 0.0;
    }
#pragma unroll
    for (int s = 0; s < KW; ++s) {
        const int us = s >> 2;
        double rs;
        switch (s & 3) {  // r_s from the quad lane that owns row s
            case 0: rs = quad_dpp<0x00>(R[us]); break;
            case 1: rs = quad_dpp<0x55>(R[us]); break;
            case 2: rs = quad_dpp<0xAA>(R[us]); break;
            default: rs = quad_dpp<0xFF>(R[us]); break;
        }
        if (g == (s & 3)) Rl[s][slot] = R[us];
        // row 4 us + g > s only in the quad lanes past the owner
        if (g > (s & 3)) R[us] = fma(NT[s][4 * us + g], rs, R[us]);
#pragma unroll
        for (int u = us + 1; u < TG; ++u) R[u] = fma(NT[s][4 * u + g], rs, R[u]);
    }
}

// The 16-row x 64-column tile of B at rows r0.. (rows >= i1 read as 0), in the
// MFMA accumulator layout under the column map: lane (kr, cl) holds rows
// r0 + kr + 4 r, columns fold_col(jb, cl).  8 loads of 16 B per lane.
__device__ __forceinline__ void fold_tile_load(const double* B, int64_t L, int64_t c0, int64_t r0, int64_t i1,
                                               dbl4 (&t)[4]) {
    const int lane = threadIdx.x & 63;
    const int kr = lane >> 4, cl = lane & 15;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int64_t i = r0 + kr + 4 * r;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            fdbl2 v = {0.0, 0.0};
            if (i < i1) v = *reinterpret_cast<const fdbl2*>(&B[i * L + c0 + 32 * h + 2 * cl]);
            t[2 * h][r] = v.x;
            t[2 * h + 1][r] = v.y;
        }
    }
}
__device__ __forceinline__ void fold_tile_store(double* B, int64_t L, int64_t c0, int64_t r0, int64_t i1,
                                                const dbl4 (&t)[4]) {
    const int lane = threadIdx.x & 63;
    const int kr = lane >> 4, cl = lane & 15;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int64_t i = r0 + kr + 4 * r;
        if (i < i1) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                fdbl2 v;
                v.x = t[2 * h][r];
                v.y = t[2 * h + 1][r];
                *reinterpret_cast<fdbl2*>(&B[i * L + c0 + 32 * h + 2 * cl]) = v;
            }
        }
    }
}

// U fragments through LDS (SPX_FOLD_ULDS = 1): a tile's 16 x KW block of U is
// contiguous, so it is loaded as KW / 8 coalesced 16-byte loads per lane and
// staged in the wave's LDS block, from which each k-step reads its A operand
// (lane (kr, cl): U[r0 + cl][4 s2 + kr]).  Read directly, every operand load
// touched 16 rows x 32 B (16 segments per instruction): fold2_bench, C3, tiles
// 62.1 us, 47.9 us with no U loads at all.
#ifndef SPX_FOLD_ULDS
#define SPX_FOLD_ULDS 1
#endif
template <int KW>
constexpr int FOLD_UP = KW + 2;  // LDS pitch of a staged U block (16-byte rows, 2-way reads)

// A tile's operands as loaded: the B rows as the raw 16-byte loads and U (the
// MFMA A operand) raw as well.  Issued unconditionally with rows clamped into
// the range, and only turned into the accumulator layout (rows past i1 and
// pivots past nf zeroed) when the tile is taken: moving a loaded value into
// another register waits for the load, so unpacking at issue time made every
// load of the prefetch wait in turn.
template <int KW>
struct FoldTilePre {
    fdbl2 b[4][2];
#if SPX_FOLD_ULDS
    fdbl2 u[KW / 8];  // lane l, load j: U row r0 + (128 j + 2 l) / KW, column (2 l) % KW
#else
    double u[KW / 4];  // lane (kr, cl): U[r0 + cl][4 s2 + kr]
#endif
};
template <int KW, bool LOADU = true>
__device__ __forceinline__ void fold_tile_issue(const double* B, const double* U, int64_t L, int64_t c0, int64_t r0,
                                                int64_t i1, FoldTilePre<KW>& t) {
    const int lane = threadIdx.x & 63;
    const int kr = lane >> 4, cl = lane & 15;
    const int64_t ilast = i1 > 0 ? i1 - 1 : 0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int64_t i0r = r0 + kr + 4 * r;
        const int64_t i = i0r < ilast ? i0r : ilast;
#pragma unroll
        for (int h = 0; h < 2; ++h) t.b[r][h] = *reinterpret_cast<const fdbl2*>(&B[i * L + c0 + 32 * h + 2 * cl]);
    }
#if SPX_FOLD_ULDS
#pragma unroll
    for (int j = 0; j < KW / 8; ++j) {
        const int e = 128 * j + 2 * lane;
        const int64_t ia0 = r0 + e / KW;
        const int64_t ia = ia0 < ilast ? ia0 : ilast;
        t.u[j] = LOADU ? *reinterpret_cast<const fdbl2*>(&U[ia * KW + e % KW]) : fdbl2{1e-3 * (j + 1), 2e-3};
    }
#else
    const int64_t ia0 = r0 + cl;
    const int64_t ia = ia0 < ilast ? ia0 : ilast;
#pragma unroll
    for (int s2 = 0; s2 < KW / 4; ++s2) t.u[s2] = LOADU ? U[ia * KW + 4 * s2 + kr] : 1e-3 * (s2 + 1);
#endif
}
// Us: the wave's LDS block (SPX_FOLD_ULDS; af unused) or af the A operand
template <int KW>
__device__ __forceinline__ void fold_tile_take(const FoldTilePre<KW>& t, int64_t r0, int64_t i1, int nf, dbl4 (&acc)[4],
                                               double (&af)[KW / 4], double (*Us)[FOLD_UP<KW>]) {
    const int lane = threadIdx.x & 63;
    const int kr = lane >> 4, cl = lane & 15;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const bool ok = r0 + kr + 4 * r < i1;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            acc[2 * h][r] = ok ? t.b[r][h].x : 0.0;
            acc[2 * h + 1][r] = ok ? t.b[r][h].y : 0.0;
        }
    }
#if SPX_FOLD_ULDS
    (void)af;
    (void)kr;
    (void)cl;
#pragma unroll
    for (int j = 0; j < KW / 8; ++j) {
        const int e = 128 * j + 2 * lane;
        const int row = e / KW, col = e % KW;
        const bool ok = r0 + row < i1;
        fdbl2 v;
        v.x = (ok && col < nf) ? t.u[j].x : 0.0;
        v.y = (ok && col + 1 < nf) ? t.u[j].y : 0.0;
        *reinterpret_cast<fdbl2*>(&Us[row][col]) = v;
    }
#else
    (void)Us;
    const bool oka = r0 + cl < i1;
#pragma unroll
    for (int s2 = 0; s2 < KW / 4; ++s2) af[s2] = (oka && 4 * s2 + kr < nf) ? t.u[s2] : 0.0;
#endif
}

// A wave's first tile, requested before the R rebuild.
template <int KW>
__device__ __forceinline__ void fold_tile_first(const double* B, const double* U, int nf, int64_t L, int64_t c0,
                                                int64_t i0, int64_t i1, FoldTilePre<KW>& pre) {
    (void)nf;
    const int64_t r0 = i0 + 16 * (int64_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    fold_tile_issue<KW>(B, U, L, c0, r0, i1, pre);
}

// B[i0:i1, stripe c0] += U[i0:i1, 0:nf] R[0:nf, stripe] with 16x16 fp64 MFMA
// tiles (the B tile is the accumulator); U is m x KW row-major.  Wave w takes
// tiles i0 + 16 w, i0 + 16 (w + nwaves), ..  The next tile's operands are
// issued once this tile's are taken, before its MFMAs; every tile but the
// wave's last is whole (ranges are whole tiles up to m), so in the loop the
// loads and stores are unconditional and the compiler's waits exact (the next
// tile's loads wait for this tile's loads, not for its stores).
// first: the wave's first tile (fold_tile_first) when have_first.  Call
// after a barrier that published Rl.
template <int KW, int RP, bool LOADU = true>
__device__ __forceinline__ void fold_tiles(double* B, const double* U, int nf, int64_t L, int64_t c0, int64_t i0,
                                           int64_t i1, const double (&Rl)[KW][RP], const FoldTilePre<KW>& first,
                                           bool have_first) {
    constexpr int KS = KW / 4;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nwaves = blockDim.x >> 6;
    const int kr = lane >> 4, cl = lane & 15;
#if SPX_FOLD_ULDS
    // one 16-row block of U per wave; only that wave writes and reads it, and
    // its LDS operations complete in order, so no barrier guards it
    __shared__ double Ush[FOLD_THREADS_H / 64][16][FOLD_UP<KW>];
    double (*Us)[FOLD_UP<KW>] = Ush[wave];
#else
    double (*Us)[FOLD_UP<KW>] = nullptr;
#endif
    int64_t r0 = i0 + 16 * wave;
    if (r0 >= i1) return;
    const int64_t step = 16 * (int64_t)nwaves;
    const int nt = (int)((i1 - r0 + step - 1) / step);  // this wave's tiles
    FoldTilePre<KW> cur;
    if (have_first) cur = first;
    else fold_tile_issue<KW, LOADU>(B, U, L, c0, r0, i1, cur);
    // R fragment (B operand) from LDS: R[4 s2 + kr][slot 16 jb + cl].  All KS
    // k-steps run (rows t >= nf of R and U's columns past nf are exact zeros;
    // a per-step nf branch kept the next step's LDS reads behind this step's
    // MFMAs), one step's fragments read ahead: the schedule barrier keeps the
    // compiler from hoisting every step's reads (256 VGPRs, one workgroup per
    // CU) or exposing each read's latency.
    auto mfmas = [&](dbl4 (&acc)[4], const double (&af)[KS]) {
        double rf[2][4];
#if SPX_FOLD_ULDS
        double uf[2];
        uf[0] = Us[cl][kr];
#endif
#pragma unroll
        for (int jb = 0; jb < 4; ++jb) rf[0][jb] = Rl[kr][16 * jb + cl];
#pragma unroll
        for (int s2 = 0; s2 < KS; ++s2) {
            if (s2 + 1 < KS) {
#if SPX_FOLD_ULDS
                uf[(s2 + 1) & 1] = Us[cl][4 * (s2 + 1) + kr];
#endif
#pragma unroll
                for (int jb = 0; jb < 4; ++jb) rf[(s2 + 1) & 1][jb] = Rl[4 * (s2 + 1) + kr][16 * jb + cl];
            }
#if SPX_FOLD_ULDS
            const double a = uf[s2 & 1];
#else
            const double a = af[s2];
#endif
#pragma unroll
            for (int jb = 0; jb < 4; ++jb)
                acc[jb] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, rf[s2 & 1][jb], acc[jb], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
        }
    };
    for (int k = 0; k + 1 < nt; ++k, r0 += step) {  // whole tiles, next one in flight
        dbl4 acc[4];
        double af[KS];
        fold_tile_take<KW>(cur, r0, i1, nf, acc, af, Us);
        fold_tile_issue<KW, LOADU>(B, U, L, c0, r0 + step, i1, cur);
        mfmas(acc, af);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int64_t i = r0 + kr + 4 * r;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                fdbl2 v;
                v.x = acc[2 * h][r];
                v.y = acc[2 * h + 1][r];
                *reinterpret_cast<fdbl2*>(&B[i * L + c0 + 32 * h + 2 * cl]) = v;
            }
        }
    }
    dbl4 acc[4];  // the wave's last tile (rows past i1 neither read nor written)
    double af[KS];
    fold_tile_take<KW>(cur, r0, i1, nf, acc, af, Us);
    mfmas(acc, af);
    fold_tile_store(B, L, c0, r0, i1, acc);
}

// Row ranges of a fold grid: gridDim.y ranges of whole 16-row tiles.
__device__ __forceinline__ void fold_rows(int64_t m, int64_t& i0, int64_t& i1) {
    const int64_t per = ((m + gridDim.y - 1) / gridDim.y + 15) / 16 * 16;
    i0 = (int64_t)blockIdx.y * per;
    i1 = (i0 + per < m) ? i0 + per : m;
}

// Fold workgroups: 8 waves, one workgroup per CU (~70 KiB of LDS): waves
// 0-3 rebuild R (fold_rebuild_R4) while 4-7 hold their first tiles, then all
// eight walk tiles (fold2_bench, C3: 75.8 us against 81-84 us for 4-wave
// workgroups at 1 or 2 per CU).
constexpr int FOLD_THREADS = FOLD_THREADS_H;
// Host: the row split of a fold grid over nx stripes — about one workgroup
// per CU, at least one 16-row tile per wave.
inline int64_t fold_grid_y(int64_t m, int nx, int cus) {
    int64_t ny = ((int64_t)cus + nx - 1) / nx;
    const int64_t maxy = (m + 16 * (FOLD_THREADS / 64) - 1) / (16 * (FOLD_THREADS / 64));
    if (ny > maxy) ny = maxy;
    if (ny < 1) ny = 1;
    return ny;
}

}  // namespace spx

// spx_reinv.hip — gfx950 kernels of the basis reinversion (spx_reinv.h).
// Not on the per-iteration loop: it runs on demand (spx_reinvert,
// spx_set_basis) or every opts.refactor_every pivots.  Deterministic: fixed
// reduction orders, no float atomics, first-index tie-breaking, so replicated
// ranks rebuild bit-identical inverses.
#include <hip/hip_runtime.h>
#include <math.h>

#include "spx_fold.h"
#include "spx_reinv.h"

namespace spx {

namespace {

typedef double dbl2 __attribute__((ext_vector_type(2)));

constexpr int RV_BLOCK = 256;

__device__ __forceinline__ bool better(double v, int64_t j, double bv, int64_t bj) {
    return (v < bv) || (v == bv && j < bj);
}

__global__ __launch_bounds__(256) void k_rv_identity(RvParams R) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < R.m) R.X[t * R.L + t] = 1.0;  // off-diagonal zeroed by the host
}

// P_s = X[:, K_s] A[K_s, J]: one 64-row x 64-column tile per workgroup and K
// split (blockIdx.y).  Wave w: rows 16w..16w+15 of the tile, 4 column tiles
// of 16; per 32-wide K chunk a lane loads 8 consecutive doubles of its X row
// and of its A column (k = k0 + 8 (lane>>4) + s for MFMA step s, the same k
// on both operands).
__global__ __launch_bounds__(256) void k_rv_gemm(RvParams R) {
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int cl = lane & 15, kr = lane >> 4;
    const int64_t L = R.L;
    const int64_t r0 = (int64_t)blockIdx.x * 64 + 16 * wave;
    const int64_t kb = (int64_t)blockIdx.y * R.ks;
    const int64_t ke = (kb + R.ks < L) ? kb + R.ks : L;
    const int64_t row = r0 + cl;
    const bool rowok = row < R.m;
    const double* xr = R.X + (rowok ? row : 0) * L;
    const double* ac[4];
    bool cok[4];
#pragma unroll
    for (int jb = 0; jb < 4; ++jb) {
        const int t = 16 * jb + cl;
        cok[jb] = t < R.nb;
        ac[jb] = R.A + (cok[jb] ? R.cols[t] : 0) * L;
    }
    dbl4 acc[4];
#pragma unroll
    for (int jb = 0; jb < 4; ++jb) acc[jb] = dbl4{0.0, 0.0, 0.0, 0.0};
    for (int64_t k0 = kb; k0 < ke; k0 += 32) {
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
    double* out = R.Ppart + (int64_t)blockIdx.y * 64 * L;
#pragma unroll
    for (int jb = 0; jb < 4; ++jb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int64_t i = r0 + kr + 4 * r;
            if (i < R.m) out[(int64_t)(16 * jb + cl) * L + i] = acc[jb][r];
        }
}

// Pivot-row selection for panel column tcol over all k_rv_reduce / k_rv_step
// workgroups: key -|alpha_i| over free rows (first index on ties), plus max
// |alpha_i| over all rows for the singularity test.  Per-workgroup partial
// (agent-scope stores, drained) + ticket; the last workgroup decides.
__device__ void rv_select(const RvParams& R, int tcol, bool valid, double v, bool freerow, int64_t i) {
    __shared__ RvSel red[RV_BLOCK / 64];
    __shared__ int s_last;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    double key = (valid && freerow) ? -fabs(v) : INFINITY;
    int64_t idx = (valid && freerow) ? i : INT64_MAX;
    double am = valid ? fabs(v) : 0.0;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const double k2 = __shfl_xor(key, off, 64);
        const int64_t i2 = __shfl_xor(idx, off, 64);
        const double a2 = __shfl_xor(am, off, 64);
        if (better(k2, i2, key, idx)) { key = k2; idx = i2; }
        am = fmax(am, a2);
    }
    if (lane == 0) red[wave] = RvSel{key, idx, am, 0.0};
    __syncthreads();
    if (tid == 0) {
        RvSel w = red[0];
        for (int k = 1; k < RV_BLOCK / 64; ++k) {
            if (better(red[k].key, red[k].idx, w.key, w.idx)) { w.key = red[k].key; w.idx = red[k].idx; }
            w.amax = fmax(w.amax, red[k].amax);
        }
        RvSel* d = &R.parts[blockIdx.x];
        __hip_atomic_store(&d->key, w.key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&d->idx, w.idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&d->amax, w.amax, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint32_t t = __hip_atomic_fetch_add(&R.rs->ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = (t == gridDim.x - 1);
    }
    __syncthreads();
    if (!s_last || tid != 0) return;
    double bk = INFINITY, ba = 0.0;
    int64_t bi = INT64_MAX;
    for (unsigned g = 0; g < gridDim.x; ++g) {
        RvSel* d = &R.parts[g];
        const double k2 = __hip_atomic_load(&d->key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int64_t i2 = __hip_atomic_load(&d->idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const double a2 = __hip_atomic_load(&d->amax, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (better(k2, i2, bk, bi)) { bk = k2; bi = i2; }
        ba = fmax(ba, a2);
    }
    if (bi == INT64_MAX || !(-bk > 1e-11 * ba)) {
        R.rs->singular = 1;
        R.rs->bad_pos = R.pos[tcol];
    } else {
        R.qsel[tcol] = bi;
    }
    __hip_atomic_store(&R.rs->ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Panel = sum of the K-split partials in split order; then pick q_0.
__global__ __launch_bounds__(256) void k_rv_reduce(RvParams R, double* Pout) {
    if (R.rs->singular) return;
    const int64_t i = (int64_t)blockIdx.x * RV_BLOCK + threadIdx.x;
    const bool ok = i < R.m;
    const int64_t L = R.L;
    double first = 0.0;
    if (ok) {
        for (int t = 0; t < R.nb; ++t) {
            double acc = 0.0;
            for (int s2 = 0; s2 < R.S; ++s2) acc += R.Ppart[((int64_t)s2 * 64 + t) * L + i];
            Pout[(int64_t)t * L + i] = acc;
            if (t == 0) first = acc;
        }
    }
    rv_select(R, 0, ok, first, ok && R.owner[i] < 0, i);
}

// One pivot of the block (tau): eta column from panel column tau and row
// q = qsel[tau]; remaining panel columns updated into Pout (ping-pong, so
// every workgroup reads the old P[q, t]); base row and U coefficients of the
// pivot kept for the fold; then q_{tau+1} selected.
__global__ __launch_bounds__(256) void k_rv_step(RvParams R, int tau, const double* Pin, double* Pout) {
    if (R.rs->singular) return;
    const int64_t L = R.L;
    const int64_t q = R.qsel[tau];
    const double a = Pin[(int64_t)tau * L + q];
    const int64_t gt = (int64_t)blockIdx.x * RV_BLOCK + threadIdx.x;
    const int64_t i = gt;
    const bool ok = i < R.m;
    double nextv = 0.0;
    bool freerow = false;
    if (ok) {
        const double pi = Pin[(int64_t)tau * L + i];
        const double e = (i == q) ? 1.0 / a - 1.0 : -pi / a;  // compute_E_q (v4:210-215) minus e_q
        R.U[i * RV_NB + tau] = e;
        for (int t = tau + 1; t < R.nb; ++t) {
            const double v = fma(e, Pin[(int64_t)t * L + q], Pin[(int64_t)t * L + i]);
            Pout[(int64_t)t * L + i] = v;
            if (t == tau + 1) nextv = v;
        }
        freerow = R.owner[i] < 0 && i != q;
    }
    const int64_t nthreads = (int64_t)gridDim.x * RV_BLOCK;
    for (int64_t k = gt; k < L; k += nthreads) R.Qrows[(int64_t)tau * L + k] = R.X[q * L + k];
    if (gt < tau) R.Urows[tau * RV_NB + gt] = R.U[q * RV_NB + gt];
    if (gt == 0) R.owner[q] = (int32_t)R.pos[tau];
    if (tau + 1 < R.nb) rv_select(R, tau + 1, ok, nextv, freerow, i);
}

__global__ __launch_bounds__(FOLD_THREADS) void k_rv_fold(RvParams R) {
    if (R.rs->singular) return;
    __shared__ double Rl[RV_NB][FOLD_RP];
    __shared__ double NT[RV_NB][FOLD_NP<RV_NB>];
    const int64_t L = R.L;
    const int64_t c0 = (int64_t)blockIdx.x * 64;
    int64_t i0, i1;
    fold_rows(R.m, i0, i1);
    FoldTilePre<RV_NB> pre;
    fold_tile_first<RV_NB>(R.X, R.U, R.nb, L, c0, i0, i1, pre);
    fold_stage_N<RV_NB>(R.Urows, R.nb, NT);
    __syncthreads();
    if (threadIdx.x < 256) fold_rebuild_R4<RV_NB, FOLD_RP>(R.Qrows, NT, R.nb, L, c0, Rl);
    __syncthreads();
    fold_tiles<RV_NB, FOLD_RP>(R.X, R.U, R.nb, L, c0, i0, i1, Rl, pre, true);
}

// B^-1[owner[q],:] = X[q,:]
__global__ __launch_bounds__(256) void k_rv_gather(Params P, RvParams R) {
    const int64_t L2 = R.L >> 1;
    const int64_t tot = R.m * L2;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const dbl2* src = reinterpret_cast<const dbl2*>(R.X);
    dbl2* dst = reinterpret_cast<dbl2*>(P.B0);
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < tot; t += stride) {
        const int64_t q = t / L2, k = t - q * L2;
        dst[(int64_t)R.owner[q] * L2 + k] = src[t];
    }
}

// one wave per row k: c_B[k] = c[b_ixs[k]], x_b[k] = B^-1[k,:] . b (v2:396-397),
// alpha_prev = e_0 (the explicit mode's pending update becomes a no-op)
__global__ __launch_bounds__(256) void k_rv_rows(Params P) {
    const int lane = threadIdx.x & 63;
    const int64_t k = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (k >= P.m) return;
    const int64_t L2 = P.L >> 1;
    const dbl2* br = reinterpret_cast<const dbl2*>(P.B0 + k * P.L);
    const dbl2* bb = reinterpret_cast<const dbl2*>(P.b);
    double a0 = 0.0, a1 = 0.0;
    for (int64_t j = lane; j < L2; j += 64) {
        const dbl2 u = br[j], v = bb[j];
        a0 = fma(u.x, v.x, a0);
        a1 = fma(u.y, v.y, a1);
    }
    double s = a0 + a1;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    if (lane == 0) {
        DevState* st = P.st;
        P.x_b[k] = s;
        if (P.xw) P.xw[k] = s;
        P.c_B[k] = P.c[P.b_ixs[k]];
        double* ap = (st->iter & 1) ? P.alpha1 : P.alpha0;
        ap[k] = (k == 0) ? 1.0 : 0.0;
    }
}

// y partials: Ypart[s][j] = sum over rows k of split s of c_B[k] B^-1[k][j]
__global__ __launch_bounds__(256) void k_rv_ycols(Params P, double* Ypart) {
    const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (j >= P.L) return;
    const int64_t S2 = gridDim.y;
    const int64_t per = (P.m + S2 - 1) / S2;
    const int64_t k0 = (int64_t)blockIdx.y * per;
    const int64_t k1 = (k0 + per < P.m) ? k0 + per : P.m;
    double acc = 0.0;
    for (int64_t k = k0; k < k1; ++k) acc = fma(P.c_B[k], P.B0[k * P.L + j], acc);
    Ypart[(int64_t)blockIdx.y * P.L + j] = acc;
}

__global__ __launch_bounds__(256) void k_rv_yreduce(Params P, const double* Ypart, int S2) {
    DevState* st = P.st;
    const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (j < P.L) {
        double acc = 0.0;
        for (int s2 = 0; s2 < S2; ++s2) acc += Ypart[(int64_t)s2 * P.L + j];
        (st->y_buf ? P.y1 : P.y0)[j] = acc;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {  // nothing pending any more
        st->y_applied = st->iter;
        st->xb_applied = st->iter;
        st->q = 0;
        st->aq = 1.0;
        st->nw = 0;
    }
}

int grid1(int64_t work, int block) {
    int64_t g = (work + block - 1) / block;
    return (int)(g < 1 ? 1 : g);
}

}  // namespace

int rv_select_grid(int64_t m) { return grid1(m, RV_BLOCK); }

hipError_t rv_launch_identity(const RvParams& R, hipStream_t s) {
    hipLaunchKernelGGL(k_rv_identity, dim3(grid1(R.m, 256)), dim3(256), 0, s, R);
    return hipGetLastError();
}

hipError_t rv_launch_gemm(const RvParams& R, hipStream_t s) {
    hipLaunchKernelGGL(k_rv_gemm, dim3((unsigned)((R.m + 63) / 64), (unsigned)R.S), dim3(256), 0, s, R);
    return hipGetLastError();
}

hipError_t rv_launch_reduce(const RvParams& R, double* Pout, hipStream_t s) {
    hipLaunchKernelGGL(k_rv_reduce, dim3(rv_select_grid(R.m)), dim3(RV_BLOCK), 0, s, R, Pout);
    return hipGetLastError();
}

hipError_t rv_launch_step(const RvParams& R, int tau, const double* Pin, double* Pout, hipStream_t s) {
    hipLaunchKernelGGL(k_rv_step, dim3(rv_select_grid(R.m)), dim3(RV_BLOCK), 0, s, R, tau, Pin, Pout);
    return hipGetLastError();
}

hipError_t rv_launch_fold(const RvParams& R, int cus, hipStream_t s) {
    const int nx = (int)(R.L / 64);
    hipLaunchKernelGGL(k_rv_fold, dim3((unsigned)nx, (unsigned)fold_grid_y(R.m, nx, cus)), dim3(FOLD_THREADS), 0, s, R);
    return hipGetLastError();
}

int rv_y_splits(int64_t m) {
    int64_t s = (m + 63) / 64;
    return (int)(s < 1 ? 1 : (s > 64 ? 64 : s));
}

hipError_t rv_launch_finish(const Params& P, const RvParams& R, double* Ypart, hipStream_t s) {
    const int64_t tot = R.m * (R.L >> 1);
    int64_t g = (tot + 255) / 256;
    if (g > 8192) g = 8192;
    hipLaunchKernelGGL(k_rv_gather, dim3((unsigned)g), dim3(256), 0, s, P, R);
    hipLaunchKernelGGL(k_rv_rows, dim3(grid1(P.m, 4)), dim3(256), 0, s, P);
    const int S2 = rv_y_splits(P.m);
    hipLaunchKernelGGL(k_rv_ycols, dim3(grid1(P.L, 256), (unsigned)S2), dim3(256), 0, s, P, Ypart);
    hipLaunchKernelGGL(k_rv_yreduce, dim3(grid1(P.L, 256)), dim3(256), 0, s, P, (const double*)Ypart, S2);
    return hipGetLastError();
}

}  // namespace spx

// spx_common.h — device helpers shared by the loop kernels (spx_kernels.hip)
// and the persistent loop kernel (spx_loop.hip): vector types, cache-policy
// loads/stores, wave reductions, agent-scope hand-off primitives and the
// pieces of the deferred pivot (one definition, so every consumer produces
// the same bits).
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <type_traits>

#include "spx_device.h"

namespace spx {

typedef double dbl2 __attribute__((ext_vector_type(2)));

// Cache policy of the three big streams (compile-time; round-1/2 tools/policy_sweep.sh, in git history
// builds the variants): 1 = non-temporal, 0 = default.  Measured at C3:
// non-temporal loads of A cut k_price 93 -> 68 us, of B^-1 k_update 69 -> 56 us.
#ifndef SPX_NT_A
#define SPX_NT_A 1      // pricing reads of A
#endif
#ifndef SPX_NT_BLOAD
#define SPX_NT_BLOAD 1  // update reads of B_old
#endif
#ifndef SPX_NT_BSTORE
#define SPX_NT_BSTORE 1 // update writes of B_new
#endif
// Eta-window FTRAN reads of the read-only base B_w (k_update): default policy
// while B_w is at most SPX_BWIN_CACHED bytes, non-temporal beyond.  B_w is
// rewritten by k_fold's default-policy stores and read back every pass between
// A streams loaded non-temporally, so a B_w that fits the 256 MiB Infinity
// Cache stays partly resident.  Measured (round-2 tools/policy_win.sh and r02_bwin.sh, in git history):
// C3 (134 MB) k_update 31.8 us nt -> 28.0 us default; C5 (2.1 GB, two-kernel
// passes) 352-360 us nt against 383-410 us default.
#ifndef SPX_BWIN_CACHED
#define SPX_BWIN_CACHED (192ll << 20)
#endif
__host__ __device__ inline bool win_b_cached(const Params& P) { return P.m * P.L * 8 <= SPX_BWIN_CACHED; }
template <int NT>
__device__ __forceinline__ dbl2 ld2(const dbl2* p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}
// A raw buffer load of 16 bytes at byte offset off of the range rs: lanes past
// the range's size read 0 and send no memory request (word 3 of a gfx9 raw
// buffer resource: 32-bit data format, no swizzle; aux 2 = nt)
#define SPX_BUF_DW3 0x00020000
template <int NT>
__device__ __forceinline__ dbl2 ldbuf2(__amdgpu_buffer_rsrc_t rs, int off) {
    return __builtin_bit_cast(dbl2, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, NT ? 2 : 0));
}
template <int NT>
__device__ __forceinline__ void st2(dbl2 v, dbl2* p) {
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// Wave butterflies.  The partner of every step is lane ^ off, off = 32, 16,
// .., 1 (the __shfl_xor order every consumer shares, so the bits of a sum do
// not depend on the kernel computing it).  SPX_DPP_SUM = 1 moves the partner
// values with permlane swaps (32, 16), DPP row rotation (8), two banked DPP
// row shifts (4) and quad permutes (2, 1) instead of ds_bpermute: the same
// pairs (tools/dpp_sum_check.hip), so the same bits, without the LDS-path
// latency per step.
#ifndef SPX_DPP_SUM
#define SPX_DPP_SUM 1
#endif
#ifndef SPX_DPP_X4A
#define SPX_DPP_X4A 0x104  // row_shl:4 (tools/dpp_sum_check.hip picks the direction)
#define SPX_DPP_X4B 0x114  // row_shr:4
#endif
template <int CTRL, int RM, int BM>
__device__ __forceinline__ double dpp_mv(double old, double v) {
    const long long o = __double_as_longlong(old), b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp((int)o, (int)b, CTRL, RM, BM, false);
    const int hi = __builtin_amdgcn_update_dpp((int)(o >> 32), (int)(b >> 32), CTRL, RM, BM, false);
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
template <int OFF>
__device__ __forceinline__ double xor_partner(double v) {
    if constexpr (!SPX_DPP_SUM) {
        return __shfl_xor(v, OFF, 64);
    } else if constexpr (OFF == 32 || OFF == 16) {
        const int lane = threadIdx.x & 63;
        const long long b = __double_as_longlong(v);
        const bool up = OFF == 32 ? lane >= 32 : ((lane >> 4) & 1) != 0;
        int l, h;
        if constexpr (OFF == 32) {
            const auto lo = __builtin_amdgcn_permlane32_swap((int)b, (int)b, false, false);
            const auto hi = __builtin_amdgcn_permlane32_swap((int)(b >> 32), (int)(b >> 32), false, false);
            l = up ? lo[0] : lo[1];
            h = up ? hi[0] : hi[1];
        } else {
            const auto lo = __builtin_amdgcn_permlane16_swap((int)b, (int)b, false, false);
            const auto hi = __builtin_amdgcn_permlane16_swap((int)(b >> 32), (int)(b >> 32), false, false);
            l = up ? lo[0] : lo[1];
            h = up ? hi[0] : hi[1];
        }
        return __longlong_as_double((long long)(((unsigned long long)(unsigned)h << 32) | (unsigned)l));
    } else if constexpr (OFF == 8) {
        return dpp_mv<0x128, 0xF, 0xF>(v, v);  // row_ror:8 (within 16 lanes: lane ^ 8)
    } else if constexpr (OFF == 4) {
        const double t = dpp_mv<SPX_DPP_X4A, 0xF, 0x5>(v, v);  // banks 0, 2 <- lane + 4
        return dpp_mv<SPX_DPP_X4B, 0xF, 0xA>(t, v);            // banks 1, 3 <- lane - 4
    } else if constexpr (OFF == 2) {
        return dpp_mv<0x4E, 0xF, 0xF>(v, v);  // quad_perm [2,3,0,1]
    } else {
        return dpp_mv<0xB1, 0xF, 0xF>(v, v);  // quad_perm [1,0,3,2]
    }
}
__device__ __forceinline__ double wave_sum(double v) {
    v += xor_partner<32>(v);
    v += xor_partner<16>(v);
    v += xor_partner<8>(v);
    v += xor_partner<4>(v);
    v += xor_partner<2>(v);
    v += xor_partner<1>(v);
    return v;
}
// two butterflies interleaved (their cross-lane latencies overlap)
// a * b rounded on its own: no fma contraction into the sum it feeds (the
// compiler's fp-contract=fast would otherwise fuse it into the first butterfly
// add in some kernels and not in others, and a product that is fused differs
// in the last bit from one that is not)
__device__ __forceinline__ double mul_nc(double a, double b) {
#pragma clang fp contract(off)
    return a * b;
}

template <int OFF>
__device__ __forceinline__ void sum_step2(double& a, double& b) {
    const double ta = xor_partner<OFF>(a);
    const double tb = xor_partner<OFF>(b);
    a += ta;
    b += tb;
}
template <int OFF>
__device__ __forceinline__ void sum_step3(double& a, double& b, double& c) {
    const double ta = xor_partner<OFF>(a);
    const double tb = xor_partner<OFF>(b);
    const double tc = xor_partner<OFF>(c);
    a += ta;
    b += tb;
    c += tc;
}
__device__ __forceinline__ void wave_sum3(double& a, double& b, double& c) {
    sum_step3<32>(a, b, c);
    sum_step3<16>(a, b, c);
    sum_step3<8>(a, b, c);
    sum_step3<4>(a, b, c);
    sum_step3<2>(a, b, c);
    sum_step3<1>(a, b, c);
}
__device__ __forceinline__ void wave_sum2(double& a, double& b) {
    sum_step2<32>(a, b);
    sum_step2<16>(a, b);
    sum_step2<8>(a, b);
    sum_step2<4>(a, b);
    sum_step2<2>(a, b);
    sum_step2<1>(a, b);
}

// ---- DPP cross-lane moves (gfx9 encodings; VALU-rate, no LDS round trip).
// dpp_* returns v of the source lane the control selects, or old in lanes the
// row mask leaves out.
enum : int {
    DPP_XOR1 = 0xB1,         // quad_perm [1,0,3,2]
    DPP_XOR2 = 0x4E,         // quad_perm [2,3,0,1]
    DPP_HALF_MIRROR = 0x141, // lane i <- 7 - i within 8
    DPP_MIRROR = 0x140,      // lane i <- 15 - i within a row of 16
    DPP_BCAST15 = 0x142,     // rows 1, 3 <- lane 15 of the row before (row mask 0xA)
    DPP_BCAST31 = 0x143,     // rows 2, 3 <- lane 31 (row mask 0xC)
};
template <int CTRL, int RM = 0xF>
__device__ __forceinline__ int dpp_i(int old, int v) {
    return __builtin_amdgcn_update_dpp(old, v, CTRL, RM, 0xF, false);
}
template <int CTRL, int RM = 0xF>
__device__ __forceinline__ int64_t dpp_l(int64_t old, int64_t v) {
    const int lo = dpp_i<CTRL, RM>((int)old, (int)v);
    const int hi = dpp_i<CTRL, RM>((int)(old >> 32), (int)(v >> 32));
    return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
template <int CTRL, int RM = 0xF>
__device__ __forceinline__ double dpp_d(double old, double v) {
    return __longlong_as_double(dpp_l<CTRL, RM>(__double_as_longlong(old), __double_as_longlong(v)));
}
// value of lane l (l wave-uniform) in every lane
__device__ __forceinline__ int64_t readlane_l(int64_t v, int l) {
    const int lo = __builtin_amdgcn_readlane((int)v, l);
    const int hi = __builtin_amdgcn_readlane((int)(v >> 32), l);
    return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
__device__ __forceinline__ double readlane_d(double v, int l) {
    return __longlong_as_double(readlane_l(__double_as_longlong(v), l));
}

// Lane reductions in the pairing order of __shfl_xor offsets 1, 2, 4, ...:
// the mirror and broadcast moves pair the same lane groups once each group
// holds its own total, so a sum has the bits of that butterfly.  N = 8: every
// lane of each aligned group of 8 ends with the group's result; N = 64: lane
// 63 ends with the wave's (the other lanes hold partial results).
template <int N, class Step>
__device__ __forceinline__ void lane_reduce(Step step) {
    static_assert(N == 8 || N == 64, "lane_reduce: 8 or 64 lanes");
    step(std::integral_constant<int, DPP_XOR1>(), std::integral_constant<int, 0xF>());
    step(std::integral_constant<int, DPP_XOR2>(), std::integral_constant<int, 0xF>());
    step(std::integral_constant<int, DPP_HALF_MIRROR>(), std::integral_constant<int, 0xF>());
    if constexpr (N == 64) {
        step(std::integral_constant<int, DPP_MIRROR>(), std::integral_constant<int, 0xF>());
        step(std::integral_constant<int, DPP_BCAST15>(), std::integral_constant<int, 0xA>());
        step(std::integral_constant<int, DPP_BCAST31>(), std::integral_constant<int, 0xC>());
    }
}
// (value, index) argmin with argmin_better's order (smallest index on ties)
template <int N>
__device__ __forceinline__ void lane_argmin(double& v, int64_t& j) {
    lane_reduce<N>([&](auto c, auto rm) {
        const double v2 = dpp_d<decltype(c)::value, decltype(rm)::value>(v, v);
        const int64_t j2 = dpp_l<decltype(c)::value, decltype(rm)::value>(j, j);
        if ((v2 < v) || (v2 == v && j2 < j)) {
            v = v2;
            j = j2;
        }
    });
}
template <int N>
__device__ __forceinline__ void lane_sum(double& v) {
    // lanes the row mask leaves out add old = 0.0
    lane_reduce<N>([&](auto c, auto rm) { v += dpp_d<decltype(c)::value, decltype(rm)::value>(0.0, v); });
}
template <int N>
__device__ __forceinline__ void lane_isum(int& v) {
    lane_reduce<N>([&](auto c, auto rm) { v += dpp_i<decltype(c)::value, decltype(rm)::value>(0, v); });
}

template <typename T>
__device__ __forceinline__ void st_agent(T* p, T v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T>
__device__ __forceinline__ T ld_agent(const T* p) {
    return __hip_atomic_load(const_cast<T*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void drain_vmem() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Last-arrival detection for a one-shot grid (the workgroup that runs a
// kernel's tail).  Atomics on one counter serialise at ~12 ns each
// (MI355X_MICROARCH.md, "fanin"), so 512 arrivals on one line cost ~6 us
// after the last workgroup's stream ends.  Instead the workgroups of shard
// blockIdx.x % ARR_SHARDS count on a line of their own and the last arriver
// of each shard counts on the root line: <= 64 + 8 serial adds at C3.
// Callers drain their partial stores (sc1, vmcnt(0)) before arriving, as for
// a single counter; every counter is reset by the workgroup that closes it,
// so the next launch starts from zero.  ctr: ARR_LINES lines of 128 B.
__device__ __forceinline__ bool arrive_last(uint32_t* ctr, uint32_t nblocks, uint32_t b) {
    const uint32_t s = b % ARR_SHARDS;
    const uint32_t nshard = (nblocks - s + ARR_SHARDS - 1) / ARR_SHARDS;
    uint32_t* line = ctr + (1 + s) * ARR_STRIDE;
    if (__hip_atomic_fetch_add(line, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != nshard - 1) return false;
    __hip_atomic_store(line, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t nroot = nblocks < ARR_SHARDS ? nblocks : ARR_SHARDS;
    if (__hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != nroot - 1) return false;
    __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return true;
}
__device__ __forceinline__ uint32_t* arrive_group(uint32_t* arrive, int g) { return arrive + g * ARR_LINES * ARR_STRIDE; }
// Workgroup barrier for data exchanged through LDS only: the LDS operations
// complete (lgkmcnt), global loads and stores stay in flight across it
// (__syncthreads()'s workgroup fence would wait for them: vmcnt(0)).
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ bool stopped(const DevState* st) {
    return st->status != ST_RUNNING || st->iter >= st->limit;
}
__device__ __forceinline__ bool stopped(const DevState& s) { return s.status != ST_RUNNING || s.iter >= s.limit; }
// The loop state in one memory round trip: DevState as independent 16-byte
// loads issued together.  (The kernels also store to *st, so the compiler
// cannot use scalar loads, and field-by-field reads became a chain of
// dependent vector round trips at kernel entry.)
__device__ __forceinline__ DevState st_snapshot(const DevState* st) {
    static_assert(sizeof(DevState) % 16 == 0, "DevState is a whole number of 16-byte words");
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    struct Words {
        u32x4 w[sizeof(DevState) / 16];
    } v;
    const u32x4* p = reinterpret_cast<const u32x4*>(st);
#pragma unroll
    for (int i = 0; i < (int)(sizeof(DevState) / 16); ++i) v.w[i] = p[i];
    return __builtin_bit_cast(DevState, v);
}

__device__ __forceinline__ unsigned long long rtime() { return __builtin_amdgcn_s_memrealtime(); }

// compute_E_q (v4:210-215)
__device__ __forceinline__ double eta_entry(double a_i, int64_t i, int64_t q, double aq) {
    return (i != q) ? (-a_i / aq) : (1.0 / aq - 1.0);
}
// y += s_y r (v4:356)
__device__ __forceinline__ dbl2 y_apply(double s_y, dbl2 r, dbl2 y) {
    dbl2 o;
    o.x = fma(s_y, r.x, y.x);
    o.y = fma(s_y, r.y, y.y);
    return o;
}

// Merge of ratio-test partials: argmin on (theta, idx) carrying the winner's
// scalars; nonpos and T summed.  Callers fix the order of the sums.
__device__ __forceinline__ void upd_merge(UpdPartial& a, const UpdPartial& b) {
    if (argmin_better(b.theta, b.idx, a.theta, a.idx)) {
        a.theta = b.theta;
        a.idx = b.idx;
        a.a_w = b.a_w;
        a.cb_w = b.cb_w;
        a.bix_w = b.bix_w;
    }
    a.nonpos += b.nonpos;
    a.T += b.T;
}
// the same merge with selects (the workgroup's final merge of its wave
// partials: the branch form became a scalar branch per step on the uniform
// LDS values, each step waiting for its own read)
__device__ __forceinline__ void upd_merge_sel(UpdPartial& a, const UpdPartial& b) {
    const bool t = argmin_better(b.theta, b.idx, a.theta, a.idx);
    a.theta = t ? b.theta : a.theta;
    a.idx = t ? b.idx : a.idx;
    a.a_w = t ? b.a_w : a.a_w;
    a.cb_w = t ? b.cb_w : a.cb_w;
    a.bix_w = t ? b.bix_w : a.bix_w;
    a.nonpos += b.nonpos;
    a.T += b.T;
}
__device__ __forceinline__ UpdPartial upd_empty() { return UpdPartial{INFINITY, INT64_MAX, 0, 0.0, 0.0, 0.0, -1, 0}; }
__device__ __forceinline__ UpdPartial upd_shfl_xor(const UpdPartial& v, int off) {
    UpdPartial o;
    o.theta = __shfl_xor(v.theta, off, 64);
    o.idx = __shfl_xor(v.idx, off, 64);
    o.nonpos = __shfl_xor(v.nonpos, off, 64);
    o.T = __shfl_xor(v.T, off, 64);
    o.a_w = __shfl_xor(v.a_w, off, 64);
    o.cb_w = __shfl_xor(v.cb_w, off, 64);
    o.bix_w = __shfl_xor(v.bix_w, off, 64);
    o.pad = 0;
    return o;
}

// y-update scalar (v4:352-355): c_B_new.E_q + c_p - c_Bq with E_i = -alpha_i /
// alpha_q (i != q), E_q = 1/alpha_q - 1, c_B_new[q] = c_p, evaluated from the
// gathered T = sum_i c_B[i] alpha_i (so the tail needs no O(m) pass):
// c_B_new.E_q = -(T - c_Bq alpha_q)/alpha_q + c_p (1/alpha_q - 1).
__device__ __forceinline__ double y_scalar(double T, double aq, double c_bq, double c_p) {
    const double sy = -(T - c_bq * aq) / aq + c_p * (1.0 / aq - 1.0);
    return sy + (c_p - c_bq);  // compute_scalar (v4:195-197)
}

}  // namespace spx

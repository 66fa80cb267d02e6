// spx_grid.h — the grid barrier of the persistent cooperative kernels
// (k_loop, spx_loop.hip; k_tab_loop, spx_tableau.hip).  Device code only.
#pragma once
#include <hip/hip_runtime.h>

#include "spx_common.h"
#include "spx_loop.h"

namespace spx {

// Entry check of a persistent launch: a plain launch does not guarantee that
// all workgroups are resident together (another stream or process may hold
// CUs), and a grid barrier over a partly resident grid only ends at its spin
// bound.  Every workgroup counts itself in before it reads or writes any
// state, then waits (bounded by the wall clock, SPX_ARRIVE_TICKS of the
// 100 MHz s_memrealtime) until the whole grid has arrived.  If it has not,
// err = 2, nores += 1 and every workgroup leaves at once -- those not yet
// resident leave when they start, seeing err -- so the launch changes nothing
// and the host reruns its passes as two-kernel passes (iterate_persist).
#ifndef SPX_ARRIVE_TICKS
#define SPX_ARRIVE_TICKS 200000ull  // 2 ms
#endif
__device__ __forceinline__ bool grid_arrive(LoopState* ls, int* s_ok) {
    if (threadIdx.x == 0) {
        int ok = 1;
        const uint32_t G = gridDim.x;
        const uint32_t old = __hip_atomic_fetch_add(&ls->arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (ld_agent(&ls->err)) ok = 0;
        else if (old + 1 < G) {
            const unsigned long long t0 = rtime();
            uint32_t spins = 0;
            while (ld_agent(&ls->arrive) < G) {
                if ((++spins & 63u) == 0) {
                    if (ld_agent(&ls->err)) { ok = 0; break; }
                    if (rtime() - t0 > SPX_ARRIVE_TICKS) {
                        int expected = 0;  // the first to time out counts the launch
                        if (__hip_atomic_compare_exchange_strong(&ls->err, &expected, 2, __ATOMIC_RELAXED,
                                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                            __hip_atomic_fetch_add(&ls->nores, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        drain_vmem();
                        ok = 0;
                        break;
                    }
                }
            }
            // (all arrived: a late err from a timed-out peer still wins)
            if (ok && ld_agent(&ls->err)) ok = 0;
        }
        *s_ok = ok;
    }
    __syncthreads();
    return *s_ok != 0;
}

// Grid barrier: every wave drains its stores, workgroup barrier, one lane
// adds to the counter and polls it (sc1) up to the target, workgroup barrier.
// Bounded: returns false (and sets err) when the counter does not arrive.
__device__ __forceinline__ bool grid_sync(LoopState* ls, uint32_t target, int* s_ok) {
    drain_vmem();
    __syncthreads();
    if (threadIdx.x == 0) {
        int ok = 1;
        const uint32_t old = __hip_atomic_fetch_add(&ls->bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (old + 1 < target) {
            uint32_t spins = 0;
            // one load in flight per poll; the error word and the spin
            // bound are checked every 256 polls only
            while (ld_agent(&ls->bar) < target) {
                if ((++spins & 255u) == 0 && (spins > (1u << 24) || ld_agent(&ls->err))) {
                    st_agent(&ls->err, 1);
                    ok = 0;
                    break;
                }
            }
        }
        *s_ok = ok;
    }
    __syncthreads();
    return *s_ok != 0;
}


}  // namespace spx

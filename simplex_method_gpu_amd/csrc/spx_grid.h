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
// The failure is sticky: nores is not reset between the launches of one call,
// so once a launch has found its grid not resident every later launch of that
// call leaves at entry as well, and the device window stays where the host's
// readback after the call finds it (a later resident launch could otherwise
// start from a window the host had already counted as advanced).
//
// Timeout and completion are exclusive through the arrive word itself: a
// workgroup that times out CASes arrive from the count it observed (< G) to
// that count | ARRIVE_CLOSED.  A fetch_add that returns a value with the bit
// set came after the close and leaves; a failed CAS means another workgroup
// arrived (or closed) in between, so the spinner re-reads instead of closing.
// Nobody proceeds unless it saw arrive == G with the bit clear, and once the
// bit is set arrive can never read G.
#ifndef SPX_ARRIVE_TICKS
#define SPX_ARRIVE_TICKS 200000ull  // 2 ms
#endif
constexpr uint32_t ARRIVE_CLOSED = 0x80000000u;
__device__ __forceinline__ bool grid_arrive(LoopState* ls, int* s_ok) {
    if (threadIdx.x == 0) {
        int ok = 1;
        const uint32_t G = gridDim.x;
        const uint32_t old = __hip_atomic_fetch_add(&ls->arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((old & ARRIVE_CLOSED) || ld_agent(&ls->nores) || ld_agent(&ls->err)) ok = 0;
        else if (old + 1 < G) {
            const unsigned long long t0 = rtime();
            uint32_t spins = 0;
            for (;;) {
                uint32_t v = ld_agent(&ls->arrive);
                if (v & ARRIVE_CLOSED) { ok = 0; break; }
                if (v >= G) break;
                if ((++spins & 63u) == 0 && rtime() - t0 > SPX_ARRIVE_TICKS) {
                    // close the entry at the count seen; losing the CAS means
                    // the count moved (or someone closed it): look again
                    if (__hip_atomic_compare_exchange_strong(&ls->arrive, &v, v | ARRIVE_CLOSED, __ATOMIC_RELAXED,
                                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                        st_agent(&ls->err, 2);
                        __hip_atomic_fetch_add(&ls->nores, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        drain_vmem();
                        ok = 0;
                        break;
                    }
                }
            }
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

// spx_grid.h — the grid barrier of the persistent cooperative kernels
// (k_loop, spx_loop.hip; k_tab_loop, spx_tableau.hip).  Device code only.
#pragma once
#include <hip/hip_runtime.h>

#include "spx_common.h"
#include "spx_loop.h"

namespace spx {

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

// spx_tableau.h — host-side launchers of the window-tableau kernels
// (spx_tableau.hip; SPX_FLAG_TABLEAU).
#pragma once
#include <hip/hip_runtime.h>

#include "spx_device.h"
#include "spx_loop.h"

namespace spx {

// T_w += U Wt^T and dw += SY Wt^T for the nw-1 complete pivots of the window
// when nw >= min_nw (the same test as k_fold, which must run after it: k_fold
// resets nw).  No-op unless P.tab.
hipError_t launch_tab_fold(const Params& P, int min_nw, int cus, hipStream_t s);
// B_w from T_w's slack block (P.tab_slack; before readbacks that read B_w)
hipError_t launch_tab_binv(const Params& P, hipStream_t s);
// T_w = B_w A (B_w = P.B0, row-major): after a reinversion or a warm start.
hipError_t launch_tab_build(const Params& P, hipStream_t s);
// Persistent tableau loop (k_tab_loop): whole passes in one cooperative
// launch; grid_hint > 0 forces the workgroup count; ok = false when it cannot
// be used (caches do not fit, or no cooperative launch).
hipError_t tab_loop_prepare(const Params& P, int cus, int grid_hint, LoopCfg& c);
hipError_t launch_tab_loop(const Params& P, const LoopArgs& a, const LoopCfg& c, hipStream_t s);
// bytes of the loop's partial buffers (LoopArgs::xp, ::xu) for c.grid workgroups
void tab_loop_partial_bytes(const LoopCfg& c, size_t* xp, size_t* xu);

}  // namespace spx

// spx_loop.h — the persistent loop kernel (spx_loop.hip): whole simplex
// passes of the eta-window representation in ONE cooperative launch, one
// workgroup per CU, two grid barriers per pass instead of two kernel
// boundaries.
//
// Per pass, every workgroup:
//   A  prices its share of the non-basic columns (grid-stride over the compact
//      list, the last pivot's list change applied as a local patch): e_j and
//      the pending pivot's row entry r.A_j -> Wt[j][tau]; workgroup argmin
//      partial.                                             -> grid barrier 1
//   B  reduces the pricing partials itself (every workgroup, same order, same
//      result: no broadcast needed), then FTRAN + ratio test for its own rows
//      of B_w; ratio-test partial.                          -> grid barrier 2
//   C  reduces the ratio-test partials itself, decides q, s_y and the list
//      change, stages the new pending base row B_w[q,:] in LDS; workgroup 0
//      writes the global bookkeeping.  No barrier: the next pass's readers of
//      that bookkeeping either use the local patch or read it after barrier 1.
// Cross-workgroup data moves only through agent-scope (sc1) stores and loads,
// every storing wave drains (s_waitcnt vmcnt(0)) before the workgroup barrier
// behind which one lane adds to the grid counter (MI355X_MICROARCH.md, valid
// hand-off forms, first table row).  Every spin is bounded: a barrier that
// does not complete sets err and all workgroups leave.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "spx_device.h"

namespace spx {

struct alignas(16) LoopState {
    uint32_t bar;    // grid barrier counter (zeroed before every launch)
    int32_t err;     // 1: a barrier timed out; 2: the grid was not co-resident
    int32_t passes;  // passes completed by this launch
    uint32_t arrive; // workgroups that reached the entry check (grid_arrive)
    // not zeroed per launch: launches whose grid was not all resident
    // (another kernel or process held CUs), read and cleared by the host
    int32_t nores;
    int32_t pad[3];
};
// bytes of LoopState reset before every launch
constexpr size_t LOOP_STATE_RESET = 16;

struct LoopArgs {
    PricePartial* pp;           // G pricing partials
    UpdPartial* up;             // G ratio-test partials
    LoopState* ls;
    unsigned long long* clock;  // optional: per pass {start, barrier 1, barrier 2} (s_memrealtime), WG 0
    int32_t npasses;            // passes to run (the window must not fill)
    uint32_t epoch;             // tableau loop: launch number (tags of the partial words)
    void* xp;                   // tableau loop: G tagged pricing partials (spx_tableau.hip)
    void* xu;                   // tableau loop: G tagged ratio-test partials
    int32_t call_launch;        // host: launch number within one spx_iterate call (SPX_LOOP_OVERSUB=2)
};

struct LoopCfg {
    int block = 1024;   // threads per workgroup
    int grid = 0;       // workgroups = CUs (co-resident: cooperative launch)
    bool lds_r = true;  // pending base row in LDS next to y_w
    size_t lds_bytes = 0;
    bool ok = false;    // the persistent path is usable for this context
    int bc_lds = 0;     // compact FTRAN operand: A_p-on-the-list doubles in LDS (0: none)
    int cpw = 0;        // tableau loop: list slots cached per wave
    int rw = 0;         // tableau loop: rows per wave
};

// Shapes the launch for P (window mode, one rank); ok = false when the device
// cannot hold one workgroup per CU.
hipError_t loop_prepare(const Params& P, int cus, LoopCfg& c, bool want_bc = false);
hipError_t launch_loop(const Params& P, const LoopArgs& a, const LoopCfg& c, hipStream_t s);

// the grid a persistent launch uses (tests: SPX_LOOP_OVERSUB=1 oversubscribes
// every launch, =2 only the first launch of each spx_iterate call)
int loop_grid_launched(int grid, int call_launch);

}  // namespace spx

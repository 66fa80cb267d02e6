// spx_kernels.h — host-side launchers for the gfx950 kernels (spx_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "spx_device.h"

namespace spx {

struct PriceCfg {
    int block;         // 256 / 512 / 1024 threads
    bool lds_y;        // stage y in LDS (L*8 bytes) or read it from global
    int wm;            // 0 explicit B^-1; eta window: 1 base row in LDS, 2 in global; 3 tableau;
                       // 4 / 5 = 1 / 2 with steepest edge (B_w^T alpha in LDS / global)
    size_t lds_bytes;  // dynamic LDS per workgroup
    int grid;          // workgroups (persistent-style, grid-stride over columns)
    bool tk = false;   // wm 1: the instantiation with the ticketed tail (Params::price_dyn)
};

struct UpdateCfg {
    int block;  // threads per workgroup (256 / 512 / 1024)
    int rows;   // B^-1 rows per wave (1/2/4/8)
    int grid;   // ceil(m / (block / 64 * rows))
    int bc_entry;  // compact FTRAN, 1 row per wave: k_ftran_bc (>= 1) or k_update<..., BC> (0);
                   // with the deferred tail, k_ftran_bc's rows per wave (1, 2, 4: SPX_FTRAN_RPW)
    int mark;      // diagnostic: k_mark before the launch (SPX_DIAG_MARK=1, stamps only)
};

bool kernels_inplace();  // B^-1 updated in place (one buffer) or ping-pong
hipError_t price_prepare(const PriceCfg& c, int* blocks_per_cu);
hipError_t launch_price(const Params& P, const PriceCfg& c, hipStream_t s, hipEvent_t e0, hipEvent_t e1);
hipError_t launch_update(const Params& P, const UpdateCfg& c, hipStream_t s, hipEvent_t e0, hipEvent_t e1);
// a pending deferred ratio-test tail (Params::defer_tail), applied on its own
hipError_t launch_apply_tail(const Params& P, hipStream_t s);
hipError_t launch_generate(double* A, double* b, double* c, int64_t m, int64_t n, int64_t L, uint64_t seed,
                           hipStream_t s);
hipError_t launch_reset(const Params& P, hipStream_t s);
hipError_t launch_flush(const Params& P, hipStream_t s);
hipError_t launch_finalize_rs(const Params& P, hipStream_t s);
hipError_t launch_exchange(const Params& P, hipStream_t s);
hipError_t launch_compact(const Params& P, hipStream_t s);
hipError_t launch_tail(const Params& P, int nparts, hipStream_t s);
hipError_t launch_materialize(const Params& P, double* out, hipStream_t s);
hipError_t launch_reduced_costs(const Params& P, double* e, hipStream_t s);
hipError_t launch_objective(const Params& P, hipStream_t s);
hipError_t launch_fold(const Params& P, int min_nw, int cus, hipStream_t s);
// steepest edge (P.steep): weights at the slack basis; B_w^T alpha, U^T alpha
// and gamma_p of the pending pivot before a pricing pass
hipError_t launch_se_init(const Params& P, hipStream_t s);
hipError_t launch_se_prep(const Params& P, hipStream_t s, int fused_parts = 0);  // fused_parts: the FTRAN pass's partials
int se_parts_for(int64_t m);

}  // namespace spx

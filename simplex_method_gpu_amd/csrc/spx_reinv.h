// spx_reinv.h — basis reinversion on the device (spx_reinvert / spx_set_basis,
// SURVEY.md §8f row 4): B^-1 rebuilt from the basis columns of A.
//
// Procedure (the same as oracle/simplex_oracle.c orc_reinvert, blocked):
//   X = I (the slack basis; A's last m columns are the identity, v4:272-277).
//   Every slack column n-m+i of the target basis keeps row i.  The structural
//   columns, in basis order, are pivoted in 64 at a time:
//     k_rv_gemm    P = X A_J for the block's columns J (m x m x 64 fp64 MFMA,
//                  split over K; partials summed in fixed order by k_rv_reduce)
//     k_rv_step    for tau = 0..nb-1: q_tau = argmax |P[:,tau]| over free rows
//                  (first index on ties; singular when |P[q,tau]| <= 1e-11 max
//                  |P[:,tau]|), eta column into U, P[:,t>tau] += eta P[q,t],
//                  base row X[q,:] and U[q,0:tau] kept for the fold
//     k_rv_fold    X += U R (rank-nb, spx_fold.h: the eta-window fold's tiles)
//   Then B^-1[k,:] = X[row owned by position k,:], x_b = B^-1 b, c_B, and
//   y = c_B B^-1 (the v2 formulas, v2_quadratic_B_inv.cu:337-338,396-397).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "spx_device.h"

namespace spx {

constexpr int RV_NB = 64;  // pivots per block (the MFMA fold's width)

struct alignas(16) RvSel {  // argmax partial: key = -|alpha| (argmin order), idx, max |alpha|
    double key;
    int64_t idx;
    double amax;
    double pad;
};

struct alignas(16) RvState {
    int32_t singular;  // set once a column had no pivot above tolerance
    uint32_t ticket;
    int64_t bad_pos;   // basis position of that column
};

struct RvParams {
    const double* A;
    int64_t m, L;
    double* X;        // m x L row-major: the inverse being built
    double* Ppart;    // S x 64 x L split-K partials of the panel
    int32_t S;        // K splits of k_rv_gemm
    int32_t nb;       // columns in the current block
    int64_t ks;       // K range per split (multiple of 32)
    double* U;        // m x 64 eta columns of the block
    double* Qrows;    // 64 x L base rows X[q_tau,:]
    double* Urows;    // 64 x 64 coefficients U[q_tau][s < tau]
    int32_t* owner;   // m: basis position owning the row, -1 free
    const int64_t* cols;  // block columns (global index in A)
    const int64_t* pos;   // their basis positions
    int64_t* qsel;        // 64 selected rows
    RvSel* parts;         // per-workgroup selection partials
    RvState* rs;
};

hipError_t rv_launch_identity(const RvParams& R, hipStream_t s);
hipError_t rv_launch_gemm(const RvParams& R, hipStream_t s);
hipError_t rv_launch_reduce(const RvParams& R, double* Pout, hipStream_t s);
hipError_t rv_launch_step(const RvParams& R, int tau, const double* Pin, double* Pout, hipStream_t s);
hipError_t rv_launch_fold(const RvParams& R, int cus, hipStream_t s);
int rv_select_grid(int64_t m);  // workgroups of k_rv_reduce / k_rv_step (RvSel partials needed)

// Finish: B^-1 rows from X (B = P.B0), c_B from b_ixs, x_b = B^-1 b, y =
// c_B B^-1 into ybuf[st->y_buf], and the deferred-state fields reset so no
// pivot is pending (y_applied = xb_applied = iter, nw = 0, xw = x_b; the
// explicit mode's pending rank-1 update made a no-op: alpha_prev = e_0, q = 0,
// aq = 1).  Ypart: S2 x L scratch, S2 = rv_y_splits(m).
int rv_y_splits(int64_t m);
hipError_t rv_launch_finish(const Params& P, const RvParams& R, double* Ypart, hipStream_t s);

}  // namespace spx

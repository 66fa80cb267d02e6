// spx_device.h — device-state layout and kernel parameter block shared by the
// gfx950 kernels (spx_kernels.hip) and the host runtime (spx_api.cpp).
//
// HBM layout (all fp64, L = round_up(m, 128) doubles = whole 1 KiB lines):
//   A      L x n, column-major (column j at A + j*L; rows m..L-1 zero).  The
//          reference's D = [-c; A] copy (v4:248,278-279) is not built: pricing
//          reads A and c directly.
//   B[2]   m x L, ROW-major B^-1 (the reference is column-major, v4:59-60), two
//          buffers: the update kernel reads B[iter&1] and writes B[(iter+1)&1].
//          The true inverse is B[iter&1] + E[iter&1] r[iter&1]^T (one rank-1
//          update is always pending and is applied inside the next FTRAN).
//   E[2], r[2]  pending eta column and pivot row (L each, padding zero).
//   y, x_b, c_B, alpha (L each), b_ixs (m int64), b (L), c (n).
//   nb_list / nb_pos   this rank's non-basic columns (compact list + position,
//          swap-remove / append per pivot) so pricing touches non-basic
//          columns only.
#pragma once
#include <stdint.h>

namespace spx {

enum : int32_t { ST_RUNNING = 0, ST_OPTIMAL = 1, ST_UNBOUNDED = 2 };

// (value, global index) candidate; the order is value, then smallest index —
// cub::DeviceReduce::ArgMin's first-index semantics (v4:294,324) for every
// reduction tree, every grid and every rank count.
struct alignas(16) ArgMinEntry {
    double val;
    int64_t idx;
};

struct alignas(16) UpdPartial {
    double theta;
    int64_t idx;
    int64_t nonpos;
    int64_t pad;
};

struct alignas(16) DevState {
    int32_t status;      // ST_*
    int32_t nb_count;    // entries in nb_list
    int64_t iter;        // pivots made
    int64_t limit;       // kernels do nothing once iter >= limit
    int64_t p;           // last entering column
    int64_t q;           // last leaving row
    double min_e;        // last entering reduced cost
    double z;            // objective (spx_objective)
    uint32_t ticket_price;
    uint32_t ticket_update;
    int64_t pad[2];
};

__host__ __device__ inline bool argmin_better(double v, int64_t j, double bv, int64_t bj) {
    return (v < bv) || (v == bv && j < bj);
}

struct Params {
    // problem
    const double* A;
    const double* b;
    const double* c;
    int64_t m, n, L, ns;   // ns = n - m structural columns
    double eps;
    // basis state
    double* B0;
    double* B1;
    double* E0;
    double* E1;
    double* r0;
    double* r1;
    double* y;
    double* x_b;
    double* c_B;
    double* alpha;
    int64_t* b_ixs;
    int32_t* nb_list;
    int32_t* nb_pos;       // n entries, -1 when basic or not owned
    // column shard of this rank: structural [s_lo, s_hi), slack [k_lo, k_hi)
    int64_t s_lo, s_hi, k_lo, k_hi;
    // reductions
    ArgMinEntry* price_partials;
    ArgMinEntry* price_out;        // this rank's entering candidate
    const ArgMinEntry* price_in;   // all ranks' candidates (== price_out at 1 rank)
    int32_t nin;
    UpdPartial* upd_partials;
    DevState* st;
    // diagnostics (SPX_FLAG_STAMPS): per kernel {min WG start, sum body, sum tail}
    // in s_memrealtime ticks (100 MHz); nullptr in normal runs
    unsigned long long* stamps;
};

__host__ __device__ inline bool owns_col(const Params& P, int64_t j) {
    return (j < P.ns) ? (j >= P.s_lo && j < P.s_hi) : (j >= P.k_lo && j < P.k_hi);
}

}  // namespace spx

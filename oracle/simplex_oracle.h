/*
 * simplex_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (fp64) of the reference's dense revised-simplex loop
 * (Girjoaba/simplex_method_gpu, src/v4_cub_reduction.cu:219-380).  It is the
 * parity checker for the HIP product path and the `cpu_baseline` leg of
 * bench.py.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * may load it; the product (libsimplex.so, ./solver) never links it.
 *
 * Parity pinning: the reference ships no tests; its only known answer is
 * input/sample.txt:15-16 (z = 9 at x0 = 1, x1 = 3).  The restatement is
 * checked against that and against golden optima produced in this container
 * by an independent solver (scipy 1.15.3 HiGHS, tests/golden/make_golden.py),
 * standing in for the GLPK driver (solver_glpk.cpp:23) whose library is not
 * installed here.  The reference binaries themselves cannot be built here
 * (CUDA/cuBLAS/CUB absent).
 */
#ifndef SIMPLEX_ORACLE_H
#define SIMPLEX_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Status values follow the reference's SolveStatus (v4_cub_reduction.cu:49-54). */
enum {
    ORC_MAX_ITER = 0,
    ORC_OPTIMUM_FOUND = 1,
    ORC_UNBOUNDED = 2,
    ORC_THETA_OVERFLOW = 3
};

/* splitmix64 finaliser and the seeded uniform of SURVEY.md §8(d). */
uint64_t orc_splitmix64(uint64_t x);
double orc_uniform(uint64_t seed, uint64_t stream, uint64_t idx);

/* Dense random LP of SURVEY.md §8(d): A = [U | I_m] (column-major, ld = m),
 * b_i = (n-m)/4 * U(1,2), c_j = U(0,1) for structural columns, 0 for slacks. */
void orc_generate(int64_t m, int64_t n, uint64_t seed,
                  double* A_colmajor, double* b, double* c);

/* Full solve, restating v4_cub_reduction.cu:268-368 in fp64.
 *   A_colmajor: m x n, column j at A + j*m (the reference's R2C, v4:59-60)
 *   max_iter  : loop passes (reference MAX_ITER, v4:19)
 *   eps       : optimality tolerance on reduced costs (reference EPS, v4:18)
 *   threads   : OpenMP threads (<= 0: runtime default)
 * Outputs (any may be NULL):
 *   z, x_b[m], b_ixs[m]     basic solution in basis order (v4:363-368)
 *   pivots                  pivots completed (the reference's loop counter i)
 *   trace_p/trace_q[trace_cap]  entering / leaving index of the first pivots
 *   y_out[m]                final simplex multipliers y = c_B B^-1
 *   binv_out[m*m]           final B^-1, ROW-major (binv_out[i*m + k])
 * Unlike the reference, z/x_b/b_ixs are written for every status so tests can
 * inspect partial runs.  Returns the status. */
int orc_solve(int64_t m, int64_t n, const double* A_colmajor,
              const double* b, const double* c,
              int64_t max_iter, double eps, int threads,
              double* z, double* x_b, int64_t* b_ixs, int64_t* pivots,
              int64_t* trace_p, int64_t* trace_q, int64_t trace_cap,
              double* y_out, double* binv_out);

/* Extended options, mirroring spx_opts of the product:
 *   ratio: 0 reference (v4:199-208), 1 guarded, 2 Harris (include/simplex.h
 *          SPX_RATIO_* has the definitions; piv_tol / feas_tol as there)
 *   refactor_every: rebuild B^-1 from the basis columns (orc_reinvert) every
 *          K pivots, then x_b = B^-1 b and y = c_B B^-1 (0 = never). */
typedef struct {
    int64_t max_iter;
    double eps;
    int threads;
    int ratio;
    double piv_tol;
    double feas_tol;
    int64_t refactor_every;
    int pricing; /* 0 Dantzig (v4:288-302), 1 Devex (simplex_oracle.c devex_choose),
                    2 steepest edge with the Goldfarb-Reid recurrence (se_choose) */
    double* w_out; /* optional: the final pricing weights (n), Devex / steepest edge */
} orc_opts;

void orc_default_opts(orc_opts* o);

/* orc_solve with orc_opts; same outputs. */
int orc_solve_ex(int64_t m, int64_t n, const double* A_colmajor,
                 const double* b, const double* c, const orc_opts* o,
                 double* z, double* x_b, int64_t* b_ixs, int64_t* pivots,
                 int64_t* trace_p, int64_t* trace_q, int64_t trace_cap,
                 double* y_out, double* binv_out);

/* Basis reinversion by pivoting the basis columns into the slack basis
 * (the procedure libsimplex's spx_reinvert runs on the device):
 *   X = I; every slack column n-m+i of the basis keeps row i; then, in basis
 *   order, every structural column j: alpha = X A_j, q = argmax |alpha_i|
 *   over rows not yet taken (first index on ties), singular when
 *   |alpha_q| <= 1e-11 max_i |alpha_i|; X += eta X[q,:] with the compute_E_q
 *   column (v4:210-215) minus e_q; row q taken by j.  Finally B^-1[k,:] =
 *   X[row of basis[k],:], so B^-1 follows the given basis order.
 * Requires A's last m columns to be the identity (the reference's slack
 * assumption, v4:272-277).  Outputs (any may be NULL): binv_out ROW-major,
 * x_b = B^-1 b, y = c_B B^-1 (c_B[k] = c[basis[k]]).  Returns 0, -1 on bad
 * input (index out of range / repeated), -7 when singular. */
int orc_reinvert(int64_t m, int64_t n, const double* A_colmajor,
                 const double* b, const double* c, const int64_t* basis,
                 int threads, double* binv_out, double* x_b, double* y);

/* Timed sample for the CPU baseline: runs `iters` pivots from the slack basis
 * and returns wall seconds of the iteration loop only (steady clock). */
double orc_time_iterations(int64_t m, int64_t n, const double* A_colmajor,
                           const double* b, const double* c,
                           int64_t iters, int threads, int64_t* done);

/* Reduced costs e_j = -c_j + y.A_j for every column (v4:288-290), for
 * per-step parity tests. */
void orc_price(int64_t m, int64_t n, const double* A_colmajor,
               const double* c, const double* y, double* e, int threads);

int orc_max_threads(void);

#ifdef __cplusplus
}
#endif
#endif

/*
 * simplex.h — C-ABI of libsimplex, the MI355X (gfx950) dense revised-simplex
 * hot loop.  Plain pointers and sizes only; no HIP, torch or C++ types.
 *
 * What it replaces in the reference (Girjoaba/simplex_method_gpu):
 *   spx_create + spx_solve + spx_destroy
 *        <- std::pair<real,SolveStatus> solve(real* A, real* b, real* c,
 *              real* x_b, int* b_ixs, int m, int n, TimeStruct&)
 *              src/v4_cub_reduction.cu:219-380 (host buffers in, x_b/b_ixs out)
 *   spx_price   <- pricing Sgemm + entering ArgMin + optimality test
 *              src/v4_cub_reduction.cu:288-302
 *   spx_pivot   <- FTRAN Sgemv, compute_theta, leaving ArgMin, E_q, Sger,
 *              basis bookkeeping, x_b and y updates
 *              src/v4_cub_reduction.cu:306-357 (kernels :195-215)
 *   status codes <- enum class SolveStatus, src/v4_cub_reduction.cu:49-54
 * The `./solver <file>` CLI built on top of this header replaces main()
 * (src/v4_cub_reduction.cu:384-473).
 *
 * Conventions
 *   - A is m x n COLUMN-major (column j at A + j*m), as the reference's R2C
 *     (src/v4_cub_reduction.cu:59-60); the last m columns must be the slack
 *     identity and b >= 0 (the reference's unchecked assumption, v4:272-277).
 *   - Everything is fp64.  Indices are 0-based int64.
 *   - Every function returns SPX_OK (0) or a negative SPX_ERR_* code; nothing
 *     exits or throws across the ABI.  spx_last_error() gives a message.
 *   - The caller owns host buffers; the context owns device memory.  One
 *     context per host thread; a context is not re-entrant.
 *   - Multi-GPU: one process per GPU.  Pricing columns are sharded over
 *     opts.nranks ranks (structural and slack columns each split in
 *     contiguous blocks); B^-1, x_b, y are replicated.  After spx_create,
 *     every rank calls spx_attach_comm with the id rank 0 obtained from
 *     spx_comm_unique_id (exchange it out of band, e.g. torch.distributed).
 */
#ifndef SIMPLEX_MI355X_H
#define SIMPLEX_MI355X_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SPX_ABI_VERSION 8

/* SolveStatus of the reference (v4_cub_reduction.cu:49-54), same numbering. */
#define SPX_STATUS_MAX_ITER       0
#define SPX_STATUS_OPTIMUM_FOUND  1
#define SPX_STATUS_UNBOUNDED      2
#define SPX_STATUS_THETA_OVERFLOW 3 /* kept for ABI parity; unreachable since v2 */

#define SPX_OK             0
#define SPX_ERR_ARG       -1  /* bad argument (m > n, m <= 0, NULL, ...)     */
#define SPX_ERR_HIP       -2  /* a HIP runtime call failed                     */
#define SPX_ERR_OOM       -3  /* device allocation failed                      */
#define SPX_ERR_RCCL      -4  /* an RCCL call failed                           */
#define SPX_ERR_STATE     -5  /* call not valid in the context's state         */
#define SPX_ERR_NO_DEVICE -6  /* no HIP device visible                         */
#define SPX_ERR_SINGULAR  -7  /* spx_reinvert / spx_set_basis: the basis matrix
                                 is singular (no pivot above tolerance)        */

typedef struct spx_ctx spx_ctx;

typedef struct spx_opts {
    double  eps;          /* optimality tolerance on reduced costs: optimum when
                             min_j e_j >= -eps (reference EPS, v4:18: 1e-4 f32);
                             default 1e-7 (fp64)                */
    int32_t device;       /* HIP device ordinal; -1 = keep the current device  */
    int32_t rank;         /* pricing shard of this process (default 0)         */
    int32_t nranks;       /* number of shards (default 1)                      */
    int32_t graph_batch;  /* iterations per captured hipGraph; 0 = auto (16,
                             RCCL calls captured too; a capture RCCL refuses
                             falls back to eager), -1 = eager launches       */
    int32_t price_block;  /* tuning: threads per pricing workgroup, 0 = auto   */
    int32_t update_rows;  /* tuning: B^-1 rows per wave in the update, 0 = auto */
    int32_t price_grid;   /* tuning: pricing workgroups, 0 = auto              */
    int32_t flags;        /* SPX_FLAG_* bits                                   */
    int32_t update_block; /* tuning: threads per update workgroup, 0 = auto    */
    int32_t window;       /* B^-1 representation: 0 = auto
                             (window 64 at m >= 2048, else explicit),
                             -1 = explicit B^-1 rewritten by a rank-1 update
                             every pivot (v4:331-333), 8/16/32/64 = eta window:
                             B^-1 = B_w + U R kept for up to window-1 pivots,
                             then folded by one rank-(window-1) update.  The
                             window is single-shard / replicated-B^-1 only.   */
    int32_t ratio_test;   /* leaving-row rule, SPX_RATIO_* (default REFERENCE)  */
    int32_t refactor_every; /* spx_solve / spx_iterate: rebuild B^-1 from the
                             basis columns (spx_reinvert) every K pivots;
                             0 = never (the reference never does)            */
    double  piv_tol;      /* SPX_RATIO_GUARDED / HARRIS: rows need alpha_i >
                             piv_tol (default 1e-9)                           */
    double  feas_tol;     /* SPX_RATIO_HARRIS: primal feasibility tolerance
                             delta of the first pass (default 1e-9)          */
    int32_t pricing;      /* entering-column rule, SPX_PRICING_* (default DANTZIG) */
    int32_t loop_block;   /* tuning: threads per workgroup of the persistent loop
                             kernel (512 / 1024), 0 = auto                     */
    int32_t trace_cap;    /* record the first trace_cap pivots' (entering column
                             p, leaving row q) on the device, written by the
                             kernel that commits each pivot (spx_get_trace);
                             0 = off.  The reference prints nothing of the
                             kind; the parity tests compare it with the
                             oracle's pivot sequence.                        */
    int32_t reserved;
} spx_opts;

/* Entering-column rules (README.md:16-17 "steepest edge").
 * DANTZIG: most negative e_j (v4:288-302).
 * DEVEX:   Devex reference weights w_j (1 at the start): after a pivot with
 *          pivot element alpha_q, entering weight w_p and pivot row
 *          alpha_rj = r.A_j (r = row q of B^-1 before the pivot),
 *          w_j = max(w_j, (alpha_rj/alpha_q)^2 w_p) for non-basic j and
 *          w_leave = max(w_p/alpha_q^2, 1); p = argmin of -e_j^2/w_j over
 *          e_j < -eps (first index on ties).  The pivot row comes free from
 *          the eta-window pricing pass (it computes r.A_j for every column),
 *          so DEVEX needs the window (opts.window 0 selects 64).  On a column-
 *          shard group the winner's record carries its reduced cost and weight
 *          (not with SPX_FLAG_SPLIT_TAIL / SPX_RATIO_HARRIS).  spx_price's min_e
 *          is then the entering column's reduced cost. */
#define SPX_PRICING_DANTZIG 0
#define SPX_PRICING_DEVEX   1
/* STEEPEST: steepest edge with a recurrence (README.md:16-17): exact weights
 *          gamma_j = 1 + ||B^-1 A_j||^2, 1 + ||A_j||^2 at the slack basis,
 *          kept by Goldfarb & Reid's update after a pivot with alpha = B^-1 A_p,
 *          pivot element alpha_q, pivot row alpha_rj, g = alpha_rj / alpha_q,
 *          gamma_p = 1 + ||alpha||^2 and d_j = A_j . B^-T alpha (B^-1 before
 *          the pivot): gamma_j = max(gamma_j - 2 g d_j + g^2 gamma_p, 1 + g^2),
 *          gamma_leave = max(gamma_p / alpha_q^2, 1); p = argmin of
 *          -e_j^2/gamma_j over e_j < -eps.  d_j rides on the pricing pass's
 *          A stream as a third dot (B_w^T alpha in LDS beside y_w and the base
 *          row, plus the window terms), so it needs the window, runs two-kernel
 *          passes, and not with the tableau; on a column-shard group as DEVEX
 *          (every rank forms B_w^T alpha from the replicated B^-1).  spx_set_basis
 *          restarts the weights at 1 + ||A_j||^2. */
#define SPX_PRICING_STEEPEST 2

/* Leaving-row rules.
 * REFERENCE: theta_i = x_b_i / alpha_i over alpha_i > 0, first index on ties
 *            (compute_theta + ArgMin, v4:199-208,324); no guard, no filter.
 * GUARDED:   only alpha_i > piv_tol (the pivot-size guard of the thesis code,
 *            archive/thesis/cpu/liblp.c:39, gpu/culiblp.cu:401) and
 *            theta_i = max(x_b_i, 0) / alpha_i (its x_b >= -EPS filter,
 *            liblp.c:18-20; README.md:29-30 "x_b_t < 0", "division by a small
 *            number").
 * HARRIS:    two passes: theta_max = min (max(x_b_i,0) + feas_tol) / alpha_i
 *            over alpha_i > piv_tol, then the largest alpha_i among rows with
 *            max(x_b_i,0) / alpha_i <= theta_max (first index on ties).
 *            Single rank or replicated B^-1 only; runs the pivot tail as its
 *            own launch. */
#define SPX_RATIO_REFERENCE 0
#define SPX_RATIO_GUARDED   1
#define SPX_RATIO_HARRIS    2

#define SPX_FLAG_TIMING 1 /* record per-kernel hipEvents (spx_kernel_times)  */
#define SPX_FLAG_STAMPS 2 /* in-kernel phase stamps (spx_phase_times); diagnostic */
#define SPX_FLAG_GLOBAL_Y 4 /* pricing reads y from global memory instead of LDS
                               (automatic when L*8 bytes do not fit in LDS)   */
#define SPX_FLAG_SPLIT_TAIL 16 /* tuning: run the pivot tail as its own launch
                                  instead of the update kernel's last workgroup */
#define SPX_FLAG_NO_PERSIST 32 /* tuning: never use the persistent loop kernel */
#define SPX_FLAG_PERSIST 64    /* tuning: use the persistent cooperative loop kernel
                                  (k_loop: one launch per window, two grid
                                  barriers per pass instead of two kernels) where
                                  it applies (window > 0, one rank, no Harris, no
                                  stamps).  Default: only when y_w and the base
                                  row do not both fit in LDS (m > ~9400, e.g. C5:
                                  +7 %); at C3 the two-kernel pass is faster.   */
#define SPX_FLAG_COMM1 128 /* test: with nranks == 1, run the MINLOC exchange through
                              RCCL anyway (spx_attach_comm with a one-rank id), so
                              the communicator path, graph-captured RCCL calls
                              included, can be checked on one GPU            */
#define SPX_FLAG_TABLEAU 256 /* window tableau: with the eta window,
                                also keep T_w = B_w A and dw = y_w A - c in HBM and
                                fold them with B_w (fp64 MFMA), so a pass reads no
                                A column and no B_w row: pricing reads T_w[q, j],
                                dw[j] and the window row of each non-basic column,
                                FTRAN the column T_w[:, p].  Needs the window (0 =
                                auto selects 64) and one rank; twice A's memory. */
#define SPX_FLAG_COUNTED_TAIL 512 /* tuning: the update kernel's workgroups hand
                                     their ratio-test partials (and the pricing
                                     kernel's, where it reduces them itself)
                                     to the tail by drained stores + a
                                     last-arrival count instead of tagged
                                     words polled by the last workgroup (the
                                     default)                                 */
#define SPX_FLAG_PRICE_TAIL 1024 /* tuning: the pricing kernel's last workgroup
                                    merges the entering candidates (default on
                                    one rank with the window: every update
                                    workgroup merges k_price's partials)     */
#define SPX_FLAG_ROW_SHARD 8 /* nranks > 1: B^-1 row-sharded over the ranks
                                (ceil(m/nranks) rows each) instead of
                                replicated; one extra all-gather per pass
                                carries the pivot row.  Readback functions
                                then gather x_b over the communicator
                                (collective: every rank must call them).     */

void spx_default_opts(spx_opts* opts);

/* Allocate device state, upload A (column-major, ld = m), b, c and set the
 * slack basis (B^-1 = I, x_b = b, y = c_B; v4:268-280). */
int spx_create(spx_ctx** out, int64_t m, int64_t n, const double* A_colmajor,
               const double* b, const double* c, const spx_opts* opts);

/* Same, but A, b, c are produced on the device by the seeded generator of
 * SURVEY.md §8(d) (bit-identical to oracle/simplex_oracle.c orc_generate). */
int spx_create_generated(spx_ctx** out, int64_t m, int64_t n, uint64_t seed,
                         const spx_opts* opts);

void spx_destroy(spx_ctx* ctx);

/* RCCL plumbing for opts.nranks > 1 (no-ops returning SPX_OK when nranks == 1). */
#define SPX_COMM_ID_BYTES 128
int spx_comm_unique_id(uint8_t id[SPX_COMM_ID_BYTES]);
int spx_attach_comm(spx_ctx* ctx, const uint8_t id[SPX_COMM_ID_BYTES]);

/* Evidence of what actually joined the exchange (no reference counterpart:
 * the reference is one process on one GPU).  out[0] = ranks the attached RCCL
 * communicator reports (ncclCommCount; -1 when none is attached), out[1] =
 * this rank in it (ncclCommUserRank; -1), out[2] = the HIP device RCCL bound
 * (ncclCommCuDevice; -1), out[3] = the context's HIP device ordinal, out[4] =
 * 1 when loop passes replay captured hipGraphs (the all-gathers inside them),
 * 0 when they run eagerly, out[5] = 1 when a capture with RCCL calls failed
 * and the context fell back to eager passes, out[6] = opts.nranks, out[7] =
 * opts.rank.  bus_id: the context device's PCI bus id (hipDeviceGetPCIBusId,
 * NUL-terminated).  Whether graphs are used is known once the first batch
 * has been captured (the first spx_iterate long enough for one). */
#define SPX_COMM_INFO_FIELDS 8
#define SPX_BUS_ID_BYTES 64
int spx_comm_info(spx_ctx* ctx, int32_t out[SPX_COMM_INFO_FIELDS], char bus_id[SPX_BUS_ID_BYTES]);

/* Peer mailboxes: the pricing MINLOC exchange (the RCCL all-gather of the
 * candidate records after src/v4_cub_reduction.cu:294-302's argmin) as direct
 * stores into every rank's device mailbox over xGMI, one small kernel per pass
 * (k_exchange), instead of ncclAllGather.  Every rank calls spx_mbox_export,
 * gathers all handles in rank order out of band (e.g. torch.distributed
 * all_gather_object) and calls spx_mbox_attach with them; from then on the
 * MINLOC exchange goes through the mailboxes.  The row-sharded B^-1 still
 * needs spx_attach_comm (its ratio-test exchange is RCCL).  Collective in
 * effect: all ranks must attach before any of them iterates.  Handles are
 * hipIpcMemHandle_t bytes; a rank's own handle is not opened (its mailbox is
 * used directly), so one rank (SPX_FLAG_COMM1) runs the same kernel alone.
 * Ranks may share a device (several processes on one GPU). */
#define SPX_MBOX_HANDLE_BYTES 64
int spx_mbox_export(spx_ctx* ctx, uint8_t handle[SPX_MBOX_HANDLE_BYTES]);
int spx_mbox_attach(spx_ctx* ctx, const uint8_t* handles /* nranks x SPX_MBOX_HANDLE_BYTES */);

/* In-process shard group: G contexts created with nranks = G and ranks
 * 0..G-1 (any devices, no communicator) run k lockstep iterations with the
 * MINLOC candidates exchanged by device-to-device copies instead of RCCL
 * (one host thread drives all shards; single-process multi-GPU, and the
 * way the sharded path is validated on one GPU).  status/pivots: rank 0's. */
int spx_group_iterate(spx_ctx** ctxs, int32_t G, int64_t k, int32_t* status,
                      int64_t* pivots);

/* Row-sharded groups (SPX_FLAG_ROW_SHARD, no communicator): flush every
 * member and copy each member's x_b rows to all members, so per-context
 * readback (spx_get_state x_b / spx_objective / spx_solve) is complete.
 * spx_get_state's B^-1 then still holds only the member's own rows. */
int spx_group_sync(spx_ctx** ctxs, int32_t G);

/* Back to the slack basis (keeps A, b, c). */
int spx_reset(spx_ctx* ctx);

/* Rebuild B^-1 from the current basis columns of A on the device (pivot-in
 * reinversion, 64-column MFMA blocks; procedure: oracle/simplex_oracle.h
 * orc_reinvert) and recompute x_b = B^-1 b, y = c_B B^-1 (the v2 formulas,
 * v2_quadratic_B_inv.cu:337-338,396-397).  The basis order is kept.  Also
 * run every opts.refactor_every pivots by spx_iterate / spx_solve.  Replicated
 * B^-1 only (not with SPX_FLAG_ROW_SHARD).  SPX_ERR_SINGULAR when the basis
 * matrix has no pivot above 1e-11 of a column's largest entry.  With
 * nranks > 1 every rank must call it (no communication; the results are
 * bit-identical). */
int spx_reinvert(spx_ctx* ctx);

/* Warm start: make basis[0..m) (distinct column indices, basis order) the
 * current basis, B^-1 by reinversion, status back to running (pivot count
 * kept).  The primal simplex needs x_b = B^-1 b >= 0: read x_b back to check.
 * On SPX_ERR_SINGULAR the context has no valid basis until spx_reset. */
int spx_set_basis(spx_ctx* ctx, const int64_t* basis);

/* Whole solve, device-resident: at most max_iter loop passes (reference
 * MAX_ITER, v4:19, do/while at v4:286-359).  Writes z, x_b[m], b_ixs[m] (basis
 * order) for every status (the reference writes them only on optimum);
 * pivots = pivots made (the reference's loop counter).  Any output may be
 * NULL.  Continues from the current basis (call spx_reset to restart). */
int spx_solve(spx_ctx* ctx, int64_t max_iter, double* z, int64_t* b_ixs,
              double* x_b, int32_t* status, int64_t* pivots);

/* Run up to k further pivots with no host synchronisation between them; one
 * sync at the end.  status: SPX_STATUS_MAX_ITER while the loop can go on. */
int spx_iterate(spx_ctx* ctx, int64_t k, int32_t* status, int64_t* pivots);

/* Step-wise API (tests/debugging; each call synchronises).
 * spx_price: pricing + entering argmin (+ cross-rank MINLOC).  p = entering
 *   column (first index on ties), min_e = its reduced cost, optimal = 1 when
 *   min_e >= -eps.
 * spx_pivot: apply the pending rank-1 update of B^-1 fused with FTRAN
 *   (alpha = B^-1 A_p), ratio test + leaving argmin, E_q, x_b, y, c_B, basis
 *   bookkeeping.  Requires a preceding spx_price.  status after the pivot. */
int spx_price(spx_ctx* ctx, int64_t* p, double* min_e, int32_t* optimal);
int spx_pivot(spx_ctx* ctx, int64_t* q, int32_t* status);

/* Current state (any pointer may be NULL).  binv_rowmajor: m*m, B^-1[i][k] at
 * i*m + k (with the pending rank-1 update applied). */
int spx_get_state(spx_ctx* ctx, double* x_b, int64_t* b_ixs, double* y,
                  double* c_b, double* binv_rowmajor, int32_t* status,
                  int64_t* pivots);

/* Reduced costs e_j = -c_j + y.A_j for all n columns from the current y
 * (debug/parity; basic columns included, like v4:288-290). */
int spx_reduced_costs(spx_ctx* ctx, double* e);

/* Objective z = c_B . x_b (v4:365), computed on the device. */
int spx_objective(spx_ctx* ctx, double* z);

/* Pivot trace (opts.trace_cap > 0): copies the first min(pivots made,
 * trace_cap, cap) pivots' entering columns into p[] and leaving rows into q[]
 * (either may be NULL) and stores that count in *count.  Indexed by pivot
 * number, so a spx_reset / re-solve overwrites it. */
int spx_get_trace(spx_ctx* ctx, int64_t* p, int64_t* q, int64_t cap, int64_t* count);

/* Devex / steepest-edge pricing weights w_j of every column (n entries; the
 * non-basic ones are the live weights, as updated by the last pricing pass).
 * SPX_ERR_STATE under Dantzig pricing. */
int spx_get_weights(spx_ctx* ctx, double* w);

/* With SPX_FLAG_TIMING: total device milliseconds and launch counts of the
 * pricing kernel and of the fused update kernel since the last call (resets). */
int spx_kernel_times(spx_ctx* ctx, double* price_ms, int64_t* price_launches,
                     double* update_ms, int64_t* update_launches);

/* With SPX_FLAG_TIMING: device milliseconds summed since the last call (resets)
 * of out[0] the pricing kernel, out[1] pricing + the cross-rank MINLOC
 * exchange (RCCL all-gather; == out[0] at one rank), out[2] the update kernel;
 * passes = timed passes. */
int spx_pass_times(spx_ctx* ctx, double out[3], int64_t* passes);

/* With SPX_FLAG_STAMPS: microseconds summed since the last call of, per
 * kernel, the body (earliest workgroup start -> last workgroup's ticket) and
 * the last-workgroup tail (final reduction; for the update kernel also E_q,
 * r, x_b, y and the basis bookkeeping).  out[0..3] = price body, price tail,
 * update body, update tail; out[4..8] = update-tail sub-phases (partials ->
 * q, s_y dot, block sum, bookkeeping, -); out[9..12] = update prologue
 * (earliest workgroup start -> earliest row stream start), update drain
 * (latest stream end -> last ticket), price prologue, price drain;
 * out[13..17] = the update kernel's workgroup 0, from its start to: status
 * read, entering column known, row stream start, its wave 0's stream end,
 * partial published.  Resets.
 * Loop passes that defer the pricing tail (window passes and explicit passes
 * at m <= 2048 on one rank, Params::defer_price) have no pricing ticket, so
 * out[0], out[1], out[11] and out[12] stay 0 for them; the per-workgroup
 * clocks of spx_wg_times cover those passes.  The step-wise API
 * (spx_price / spx_pivot) keeps the pricing tail and fills every slot. */
#define SPX_PHASES 18
int spx_phase_times(spx_ctx* ctx, double out[SPX_PHASES]);

/* With SPX_FLAG_STAMPS: the compact fold's (k_cfold) per-workgroup clocks of
 * its last launch, 8 words per workgroup (up to 1024 workgroups): entry,
 * coefficients staged, R in LDS, tiles done, the y / xw updates done, the
 * arrival counted (s_memrealtime, 100 MHz).  count = words written. */
int spx_fold_times(spx_ctx* ctx, uint64_t* out, int64_t cap, int64_t* count);

/* Diagnostic (SPX_FLAG_STAMPS, compact window passes): the clocks of the
 * last two passes, s_memrealtime ticks (100 MHz), one block per pass parity
 * (iteration & 1, parity 0 first).  A block holds, per workgroup g of that
 * pass's FTRAN launch (k_ftran_bc), 4 ticks at k = 0 entry, 1 entering column
 * known, 2 A_p on the column list in LDS (the p-dependent round trip done),
 * 3 partial published (4 grid values); then per workgroup h of its pricing
 * launch (k_price) 4 ticks: start, end of its column loop, the deferred
 * ratio-test tail reduced, the staging in LDS (4 price grid values); then
 * the tick at which the FTRAN tail had issued the pivot's
 * bookkeeping (1 value), then the tick at which the diagnostic one-wave
 * kernel launched before the FTRAN pass started (SPX_DIAG_MARK=1; 1 value),
 * then the tick k_price's workgroup 0 had issued the deferred tail's
 * bookkeeping (1 value).
 * Copies min(cap, 2 (4 grid + 4 price grid + 3)) values; *count = grid. */
int spx_wg_times(spx_ctx* ctx, uint64_t* out, int64_t cap, int64_t* count);

/* With SPX_FLAG_TIMING and the persistent loop kernel (spx_config out[8]
 * = 1): out[0] device milliseconds of the loop launches (hipEvents) and out[1]
 * the passes they ran, since the last call; out[2..4] microseconds summed
 * over passes of the in-kernel phases seen by workgroup 0 (s_memrealtime):
 * pricing to grid barrier 1, FTRAN + ratio test to barrier 2, tail to the
 * next pass; passes = passes with a phase split; out[5] device milliseconds
 * of the window folds launched between loop launches (hipEvents) and out[6]
 * their count.  Resets. */
#define SPX_LOOP_FIELDS 7
int spx_loop_times(spx_ctx* ctx, double out[SPX_LOOP_FIELDS], int64_t* passes);

/* Geometry and algorithmic bytes.  bytes_price: one pricing launch on this
 * rank (8*(m+1)*local non-basic columns), bytes_update: the B^-1 bytes per
 * pivot — 16*m*m for the explicit rank-1 update, or
 * 8*m*m*(1 + 2/(window-1)) for the eta window (stream + amortised fold). */
int spx_info(spx_ctx* ctx, int64_t* m, int64_t* n, int64_t* ld,
             int64_t* local_nonbasic, double* bytes_price, double* bytes_update);

/* Resolved configuration: out[0] window (0 = explicit B^-1), [1] pricing
 * threads per workgroup, [2] pricing workgroups, [3] pricing LDS mode (0 y
 * in global, 1 y in LDS, 2 y and the window base row in LDS), [4] update
 * threads per workgroup, [5] update rows per wave, [6] update workgroups,
 * [7] passes per captured hipGraph (0 = eager), [8] persistent loop kernel
 * in use (1) or not (0), [9] its threads per workgroup, [10] window tableau
 * (SPX_FLAG_TABLEAU) in use, [11] workgroups of the persistent loop kernel,
 * [12] the ratio-test tail deferred into the next pricing pass (1; compact
 * window passes on one rank, SPX_DEFER_TAIL=0 turns it off) or run by the
 * FTRAN pass's last workgroup (0), [13] the window fold updates only B_w's
 * listed (non-unit) columns (1: k_cfold; SPX_DENSE_FOLD=1 turns it off) or
 * the dense B_w (0), [14] k_ftran_bc rows per wave (0: not in use), [15]
 * (after spx_mbox_attach) loop passes exchange through the mailboxes inside
 * k_price and k_ftran_bc (1: the fused exchange; SPX_MBOX_FUSED=0 turns it
 * off) or with a k_exchange launch per pass (0). */
#define SPX_CONFIG_FIELDS 16
int spx_config(spx_ctx* ctx, int32_t out[SPX_CONFIG_FIELDS]);

/* Columns of B^-1 the FTRAN stream reads per row: m, or with the eta window's
 * compact operand (A[:, n-m:] = I, two-kernel passes; SPX_DENSE_FTRAN=1 turns
 * it off) the non-unit columns of B_w as of the last fold: B_w is I except in
 * the columns of rows whose slack has left the basis. */
int spx_ftran_cols(spx_ctx* ctx, int32_t* cols);

/* What the loop has enqueued since spx_create (monotone counters, so a
 * caller can difference them around a timed region): out[0] passes launched
 * eagerly (step-wise spx_price/spx_pivot included), [1] captured-hipGraph
 * replays, [2] passes inside those replays, [3] persistent loop-kernel
 * launches, [4] passes inside them, [5] eta-window folds (k_fold) enqueued,
 * [6] the window position (pivots since the last fold + 1; a fold is due
 * before the next pass when it equals [7]), [7] the window size KW (0 =
 * explicit B^-1), [8] persistent launches whose grid was found not
 * co-resident (another stream or process held CUs; the context then
 * switched to two-kernel passes and made those pivots that way), [9] batch
 * hipGraphs built (captured, instantiated and uploaded; 0 or 1 per context,
 * rebuilt once after spx_mbox_attach). */
#define SPX_DISPATCH_FIELDS 10
int spx_dispatch_stats(spx_ctx* ctx, int64_t out[SPX_DISPATCH_FIELDS]);

/* Capture, instantiate and upload the batch hipGraph now, so that no later
 * spx_iterate pays for it.  spx_create does this itself on one rank; with a
 * communicator or mailboxes the graph can only be captured once they are
 * attached (spx_attach_comm / spx_mbox_attach), and spx_iterate would
 * otherwise build it on its first call that spans a whole batch.  A no-op
 * when the graph exists, for eager dispatch (graph_batch < 0, timing) and for
 * the persistent loop kernel.  If RCCL refuses the capture the context runs
 * eager passes (spx_comm_info's graph_fallback). */
int spx_prepare(spx_ctx* ctx);

/* Host-only helpers (no device needed), shared with the device code:
 * spx_shard_range: this rank's column shard — structural columns
 *   [out[0], out[1]) and slack columns [out[2], out[3]) (global indices).
 * spx_minloc_merge: the cross-rank MINLOC rule applied to the all-gathered
 *   candidates — smallest value, then smallest global index (CUB ArgMin's
 *   first-index semantics, v4:294). */
int spx_shard_range(int64_t m, int64_t n, int32_t rank, int32_t nranks, int64_t out[4]);
int spx_minloc_merge(const double* vals, const int64_t* idx, int32_t count,
                     double* best_val, int64_t* best_idx);

const char* spx_last_error(void);
const char* spx_status_string(int32_t status);
int spx_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif

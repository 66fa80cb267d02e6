// spx_device.h — device-state layout and kernel parameter block shared by the
// gfx950 kernels (spx_kernels.hip) and the host runtime (spx_api.cpp).
//
// HBM layout (all fp64, L = round_up(m, 128) doubles = whole 1 KiB lines):
//   A      L x n, column-major (column j at A + j*L; rows m..L-1 zero).  The
//          reference's D = [-c; A] copy (v4:248,278-279) is not built: pricing
//          reads A and c directly.
//   B      m x L, ROW-major B^-1 S (the reference is column-major, v4:59-60),
//          updated in place by k_update (SPX_INPLACE=1, default; the ping-pong
//          variant B0/B1 is a build option kept for A/B measurements).
//   rbuf   L: the pending pivot row, staged by k_price (k_update overwrites
//          row q while every wave still needs it).
//
// Deferred pivot state.  The last pivot (it-1) is kept in factored form and
// applied by the kernels that stream the data anyway:
//   true B^-1 = S + E r^T, with r = S[q,:] (row q of S is the new pivot row,
//          bit-identical to B^-1_new[q,:] of v4:331) and E_i = -alpha_i/alpha_q,
//          E_q = 1/alpha_q - 1 (compute_E_q, v4:210-215) from alpha[it&1] and the
//          scalar st->aq — applied by the next k_update stream;
//   y     = ybuf[st->y_buf] + s_y r while st->y_applied < it — applied by the
//          next k_price while it stages y in LDS;
//   x_b  += s_x E with s_x = r.b while st->xb_applied < it — applied by the
//          next k_update to the rows each wave owns.
//   k_flush applies whatever is still pending (readback, end of a solve).
//
//   x_b, c_B, b (L), c (n), alpha[2], ybuf[2] (L), b_ixs (m int64).
//
// Eta window (Params::win = KW > 0).  B^-1 is not rewritten
// every pivot.  With B stored as the window base B_w and pivots tau = 0..nw-1
// since the last fold (nw-1 the pending one, as above):
//   true B^-1 = B_w + sum_tau eta_tau r_tau^T, r_tau = row q_tau of B^-1 before
//          pivot tau, eta_tau the compute_E_q column (v4:210-215) minus e_q;
//   U      m x KW row-major, U[i*KW + tau] = eta_tau[i] (written by k_update
//          one pass after pivot tau, from alpha and aq);
//   Wt     (n+1) x KW, Wt[j*KW + tau] = r_tau . A_j, and Wt[n*KW + tau] =
//          r_tau . b — written by k_price one pass after pivot tau (basic
//          columns get their exact value: aq for the entering column, else 0),
//          so r_tau itself is never formed: r_tau . A_j = B_w[q_tau,:] . A_j +
//          sum_{s<tau} U[q_tau][s] Wt[j][s]; Wt[n*KW + tau] = r_tau . b (the
//          pending x_b update's s_x) comes from xw = B_w b, kept by k_fold;
//   y      = y_w + sum_tau SY[tau] r_tau, so e_j = y_w . A_j + sum SY[tau]
//          Wt[j][tau] - c_j; alpha = B_w A_p + sum U[:,tau] Wt[p][tau];
//   Qrows/Urows  the base rows B_w[q_tau,:] and coefficients U[q_tau][s<tau]
//          (staged by k_price) from which k_fold rebuilds the r_tau.
// Window tableau (tab = 1): with T_w = B_w A and dw = y_w A - c kept in HBM,
//   r_tau . A_j = T_w[q_tau, j] + sum_{s<tau} U[q_tau][s] Wt[j][s],
//   e_j = dw[j] + sum_tau SY[tau] Wt[j][tau],
//   alpha = T_w[:, p] + sum_tau U[:, tau] Wt[p][tau];
// the fold adds T_w += U Wt^T and dw += SY Wt^T (k_tab_fold, fp64 MFMA).
// When nw reaches KW, k_fold folds the nw-1 complete pivots into B_w and y_w
// (rank-(KW-1) update, read + write of B once) and the pending pivot becomes
// tau = 0.
//   nb_list / nb_pos   this rank's non-basic columns (compact list + position,
//          swap-remove / append per pivot) so pricing touches non-basic
//          columns only.
#pragma once
#include <stdint.h>

namespace spx {

enum : int32_t { ST_RUNNING = 0, ST_OPTIMAL = 1, ST_UNBOUNDED = 2, ST_WINDOW_FULL = 16, ST_HANDOFF_TIMEOUT = 17 };

// (value, global index) candidate; the order is value, then smallest index —
// cub::DeviceReduce::ArgMin's first-index semantics (v4:294,324) for every
// reduction tree, every grid and every rank count.
struct alignas(16) ArgMinEntry {
    double val;
    int64_t idx;
};

// Ratio-test partial of one k_update workgroup: its leaving candidate (first
// index on ties) with that row's alpha / c_B / b_ixs, the count of
// alpha_i <= 0, and T = sum of c_B[i] * alpha_i over its rows — everything
// the pivot needs, so the last workgroup's tail is one round trip.
// Pricing partial of one k_price workgroup: its entering candidate and, in the
// eta window, that column's new Wt entry.
struct alignas(16) PricePartial {
    double val;
    int64_t idx;
    double w;
    double pad;
};

struct alignas(16) UpdPartial {
    double theta;
    int64_t idx;
    int64_t nonpos;
    double T;
    double a_w;
    double cb_w;
    int64_t bix_w;
    int64_t pad;
};

// Row-sharded mode: what each rank contributes to the ratio-test all-gather —
// its local leaving candidate plus that row of B^-1_new, so every rank
// receives the pivot row without a host-side broadcast root.  Followed in
// memory by L doubles (the row); entries are rs_stride bytes apart.
struct alignas(16) RsHeader {
    double theta;    // local min ratio (first index on ties)
    int64_t idx;     // its global row, INT64_MAX if none
    int64_t nonpos;  // local count of alpha_i <= 0
    double T;        // sum over own rows of c_B[i] * alpha_i
    double a_w;      // alpha at idx
    double cb_w;     // c_B at idx
    int64_t bix_w;   // b_ixs at idx
    int64_t pad;
};

// sharded last-arrival counters (arrive_last, spx_common.h): per group one
// root line and ARR_SHARDS shard lines of 128 bytes
constexpr int ARR_SHARDS = 8;
constexpr int ARR_STRIDE = 32;  // uint32 per 128-byte line
constexpr int ARR_LINES = 1 + ARR_SHARDS;
constexpr int TICKET_WORDS = 2 * 16 * 32;  // k_price's ticket counters (Params::tk_shards <= 16)
constexpr int DYN1_MIN_COLS = 16;          // WM 1 takes the ticketed tail from this many columns per wave
enum : int { ARR_PRICE = 0, ARR_UPDATE = 1, ARR_FOLD = 2, ARR_GROUPS = 3 };
// tagged ratio-test partial: 7 eight-byte fields as 14 {32-bit half, tag} words
constexpr int UPD_WORDS = 14;
// tagged pricing partial (k_price's own tail): 4 eight-byte fields as 8 words
constexpr int PRICE_WORDS = 8;

// Deferred ratio-test tail (Params::defer_tail): the compact FTRAN pass
// publishes its workgroup partials and this record and ends; the next
// pricing pass reduces the partials in every workgroup (the leaving row q
// its base row needs) and its workgroup 0 applies the bookkeeping; a
// one-workgroup k_apply_tail does it before a fold and at the end of a
// batch.  fresh = 1 from the FTRAN pass that wrote it until k_apply_tail, or
// an FTRAN pass that stops, clears it.
struct alignas(16) TailRec {
    int64_t it;      // iteration of the pivot
    int64_t p;       // entering column
    double e_rep;    // the reduced cost the bookkeeping records (Devex: its key's e)
    double c_p;      // c[p]
    double wp;       // Devex: W[p]
    int32_t cnt;     // nb_count before the pivot
    int32_t kp;      // nb_pos[p] (-1: not on this rank's list)
    int32_t last;    // nb_list[cnt - 1]
    int32_t nw;      // window count before the pivot
    int32_t fresh;
    int32_t pad[3];
};

struct alignas(16) DevState {
    int32_t status;      // ST_*
    int32_t nb_count;    // entries in nb_list
    int64_t iter;        // pivots made
    int64_t limit;       // kernels do nothing once iter >= limit
    int64_t p;           // last entering column
    int64_t q;           // last pivot row (leaving position); -1 before any pivot
    double min_e;        // last entering reduced cost
    double z;            // objective (spx_objective)
    double aq;           // alpha_q of the last pivot
    double s_y;          // c_B_new.E_q + c_p - c_Bq of the last pivot (v4:354-355)
    int64_t y_applied;   // ybuf[y_buf] includes the first y_applied pivots
    int64_t xb_applied;  // x_b includes the first xb_applied pivots
    int32_t y_buf;
    uint32_t pad_t0;     // (the arrival counters live in Params::arrive)
    uint32_t mbox_epoch;  // fused mailbox exchange: the tags' high byte, advanced by every reset
    int32_t nw;          // eta window: pivots since the last fold (nw-1 pending)
    uint32_t uncovered;  // set by k_price: a pass's ticketed list slots were not all taken (never cleared but by a reset)
    int32_t pad1;
    int64_t leave;       // Devex: column that left at the last pivot (-1 none)
    double wp;           // Devex: weight of the last entering column
    double pad3;
};

__host__ __device__ inline bool argmin_better(double v, int64_t j, double bv, int64_t bj) {
    return (v < bv) || (v == bv && j < bj);
}

// SPX_FLAG_STAMPS layout past the 32 phase words, by pass parity (it & 1):
// k_ftran_bc 4 ticks per workgroup, k_price 4 per workgroup, and the compact
// FTRAN tail's end
constexpr int64_t STAMP_FTRAN = 32;
constexpr int64_t STAMP_PRICE = STAMP_FTRAN + 2 * 4 * 4096;
constexpr int64_t STAMP_TAIL = STAMP_PRICE + 2 * 4 * 4096;
// the compact fold's per-workgroup clocks (k_cfold, up to 1024 workgroups):
// entry, coefficients staged, R in LDS, tiles done, vectors done, arrived
constexpr int64_t STAMP_FOLD = STAMP_TAIL + 8;
constexpr int STAMP_FOLD_PER = 8;
constexpr int64_t STAMP_WORDS = STAMP_FOLD + STAMP_FOLD_PER * 1024;

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
    double* alpha0;
    double* alpha1;
    double* y0;
    double* y1;
    double* x_b;
    double* c_B;
    const double* zeros;   // L zeros (the "pivot row" before the first pivot)
    double* rbuf;          // staged pivot row (in-place B^-1 storage)
    int64_t* b_ixs;
    int32_t* nb_list;
    int32_t* nb_pos;       // n entries, -1 when basic or not owned
    // column shard of this rank: structural [s_lo, s_hi), slack [k_lo, k_hi)
    int64_t s_lo, s_hi, k_lo, k_hi;
    // reductions
    PricePartial* price_partials;
    ArgMinEntry* price_out;        // this rank's entering candidate record
    const ArgMinEntry* price_in;   // all ranks' records (== price_out at 1 rank)
    int32_t nin;
    int32_t pr_stride;             // ArgMinEntry slots per record: 1, or 1 + KW/2
                                   // (the window appends Wt[p][0..KW) to the head)
    double* upd_soa;               // k_update partials, field-major (upd_publish)
    int64_t upd_cap;               // workgroup slots per field
    // k_update partials as tagged words (UPD_WORDS per slot, field-major),
    // polled by the last workgroup instead of a drain + last-arrival count;
    // nullptr: the counted hand-off (upd_soa + arrive)
    uint64_t* upd_tag;
    // k_price partials as tagged words (PRICE_WORDS per slot, field-major) for
    // the pricing tail k_price itself runs (multi-rank, stepping API);
    // nullptr: the counted hand-off (price_partials + arrive)
    uint64_t* price_tag;
    int64_t price_cap;
    DevState* st;
    // row-sharded B^-1 (nranks > 1 with SPX_FLAG_ROW_SHARD): this rank owns
    // global rows [r0, r0 + mloc) of B^-1, stored as B0/B1 (mloc x L ping-pong)
    int32_t row_shard;
    int32_t split_tail;            // 1: the pivot tail runs as its own launch (k_tail)
    int64_t r0, mloc;
    unsigned char* rs_send;        // RsHeader + row
    const unsigned char* rs_recv;  // nin entries of rs_stride bytes
    int64_t rs_stride;
    // diagnostics (SPX_FLAG_STAMPS): per kernel {min WG start, sum body, sum tail}
    // in s_memrealtime ticks (100 MHz) in the first 32 words, then per-pass
    // clocks double-buffered by the pass parity (STAMP_*); nullptr in normal runs
    unsigned long long* stamps;
    // k_price's dynamic tail (SPX_PRICE_DYN): column-ticket counters, 16 per
    // pass parity, each on its own 128-byte line (uint32 [2][16][32])
    uint32_t* tickets;
    int32_t price_dyn;  // 1: k_price hands out its last columns by ticket (SPX_PRICE_DYN=0: off)
    int32_t tk_shards;  // ticket counters per pass parity (1..16)
    // eta window (see above); win = KW, 0 = explicit B^-1 updated every pivot
    int32_t win;
    int32_t pad_w;
    double* U;
    double* Wt;
    double* Qrows;  // KW x L
    double* Urows;  // KW x KW
    double* SY;     // KW
    double* xw;     // B_w b (L): r_tau . b = xw[q_tau] + sum_{s<tau} U[q_tau][s] Wt[n][s]
    // leaving-row rule (include/simplex.h SPX_RATIO_*): candidates alpha_i >
    // piv_tol (0 for the reference rule); GUARDED/HARRIS clamp x_b_i at 0
    int32_t ratio;
    int32_t devex;         // SPX_PRICING_DEVEX (eta window, one rank)
    double piv_tol;
    double feas_tol;
    double* W;             // Devex / steepest-edge reference weights (n)
    double* dvx_e;         // Devex: reduced cost of the chosen column (k_price -> k_update)
    // steepest edge (SPX_PRICING_STEEPEST: devex = 1 as well, so the key,
    // optimality test and reduced-cost plumbing are Devex's): exact weights
    // gamma_j = 1 + ||B^-1 A_j||^2 kept by the Goldfarb-Reid recurrence.  For
    // the pending pivot (alpha = its FTRAN column, B^-1 before it):
    // se_v = B_w^T alpha (L), se_cg[s] = U[:, s] . alpha for s < tau and
    // se_cg[KW] = gamma_p = 1 + ||alpha||^2 (k_se_part / k_se_fin before each
    // pricing pass), so that A_j . B^-T alpha = se_v . A_j + sum_s se_cg[s] Wt[j][s]
    int32_t steep;
    int32_t se_parts;      // k_se_part workgroups (row blocks)
    double* se_v;
    double* se_cg;
    double* se_part;       // se_parts x se_ncols partial sums
    // deferred pricing tail (one rank, captured/eager passes): k_price stores
    // its workgroup partials and returns; every k_update workgroup reduces the
    // price_grid partials itself (no last-workgroup fan-in, no ticket)
    int32_t defer_price;
    int32_t price_grid;
    // deferred ratio-test tail (TailRec above; one rank, compact window
    // passes): tail_parts = the FTRAN pass's workgroups
    int32_t defer_tail;
    int32_t tail_parts;
    TailRec* trec;
    // window tableau (SPX_FLAG_TABLEAU): T_w = B_w A (L x n,
    // column-major like A) and dw = y_w A - c (n), both folded with B_w, so a
    // pass reads T_w[q_tau, j], dw[j] and Wt[j][.] per column instead of A_j,
    // and FTRAN reads the column T_w[:, p] instead of streaming B_w
    int32_t tab;
    // A[:, n-m:] = I (checked at create): then B_w is T_w's slack block
    // (B_w e_i = T_w[:, n-m+i]), so the tableau folds T_w, dw, y_w and xw
    // only and skips k_fold; readbacks rebuild B_w from T_w (k_tab_binv)
    int32_t tab_slack;
    double* T;
    double* dw;
    // the fold's active columns (k_tab_active): those whose Wt row has a
    // nonzero entry among the nf folded pivots; for every other column the
    // fold adds U 0 = 0, so k_tab_fold walks this list instead of all n
    int32_t* tab_list;  // n
    int32_t* tab_cnt;   // 1
    // pivot trace (spx_opts.trace_cap): trace[2 it] = p, trace[2 it + 1] = q
    // for pivot it < trace_cap, written where the pivot is committed
    int64_t* trace;
    int64_t trace_cap;
    // sharded last-arrival counters (spx_common.h arrive_last), ARR_GROUPS
    // groups of ARR_LINES 128-byte lines
    uint32_t* arrive;
    // peer mailboxes (spx_mbox_attach): the MINLOC exchange as direct stores
    // into every rank's mailbox (k_exchange) instead of an RCCL all-gather.
    // Mailbox words: [2 parities][nin ranks][pr_stride * 4 halves], each
    // (seq << 32) | 32-bit half of the record; mbox_peer[g] is rank g's
    // mailbox as mapped here (IPC), mbox this rank's own, mbox_seq the
    // exchange counter (every rank runs the same exchanges)
    uint64_t* const* mbox_peer;
    uint64_t* mbox;
    uint32_t* mbox_seq;
    int32_t mbox_rank;
    // fused exchange (loop passes of a compact window, set per launch by
    // enqueue_pass): k_price's pricing tail stores the record into every
    // rank's mailbox itself and k_ftran_bc polls its own -- no k_exchange
    // launch.  Tags: (mbox_epoch << 24) | (iteration + 1), parity iteration & 1
    int32_t mbox_fused;
    // A[:, ns:] = I exactly (checked at create; SPX_DENSE_SLACKS=1 turns it
    // off): k_price prices a non-basic slack column without streaming it
    int32_t slack_unit;
    int32_t bc_lds;  // k_loop: doubles of A_p on the column list its LDS holds
    // B_w by its non-unit columns (eta window, two-kernel passes; DESIGN.md
    // §4a "compact FTRAN").  With A[:, ns:] = I, column k of B_w is e_k while
    // slack k has stayed basic in row k, so B_w = I + (columns rlist[0..S)).
    // bc: m rows at pitch bc_n[1] (S rounded up to 64; the allocation is m x
    // L), row i's first S entries = B_w[i][rlist[c]] (gathered after
    // every fold from the dense B_w, which stays the master copy); rmap[k] =
    // c or -1 (unit column); rleft[k] = 1 once row k has been a leaving row
    // (or, after a reinversion, when slack k is not basic in row k): a
    // superset of the non-unit columns; bc_n[0] = S, bc_n[1] = the row pitch.
    // nullptr: dense FTRAN.
    // Two buffers of that shape: bc_n[2] selects the active one (bc or bc1).
    // The compact fold (k_cfold) reads the active buffer at the old pitch,
    // writes the folded rows at the new pitch into the other one, scatters
    // the same values into the dense B_w and flips bc_n[2]; bc_n[3] / bc_n[4]
    // hold S and the pitch before k_bc_list appended the window's rows.
    double* bc;
    double* bc1;
    int32_t cfold;  // the fold updates the listed columns only (k_cfold; SPX_DENSE_FOLD=1: k_fold + gather)
    // steepest edge, set per launch: k_ftran_bc stores its workgroup's
    // partial sums of M^T alpha (k_se_part's, over its 8 rows) into se_part,
    // so the next pass's k_se_fin can skip k_se_part (spx_api.cpp se_chain)
    int32_t se_fused;
    int32_t* rlist;
    int32_t* rmap;
    int32_t* rleft;
    int32_t* bc_n;
};

// the compact operand's active buffer (bc_n[2])
__host__ __device__ inline double* bc_buf(const Params& P, int sel) { return sel ? P.bc1 : P.bc; }
constexpr int BC_N_WORDS = 8;

__device__ __forceinline__ void record_pivot(const Params& P, int64_t it, int64_t p, int64_t q) {
    if (P.trace && it < P.trace_cap) {
        P.trace[2 * it] = p;
        P.trace[2 * it + 1] = q;
    }
}

// Optimality test on the merged entering candidate (v4:299-302): the reduced
// cost itself under Dantzig; under Devex the key -e^2/w is +inf exactly when
// no e_j < -eps.
__host__ __device__ inline bool no_entering(const Params& P, double val, int64_t p) {
    return p == INT64_MAX || (P.devex ? !(val < INFINITY) : val >= -P.eps);
}

enum : int32_t { RATIO_REFERENCE = 0, RATIO_GUARDED = 1, RATIO_HARRIS = 2 };

// Ratio-test key of one row (compute_theta, v4:199-208, and the SPX_RATIO_*
// variants); INFINITY when the row is not a candidate.  HARRIS returns the
// first-pass key (max(x_b,0) + feas_tol) / alpha.
__host__ __device__ inline double ratio_key(const Params& P, double xb, double a) {
    if (!(a > P.piv_tol)) return INFINITY;
    if (P.ratio == RATIO_REFERENCE) return xb / a;
    const double xc = xb > 0.0 ? xb : 0.0;
    return P.ratio == RATIO_HARRIS ? (xc + P.feas_tol) / a : xc / a;
}

__host__ __device__ inline bool owns_col(const Params& P, int64_t j) {
    return (j < P.ns) ? (j >= P.s_lo && j < P.s_hi) : (j >= P.k_lo && j < P.k_hi);
}

}  // namespace spx

// spx_api.cpp — host runtime behind include/simplex.h.
//
// Replaces the reference's solve() (src/v4_cub_reduction.cu:219-380): device
// allocation, upload, slack-basis init, the iteration loop and readback.  The
// loop differs in shape, not in meaning: the reference blocks on 4 D2H reads
// per pass (v4:295,296,317,325) and issues ~20 cuBLAS/CUB/kernel calls; here a
// pass is two kernels, termination is a device-side status word, and batches
// of passes are replayed from one captured hipGraph with a single
// synchronisation per batch.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/simplex.h"
#include "spx_device.h"
#include "spx_kernels.h"
#include "spx_reinv.h"
#include "spx_tableau.h"
#include "spx_loop.h"

using namespace spx;

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIP_TRY(expr)                                                                          \
    do {                                                                                       \
        hipError_t e_ = (expr);                                                                \
        if (e_ != hipSuccess)                                                                  \
            return fail(e_ == hipErrorOutOfMemory ? SPX_ERR_OOM : SPX_ERR_HIP, "%s: %s (%s:%d)", \
                        #expr, hipGetErrorString(e_), __FILE__, __LINE__);                    \
    } while (0)

#define NCCL_TRY(expr)                                                                                  \
    do {                                                                                                \
        ncclResult_t r_ = (expr);                                                                       \
        if (r_ != ncclSuccess)                                                                          \
            return fail(SPX_ERR_RCCL, "%s: %s (%s:%d)", #expr, ncclGetErrorString(r_), __FILE__, __LINE__); \
    } while (0)

#define SPX_TRY(expr)          \
    do {                       \
        int rc_ = (expr);      \
        if (rc_ != SPX_OK) return rc_; \
    } while (0)

int64_t round_up(int64_t v, int64_t a) { return (v + a - 1) / a * a; }

// Structural columns [0, ns) and slack columns [ns, n) are each cut into
// nranks contiguous blocks, so the initial slack basis is spread evenly.
void shard_range(int64_t m, int64_t n, int r, int G, int64_t out[4]) {
    const int64_t ns = n - m;
    const int64_t sb = (ns + G - 1) / G, kb = (m + G - 1) / G;
    out[0] = std::min<int64_t>(ns, (int64_t)r * sb);
    out[1] = std::min<int64_t>(ns, (int64_t)(r + 1) * sb);
    out[2] = ns + std::min<int64_t>(m, (int64_t)r * kb);
    out[3] = ns + std::min<int64_t>(m, (int64_t)(r + 1) * kb);
}

}  // namespace

struct spx_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    int cus = 256;
    int64_t m = 0, n = 0, L = 0, ns = 0;
    spx_opts opts{};
    Params P{};
    PriceCfg pcfg{};
    UpdateCfg ucfg{};
    int64_t max_local_cols = 0;

    // device allocations
    std::vector<void*> allocs;
    double* A = nullptr;
    double* b = nullptr;
    double* c = nullptr;
    ArgMinEntry* send = nullptr;
    ArgMinEntry* recv = nullptr;

    // pinned host mirrors
    DevState* st_host = nullptr;
    int64_t* limit_host = nullptr;

    // multi-rank
    ncclComm_t comm = nullptr;
    bool comm_ready = false;
    bool use_comm = false;  // MINLOC through RCCL: nranks > 1, or SPX_FLAG_COMM1 (one-rank test of that path)
    bool graph_fallback = false;  // a capture with RCCL calls failed: eager passes
    // peer mailboxes (spx_mbox_export / spx_mbox_attach): MINLOC by k_exchange
    uint64_t* mbox = nullptr;
    uint32_t* mbox_seq = nullptr;
    uint64_t** mbox_peer = nullptr;  // device array of nranks mailbox pointers
    std::vector<void*> mbox_opened;  // IPC mappings of the other ranks' mailboxes
    bool mbox_ready = false;
    bool mbox_fused = false;  // loop passes exchange inside k_price / k_ftran_bc (Params::mbox_fused)
    bool bc_want = false;      // compact FTRAN operand wanted (allocated by set_slack_flags)
    bool slack_ident = false;  // A[:, n-m:] = I (checked before setup_common)
    bool defer_ok = false;        // loop passes defer the pricing tail into k_update (Params::defer_price)
    bool defer_tail = false;      // loop passes defer the ratio-test tail into k_price (Params::defer_tail)
    // steepest edge: k_ftran_bc stores k_se_part's sums (Params::se_fused) when
    // se_fuse is set; se_chain = the last pass enqueued did, and nothing since
    // changed B_w, U or alpha, so the next pass's k_se_fin reads them
    bool se_fuse = false;
    bool se_chain = false;
    int64_t se_rows = 0;

    // graph replay of `batch` passes
    hipGraphExec_t graph_exec = nullptr;
    hipGraph_t graph = nullptr;
    int batch = 0;

    // in-process group exchange
    hipEvent_t ev_sent = nullptr, ev_recv = nullptr, ev_sent2 = nullptr, ev_recv2 = nullptr;
    // row-sharded B^-1
    int64_t mb = 0;
    unsigned char* rs_recv = nullptr;

    // per-kernel timing
    bool timing = false;
    std::vector<hipEvent_t> ev_price, ev_update;  // pairs (start, stop)
    std::vector<hipEvent_t> ev_xend;              // after the MINLOC exchange
    size_t n_price = 0, n_update = 0;

    int64_t pivots = 0;
    int32_t status = SPX_STATUS_MAX_ITER;
    bool stepped_price = false;
    int nw = 0;  // eta window: device st->nw as of the last readback, advanced per enqueued pass
    // what the loop actually enqueued (spx_dispatch_stats)
    int64_t n_eager = 0, n_graph_launch = 0, n_graph_pass = 0, n_persist_launch = 0, n_persist_pass = 0;
    int64_t n_persist_fallback = 0;  // persistent launches found not co-resident
    int64_t n_folds = 0;
    int64_t n_graph_builds = 0;  // batch graphs captured + instantiated + uploaded
    int graph_folds = 0;     // folds inside one captured batch
    bool capturing = false;  // build_graph: passes are recorded, not run

    // persistent loop kernel (spx_loop.h): window mode, one rank
    LoopCfg lcfg{};
    LoopArgs la{};
    bool persist = false;
    double loop_clock[3] = {0.0, 0.0, 0.0};  // timing: phase A / B / C microseconds (in-kernel clock)
    int64_t loop_clock_passes = 0;
    uint32_t loop_epoch = 0;  // persistent launches so far (LoopArgs::epoch)
    std::vector<hipEvent_t> ev_loop;
    std::vector<int32_t> ev_loop_passes;
    size_t n_loop = 0;
    std::vector<hipEvent_t> ev_fold;  // timing: the window folds between loop launches
    size_t n_fold = 0;

    // basis reinversion (spx_reinv.h): work buffers allocated on first use
    RvParams rv{};
    double* rv_Pa = nullptr;
    double* rv_Pb = nullptr;
    double* rv_Ypart = nullptr;
    int64_t* rv_cols = nullptr;
    int64_t* rv_pos = nullptr;
    int64_t refactor_base = 0;  // pivots at the last reinversion (opts.refactor_every)
    bool broken = false;        // a failed spx_set_basis left no valid basis

    template <typename T>
    int alloc(T** p, size_t count, unsigned ext_flags = ~0u) {
        void* d = nullptr;
        size_t bytes = std::max<size_t>(count, 1) * sizeof(T);
        hipError_t e = ext_flags == ~0u ? hipMalloc(&d, bytes) : hipExtMallocWithFlags(&d, bytes, ext_flags);
        if (e != hipSuccess) return fail(SPX_ERR_OOM, "hipMalloc(%zu bytes) failed: %s", bytes, hipGetErrorString(e));
        allocs.push_back(d);
        e = hipMemsetAsync(d, 0, bytes, stream);
        if (e != hipSuccess) return fail(SPX_ERR_HIP, "hipMemsetAsync failed: %s", hipGetErrorString(e));
        *p = static_cast<T*>(d);
        return SPX_OK;
    }
};

extern "C" {

void spx_default_opts(spx_opts* o) {
    if (!o) return;
    std::memset(o, 0, sizeof(*o));
    o->eps = 1e-7;
    o->device = -1;
    o->rank = 0;
    o->nranks = 1;
    o->graph_batch = 0;
    o->ratio_test = SPX_RATIO_REFERENCE;
    o->refactor_every = 0;
    o->piv_tol = 1e-9;
    o->feas_tol = 1e-9;
    o->pricing = SPX_PRICING_DANTZIG;
}

const char* spx_last_error(void) { return g_err.c_str(); }

int spx_abi_version(void) { return SPX_ABI_VERSION; }

const char* spx_status_string(int32_t s) {
    switch (s) {
        case SPX_STATUS_MAX_ITER: return "MAX_ITER exceeded.";
        case SPX_STATUS_OPTIMUM_FOUND: return "Optimum found";
        case SPX_STATUS_UNBOUNDED: return "Problem unbounded.";
        case SPX_STATUS_THETA_OVERFLOW: return "Theta overflow.";
    }
    return "unknown";
}

}  // extern "C"

namespace {

int reset_stamps(spx_ctx* x);

bool env_on(const char* name);
bool env_off(const char* name);
// the compact FTRAN operand applies: eta window (no tableau, replicated
// storage) and A[:, n-m:] = I (x->slack_ident, known before setup)
bool bc_possible(const spx_ctx* x, const Params& P) {
    return P.win && !P.tab && !P.row_shard && x->slack_ident && !env_on("SPX_DENSE_FTRAN");
}

int setup_common(spx_ctx* x, int64_t m, int64_t n, const spx_opts* opts) {
    if (opts) x->opts = *opts; else spx_default_opts(&x->opts);
    if (x->opts.nranks < 1 || x->opts.rank < 0 || x->opts.rank >= x->opts.nranks)
        return fail(SPX_ERR_ARG, "bad rank %d / nranks %d", x->opts.rank, x->opts.nranks);
    if (!(x->opts.eps >= 0.0)) return fail(SPX_ERR_ARG, "eps must be >= 0");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(SPX_ERR_NO_DEVICE, "no HIP device visible");
    if (x->opts.device >= 0) {
        if (x->opts.device >= ndev) return fail(SPX_ERR_ARG, "device %d out of range (%d)", x->opts.device, ndev);
        HIP_TRY(hipSetDevice(x->opts.device));
    }
    HIP_TRY(hipGetDevice(&x->device));
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, x->device));
    x->cus = prop.multiProcessorCount;
    HIP_TRY(hipStreamCreateWithFlags(&x->stream, hipStreamNonBlocking));
    HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&x->st_host), sizeof(DevState), hipHostMallocDefault));
    HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&x->limit_host), sizeof(int64_t), hipHostMallocDefault));
    std::memset(x->st_host, 0, sizeof(DevState));

    x->m = m;
    x->n = n;
    x->ns = n - m;
    x->L = round_up(m, 128);
    x->timing = (x->opts.flags & SPX_FLAG_TIMING) != 0;
    const int64_t L = x->L;
    const int G = x->opts.nranks, r = x->opts.rank;

    {
        // experiment (SPX_A_MEM): memory type of A — 0 default, 1 uncached, 2 fine-grained
        const char* ev = std::getenv("SPX_A_MEM");
        const int am = ev ? std::atoi(ev) : 0;
        const unsigned fl = am == 1 ? hipDeviceMallocUncached : (am == 2 ? hipDeviceMallocFinegrained : ~0u);
        SPX_TRY(x->alloc(&x->A, (size_t)(L * n), fl));
    }
    SPX_TRY(x->alloc(&x->b, (size_t)L));
    SPX_TRY(x->alloc(&x->c, (size_t)n));

    Params& P = x->P;
    P.A = x->A;
    P.b = x->b;
    P.c = x->c;
    P.m = m;
    P.n = n;
    P.L = L;
    P.ns = x->ns;
    P.eps = x->opts.eps;
    // row shard of B^-1 (SPX_FLAG_ROW_SHARD with nranks > 1): rows
    // [r0, r0 + mloc), ping-pong storage; otherwise all rows, in place
    // (SPX_FLAG_COMM1: the row-sharded RCCL path with one rank, for tests)
    P.row_shard = ((G > 1 || (x->opts.flags & SPX_FLAG_COMM1)) && (x->opts.flags & SPX_FLAG_ROW_SHARD)) ? 1 : 0;
    // leaving-row rule (SPX_RATIO_*); Harris runs its second pass in k_tail
    const int rule = x->opts.ratio_test;
    if (rule != SPX_RATIO_REFERENCE && rule != SPX_RATIO_GUARDED && rule != SPX_RATIO_HARRIS)
        return fail(SPX_ERR_ARG, "bad ratio_test %d", rule);
    if (rule != SPX_RATIO_REFERENCE && !(x->opts.piv_tol >= 0.0)) return fail(SPX_ERR_ARG, "piv_tol must be >= 0");
    if (rule == SPX_RATIO_HARRIS && !(x->opts.feas_tol >= 0.0)) return fail(SPX_ERR_ARG, "feas_tol must be >= 0");
    if (rule == SPX_RATIO_HARRIS && G > 1 && (x->opts.flags & SPX_FLAG_ROW_SHARD))
        return fail(SPX_ERR_ARG, "the Harris ratio test needs replicated B^-1 (no row sharding)");
    if (x->opts.refactor_every < 0) return fail(SPX_ERR_ARG, "refactor_every must be >= 0");
    P.ratio = rule;
    P.piv_tol = rule == SPX_RATIO_REFERENCE ? 0.0 : x->opts.piv_tol;
    P.feas_tol = rule == SPX_RATIO_HARRIS ? x->opts.feas_tol : 0.0;
    P.split_tail = ((x->opts.flags & SPX_FLAG_SPLIT_TAIL) || rule == SPX_RATIO_HARRIS) ? 1 : 0;
    x->mb = P.row_shard ? (m + G - 1) / G : m;
    P.r0 = P.row_shard ? std::min<int64_t>(m, (int64_t)r * x->mb) : 0;
    P.mloc = P.row_shard ? std::min<int64_t>(m, P.r0 + x->mb) - P.r0 : m;
    if (P.row_shard && P.mloc <= 0) return fail(SPX_ERR_ARG, "row sharding needs m >= nranks rows per rank");
    SPX_TRY(x->alloc(&P.B0, (size_t)(std::max<int64_t>(P.mloc, 1) * L)));
    if (kernels_inplace() && !P.row_shard)
        P.B1 = P.B0;
    else
        SPX_TRY(x->alloc(&P.B1, (size_t)(std::max<int64_t>(P.mloc, 1) * L)));
    SPX_TRY(x->alloc(&P.rbuf, (size_t)L));
    SPX_TRY(x->alloc(&P.alpha0, (size_t)L));
    SPX_TRY(x->alloc(&P.alpha1, (size_t)L));
    SPX_TRY(x->alloc(&P.y0, (size_t)L));
    SPX_TRY(x->alloc(&P.y1, (size_t)L));
    SPX_TRY(x->alloc(&P.x_b, (size_t)std::max<int64_t>(L, (int64_t)G * x->mb)));  // G*mb: in-place all-gather
    SPX_TRY(x->alloc(&P.c_B, (size_t)L));
    double* zeros = nullptr;
    SPX_TRY(x->alloc(&zeros, (size_t)L));
    P.zeros = zeros;
    SPX_TRY(x->alloc(&P.b_ixs, (size_t)m));
    SPX_TRY(x->alloc(&P.nb_list, (size_t)n));
    SPX_TRY(x->alloc(&P.nb_pos, (size_t)n));
    SPX_TRY(x->alloc(&P.st, 1));
    SPX_TRY(x->alloc(&P.arrive, (size_t)(ARR_GROUPS * ARR_LINES * ARR_STRIDE)));
    SPX_TRY(x->alloc(&P.tickets, (size_t)TICKET_WORDS));
    P.price_dyn = env_off("SPX_PRICE_DYN") ? 0 : 1;
    if (x->opts.trace_cap < 0) return fail(SPX_ERR_ARG, "trace_cap must be >= 0");
    if (x->opts.trace_cap > 0) {
        P.trace_cap = x->opts.trace_cap;
        SPX_TRY(x->alloc(&P.trace, (size_t)(2 * P.trace_cap)));
    }

    // B^-1 representation: eta window of KW pivots, or the explicit rank-1 update
    int KW = x->opts.window;
    if (KW == 0) {
        // auto (measured): the window halves the B^-1 stream and
        // costs ~2 % more pricing (its Wt rows): C3 +27 %, C4 +4 %, C5 +33 %
        // against the explicit update; C2 (m = 1024, latency-bound: 45.8k vs
        // 52.1k it/s) stays explicit.  Row-sharded B^-1 is always explicit.
        const bool pays = m >= 2048;
        KW = (pays && !P.row_shard) ? 64 : -1;
    }
    // Devex pricing takes the pivot row from the eta-window pricing pass
    if (x->opts.pricing != SPX_PRICING_DANTZIG && x->opts.pricing != SPX_PRICING_DEVEX &&
        x->opts.pricing != SPX_PRICING_STEEPEST)
        return fail(SPX_ERR_ARG, "bad pricing %d", x->opts.pricing);
    // steepest edge rides on Devex's plumbing (key -e^2/w, reduced-cost hand-off)
    P.steep = x->opts.pricing == SPX_PRICING_STEEPEST ? 1 : 0;
    P.devex = (x->opts.pricing == SPX_PRICING_DEVEX || P.steep) ? 1 : 0;
    if (P.devex) {
        const char* rule = P.steep ? "steepest-edge" : "Devex";
        if (G > 1 && P.split_tail) return fail(SPX_ERR_ARG, "%s pricing on a group needs the in-pass ratio-test tail (no split tail, no Harris)", rule);
        if (G > 1 && (x->opts.flags & SPX_FLAG_ROW_SHARD)) return fail(SPX_ERR_ARG, "%s pricing needs replicated B^-1 (no row sharding)", rule);
        if (x->opts.window < 0) return fail(SPX_ERR_ARG, "%s pricing needs the eta window (window > 0 or 0 = auto)", rule);
        if (P.steep && (x->opts.flags & SPX_FLAG_TABLEAU)) return fail(SPX_ERR_ARG, "steepest-edge pricing runs without the tableau");
        if (x->opts.window == 0) KW = 64;
        SPX_TRY(x->alloc(&P.W, (size_t)n));
        SPX_TRY(x->alloc(&P.dvx_e, 1));
    }
    // window tableau: T_w = B_w A and dw = y_w A - c beside the eta window
    P.tab = (x->opts.flags & SPX_FLAG_TABLEAU) ? 1 : 0;
    if (P.tab) {
        if (G > 1 || P.row_shard || (x->opts.flags & SPX_FLAG_COMM1))
            return fail(SPX_ERR_ARG, "the window tableau runs on one rank");
        if (x->opts.window < 0) return fail(SPX_ERR_ARG, "the window tableau needs the eta window (window > 0 or 0 = auto)");
        if (x->opts.window == 0) KW = 64;
    }
    if (KW > 0 && P.row_shard) return fail(SPX_ERR_ARG, "the eta window needs replicated B^-1 (no row sharding)");
    if (KW > 0 && !(KW == 8 || KW == 16 || KW == 32 || KW == 64))
        return fail(SPX_ERR_ARG, "window must be 8, 16, 32 or 64 (got %d)", KW);
    if (KW < -1) return fail(SPX_ERR_ARG, "bad window %d", KW);
    P.win = KW > 0 ? KW : 0;
    if (P.steep) {  // B_w^T alpha (L), U^T alpha + gamma_p (KW + 1), row-block partials
        P.se_parts = se_parts_for(m);
        // rows: k_se_part's blocks, or one per k_ftran_bc workgroup (8 rows each, se_fused)
        x->se_rows = std::max<int64_t>(P.se_parts, (m + 7) / 8);
        SPX_TRY(x->alloc(&P.se_v, (size_t)L));
        SPX_TRY(x->alloc(&P.se_cg, (size_t)(KW + 1)));
        SPX_TRY(x->alloc(&P.se_part, (size_t)x->se_rows * (size_t)(L + KW + 1)));
    }
    if (P.win) {
        SPX_TRY(x->alloc(&P.U, (size_t)(m * KW)));
        SPX_TRY(x->alloc(&P.Wt, (size_t)((n + 1) * KW)));
        SPX_TRY(x->alloc(&P.Qrows, (size_t)(KW * L)));
        SPX_TRY(x->alloc(&P.Urows, (size_t)(KW * KW)));
        SPX_TRY(x->alloc(&P.SY, (size_t)KW));
        SPX_TRY(x->alloc(&P.xw, (size_t)L));
    }
    if (P.tab) {
        SPX_TRY(x->alloc(&P.T, (size_t)(L * n)));
        SPX_TRY(x->alloc(&P.dw, (size_t)n));
        SPX_TRY(x->alloc(&P.tab_list, (size_t)n));
        SPX_TRY(x->alloc(&P.tab_cnt, (size_t)1));
    }
    // the candidate record: {key, column}, then (eta window) the winner's KW
    // window coefficients, then (Devex / steepest edge) its reduced cost and
    // weight (dvx_payload)
    P.pr_stride = P.win ? 1 + P.win / 2 + (P.devex ? 1 : 0) : 1;

    // column shard: structural and slack columns each split in G contiguous blocks
    int64_t rng[4];
    shard_range(m, n, r, G, rng);
    P.s_lo = rng[0];
    P.s_hi = rng[1];
    P.k_lo = rng[2];
    P.k_hi = rng[3];
    x->max_local_cols = (P.s_hi - P.s_lo) + (P.k_hi - P.k_lo);

    // pricing geometry: y in LDS when it fits, 16 waves per CU either way
    PriceCfg& pc = x->pcfg;
    const size_t ybytes = (size_t)L * 8;
    if (x->opts.price_block == 256 || x->opts.price_block == 512 || x->opts.price_block == 1024)
        pc.block = x->opts.price_block;
    else
        // 8 waves per CU either way: with y (and the base row) taking most of
        // LDS there is one workgroup per CU, and a 1024-thread workgroup would
        // cap k_price at 128 VGPRs and spill (C5: 1,158 vs 977 us per pass)
        pc.block = 512;
    const size_t red_bytes = (size_t)(pc.block / 64) * sizeof(PricePartial) + 16;
    const size_t lds_cap = 150 * 1024;
    pc.lds_y = ybytes + red_bytes <= lds_cap && !(x->opts.flags & SPX_FLAG_GLOBAL_Y) && !P.tab;
    // eta window: the pending base row next to y when both fit; the tableau
    // pass stages nothing (wm 3)
    pc.wm = P.tab ? 3 : (!P.win ? 0 : ((pc.lds_y && 2 * ybytes + red_bytes <= lds_cap) ? 1 : 2));
    if (pc.wm == 1 && env_on("SPX_PRICE_RGLOBAL")) pc.wm = 2;  // A/B: base row from L2 though it fits
    // steepest edge: B_w^T alpha beside y and the base row when all three fit
    if (P.steep) pc.wm = (pc.lds_y && 3 * ybytes + red_bytes <= lds_cap) ? 4 : 5;
    pc.lds_bytes = (pc.lds_y ? ybytes : 0) + ((pc.wm == 1 || pc.wm == 4) ? ybytes : 0) + (pc.wm == 4 ? ybytes : 0) +
                   red_bytes;
    int per_cu = 0;
    HIP_TRY(price_prepare(pc, &per_cu));
    if (per_cu < 1) per_cu = 1;
    const int waves = pc.block / 64;
    int64_t want = (x->max_local_cols + waves - 1) / waves;
    int64_t cap = (int64_t)x->cus * per_cu;
    pc.grid = (int)std::max<int64_t>(1, std::min(want, cap));
    // small problems (C2): under 2 columns per wave the per-workgroup y staging
    // and fan-in dominate — one workgroup per CU (measured 13.0 -> 10.4 us)
    if (x->max_local_cols < 2LL * pc.grid * waves)
        pc.grid = (int)std::max<int64_t>(1, std::min<int64_t>(pc.grid, std::max<int64_t>(x->cus,
                                                                   x->max_local_cols / (2 * waves))));
    // window tableau: a column is a few short loads (no stream); each wave
    // keeps 4 columns in flight (k_price WM 3), so one pass over the list
    if (P.tab) pc.grid = (int)std::max<int64_t>(1, std::min(cap, (x->max_local_cols + 4 * waves - 1) / (4 * waves)));
    if (x->opts.price_grid > 0) pc.grid = x->opts.price_grid;
    // the ticketed pricing tail (k_price, Params::price_dyn): with the base row
    // read from L2 (WM 2, C5) always; with it in LDS (WM 1) only where a wave
    // prices many columns (C4: 62; C3: 6, where the tickets cost more than the
    // spread they remove)
    if (pc.wm == 1 && x->max_local_cols < (int64_t)DYN1_MIN_COLS * pc.grid * (pc.block / 64) &&
        !(std::getenv("SPX_PRICE_DYN") && std::getenv("SPX_PRICE_DYN")[0] == '2'))  // (2: A/B, on regardless)
        P.price_dyn = 0;
    // counters: measured (tools/pass_ab.py, 2 / 4 / 8 / 16) C4 664.6 / 627.9 / 635.2 / 633.8 us
    // per pass, C5 1,032.3 / 1,023.9 / 1,022.0 / 1,010.7
    P.tk_shards = pc.wm == 1 ? 4 : 16;
    if (const char* e = std::getenv("SPX_TK_SHARDS")) {  // A/B
        const int v = std::atoi(e);
        if (v >= 1 && v <= 16) P.tk_shards = v;
    }
    // every counter must have waves drawing from it (k_price: counter
    // (wave + workgroup) mod shards reaches WAVES + grid - 1 counters);
    // SPX_TK_UNSAFE=1 skips the cap (tests: k_price's coverage check must
    // then stop the solve)
    if (!env_on("SPX_TK_UNSAFE"))
        P.tk_shards = (int32_t)std::min<int64_t>(P.tk_shards, (int64_t)pc.block / 64 + pc.grid - 1);
    pc.tk = pc.wm == 1 && P.price_dyn;
    if (pc.tk) {  // (its own instantiation: the LDS attribute set for it too)
        int per_cu_tk = 0;
        HIP_TRY(price_prepare(pc, &per_cu_tk));
        // the grid was sized from the static instantiation's occupancy: if the
        // ticketed one holds fewer workgroups per CU, size it from that, so the
        // grid stays one dispatch round (and re-cap the counters to it)
        if (per_cu_tk >= 1 && per_cu_tk < per_cu && x->opts.price_grid <= 0) {
            pc.grid = (int)std::max<int64_t>(1, std::min<int64_t>(pc.grid, (int64_t)x->cus * per_cu_tk));
            if (!env_on("SPX_TK_UNSAFE"))
                P.tk_shards = (int32_t)std::min<int64_t>(P.tk_shards, (int64_t)pc.block / 64 + pc.grid - 1);
        }
    }

    UpdateCfg& uc = x->ucfg;
    int ub = x->opts.update_block;
    // measured (tools/itbench.py): 16 waves x 1 row at m <= 8192 (C3: 1024x1),
    // 8 waves x 2 rows beyond (C5: 512x2, 4.3 GB streamed per launch)
    // and for small m the largest block that still gives every CU a workgroup
    // (C2, m=1024: 256 threads, update 20 -> 14 us)
    const int64_t rows_here = P.mloc;
    const bool big_m = rows_here > 8192;
    // eta window (read-only stream, measured at C3): 8 waves x 1 row, 33.7 us
    // against 36.2 us for 16 x 1 and 35.5 us for 8 x 2
    if (!(ub == 256 || ub == 512 || ub == 1024)) {
        ub = (big_m || P.win) ? 512 : 1024;
        while (ub > 256 && rows_here / (ub / 64) < x->cus) ub /= 2;
    }
    int rows = x->opts.update_rows;
    if (!(rows == 1 || rows == 2 || rows == 4 || rows == 8)) rows = (big_m && !P.win) ? 2 : 1;
    if (ub == 1024 && rows == 8) rows = 4;  // <1024, 8> spills registers: not instantiated
    uc.block = ub;
    uc.rows = rows;
    uc.bc_entry = env_off("SPX_FTRAN_BC_ENTRY") ? 0 : 1;
    if (uc.bc_entry) {  // k_ftran_bc rows per wave (deferred tail; the same bits at every value)
        const char* ev = std::getenv("SPX_FTRAN_RPW");
        const int r = ev ? std::atoi(ev) : 0;
        if (r == 1 || r == 2 || r == 4) uc.bc_entry = r;
    }
    uc.mark = env_on("SPX_DIAG_MARK");
    const int64_t rows_per_wg = (int64_t)(ub / 64) * rows;
    uc.grid = (int)std::max<int64_t>(1, (P.mloc + rows_per_wg - 1) / rows_per_wg);
    if (P.tab) {  // k_tab_update: one lane per row, 256 rows per workgroup
        uc.block = 256;
        uc.rows = 1;
        uc.grid = (int)std::max<int64_t>(1, (P.mloc + 255) / 256);
    }

    SPX_TRY(x->alloc(&P.price_partials, (size_t)pc.grid));
    P.upd_cap = uc.grid;
    SPX_TRY(x->alloc(&P.upd_soa, (size_t)(7 * uc.grid)));
    if (!P.row_shard && !P.tab && !(x->opts.flags & SPX_FLAG_COUNTED_TAIL))
        SPX_TRY(x->alloc(&P.upd_tag, (size_t)(UPD_WORDS * uc.grid)));
    P.price_cap = pc.grid;
    if (!P.tab && !(x->opts.flags & SPX_FLAG_COUNTED_TAIL))
        SPX_TRY(x->alloc(&P.price_tag, (size_t)(PRICE_WORDS * pc.grid)));
    // the persistent loop kernel replaces the two-kernel pass where it applies
    if (P.win && !P.tab && G == 1 && !P.row_shard && P.ratio != RATIO_HARRIS && !P.steep &&
        !(x->opts.flags & SPX_FLAG_STAMPS) &&
        !(x->opts.flags & (SPX_FLAG_NO_PERSIST | SPX_FLAG_COMM1))) {
        x->lcfg.block = x->opts.loop_block;
        HIP_TRY(loop_prepare(P, x->cus, x->lcfg, bc_possible(x, P)));
        P.bc_lds = x->lcfg.bc_lds;
        // opt-in only (SPX_FLAG_PERSIST).  Rounds 1-2 ran it by default where y_w
        // and the base row do not both fit in LDS (C5), because the two-kernel
        // pass's pricing, then a 1024-thread workgroup capped at 128 VGPRs,
        // spilled: C5 690 vs 959 it/s.  With 512-thread pricing workgroups the
        // two-kernel pass runs C5 at 957 it/s (profiles/r03_bench_c5*.json),
        // so one dispatch -- two kernels per pass -- holds at every size and
        // every rank count (k_loop is single-rank)
        const bool want = (x->opts.flags & SPX_FLAG_PERSIST) != 0;
        if (x->lcfg.ok && want) {
            SPX_TRY(x->alloc(&x->la.pp, (size_t)x->lcfg.grid));
            SPX_TRY(x->alloc(&x->la.up, (size_t)x->lcfg.grid));
            SPX_TRY(x->alloc(&x->la.ls, 1));
            SPX_TRY(x->alloc(&x->la.clock, (size_t)(3 * 64)));
            x->persist = true;
        }
    }
    // window tableau: the persistent tableau loop (k_tab_loop) unless told not to
    if (P.tab && G == 1 && P.ratio != RATIO_HARRIS &&
        !(x->opts.flags & (SPX_FLAG_STAMPS | SPX_FLAG_NO_PERSIST | SPX_FLAG_COMM1))) {
        HIP_TRY(tab_loop_prepare(P, x->cus, x->opts.price_grid, x->lcfg));
        if (x->lcfg.ok) {
            size_t xpb = 0, xub = 0;
            tab_loop_partial_bytes(x->lcfg, &xpb, &xub);
            unsigned char *xp = nullptr, *xu = nullptr;
            SPX_TRY(x->alloc(&xp, xpb));
            SPX_TRY(x->alloc(&xu, xub));
            // tagged partial words (spx_tableau.hip): no tag matches 0xFF..
            HIP_TRY(hipMemset(xp, 0xFF, xpb));
            HIP_TRY(hipMemset(xu, 0xFF, xub));
            x->la.xp = xp;
            x->la.xu = xu;
            SPX_TRY(x->alloc(&x->la.pp, (size_t)x->lcfg.grid));
            SPX_TRY(x->alloc(&x->la.up, (size_t)x->lcfg.grid));
            SPX_TRY(x->alloc(&x->la.ls, 1));
            SPX_TRY(x->alloc(&x->la.clock, (size_t)(3 * 64)));
            x->persist = true;
        }
    }
    // compact FTRAN operand (Params::bc): two-kernel window passes on one
    // device-resident B_w with A[:, n-m:] = I (checked below, after the
    // upload), while A_p's gather fits beside the k_update LDS
    x->bc_want = bc_possible(x, P) && (!x->persist || x->lcfg.bc_lds > 0);
    if (x->opts.flags & SPX_FLAG_STAMPS) {
        // 32 phase slots, 4 per k_ftran_bc workgroup (up to 4096), 2 per k_price workgroup
        SPX_TRY(x->alloc(&P.stamps, (size_t)STAMP_WORDS));
        SPX_TRY(reset_stamps(x));
    }
    SPX_TRY(x->alloc(&x->send, (size_t)P.pr_stride));
    SPX_TRY(x->alloc(&x->recv, (size_t)(G * P.pr_stride)));
    if (P.row_shard) {
        P.rs_stride = (int64_t)sizeof(RsHeader) + 8 * L;
        unsigned char *sb = nullptr, *rb = nullptr;
        SPX_TRY(x->alloc(&sb, (size_t)P.rs_stride));
        SPX_TRY(x->alloc(&rb, (size_t)(P.rs_stride * G)));
        P.rs_send = sb;
        P.rs_recv = rb;
        x->rs_recv = rb;
    }
    x->use_comm = G > 1 || (x->opts.flags & SPX_FLAG_COMM1);
    P.price_grid = pc.grid;
    P.defer_price = 0;  // set per launch by enqueue_pass (the step-wise API keeps the tail)
    // measured: C3 window 107.0 -> 105.8 us per pass (the B_w rows are already
    // in flight when k_update reduces the partials), C2 explicit 24.9 -> 23.2
    // us; C3 explicit 126.5 -> 128.5 us (its stream waits for the reduction),
    // so not for large explicit passes
    x->defer_ok = (P.win || m <= 2048) && !x->use_comm && !P.split_tail && !P.row_shard &&
                  !(x->opts.flags & SPX_FLAG_PRICE_TAIL);
    P.price_out = x->send;
    P.price_in = x->use_comm ? x->recv : x->send;
    P.nin = G;

    // passes (RCCL calls included) are captured into hipGraphs of 16; a
    // capture that fails falls back to eager launches (build_graph)
    int gb = x->opts.graph_batch;
    if (gb == 0) gb = 16;
    x->batch = (gb < 0 || x->timing) ? 0 : gb;
    // eta window: a captured batch starts with a fold and spans whole windows
    if (x->batch > 0 && P.win) x->batch = (int)round_up(x->batch, P.win - 1);
    return SPX_OK;
}

// Window tableau: T_w = B_w A and dw = y_w A - c from the current state (no
// pivot pending).  At the slack basis B_w = I, so T_w is a copy of A.
int tab_rebuild(spx_ctx* x, bool slack) {
    if (!x->P.tab) return SPX_OK;
    if (slack)
        HIP_TRY(hipMemcpyAsync(x->P.T, x->A, (size_t)(x->L * x->n) * sizeof(double), hipMemcpyDeviceToDevice,
                               x->stream));
    else
        HIP_TRY(launch_tab_build(x->P, x->stream));
    HIP_TRY(launch_reduced_costs(x->P, x->P.dw, x->stream));
    return SPX_OK;
}

// k_price's column tickets (WM 2): each pass zeroes the other parity's
// counter for the pass after it, so a pass that prices twice at one iteration
// count (spx_price repeated, a basis set or rebuilt after the last pricing)
// needs both cleared first
int clear_tickets(spx_ctx* x) {
    HIP_TRY(hipMemsetAsync(x->P.tickets, 0, TICKET_WORDS * sizeof(uint32_t), x->stream));
    return SPX_OK;
}

int do_reset(spx_ctx* x) {
    const size_t mb = (size_t)(std::max<int64_t>(x->P.mloc, 1) * x->L) * sizeof(double);
    HIP_TRY(hipMemsetAsync(x->P.B0, 0, mb, x->stream));
    if (x->P.B1 != x->P.B0) HIP_TRY(hipMemsetAsync(x->P.B1, 0, mb, x->stream));
    for (double* v : {x->P.alpha0, x->P.alpha1, x->P.y0, x->P.y1, x->P.x_b, x->P.c_B})
        HIP_TRY(hipMemsetAsync(v, 0, (size_t)x->L * sizeof(double), x->stream));
    SPX_TRY(clear_tickets(x));
    HIP_TRY(launch_reset(x->P, x->stream));
    HIP_TRY(launch_se_init(x->P, x->stream));  // steepest edge: gamma_j = 1 + ||A_j||^2
    if (x->P.bc) {  // B_w = I: no column list
        HIP_TRY(hipMemsetAsync(x->P.rleft, 0, (size_t)x->L * sizeof(int32_t), x->stream));
        HIP_TRY(hipMemsetAsync(x->P.rmap, 0xFF, (size_t)x->L * sizeof(int32_t), x->stream));
        HIP_TRY(hipMemsetAsync(x->P.bc_n, 0, BC_N_WORDS * sizeof(int32_t), x->stream));
    }
    SPX_TRY(tab_rebuild(x, true));
    HIP_TRY(hipStreamSynchronize(x->stream));
    x->pivots = 0;
    x->status = SPX_STATUS_MAX_ITER;
    x->stepped_price = false;
    x->nw = 0;
    return SPX_OK;
}

// Eta window: a fold is due before a pass that starts with nw == KW; each
// pass adds one pivot (a pass that makes none leaves the device's nw behind
// the host's count — harmless: k_fold re-checks nw, and every call starts
// from a readback).
bool fold_due(const spx_ctx* x) { return x->P.win && x->nw >= x->P.win; }
void advance_window(spx_ctx* x, bool folded) {
    if (x->P.win) x->nw = (folded ? 1 : x->nw) + 1;
}

// The next pair of fold events (timing): spx_loop_times' fold_ms / folds.
int fold_events(spx_ctx* x, hipEvent_t* f0, hipEvent_t* f1) {
    if (x->ev_fold.size() < 2 * (x->n_fold + 1)) {
        for (int i = 0; i < 2; ++i) {
            hipEvent_t e;
            HIP_TRY(hipEventCreate(&e));
            x->ev_fold.push_back(e);
        }
    }
    *f0 = x->ev_fold[2 * x->n_fold];
    *f1 = x->ev_fold[2 * x->n_fold + 1];
    ++x->n_fold;
    return SPX_OK;
}

// One loop pass: pricing, (MINLOC exchange), fused update.
int enqueue_pass(spx_ctx* x, bool timed) {
    hipEvent_t p0 = nullptr, p1 = nullptr, u0 = nullptr, u1 = nullptr;
    if (timed) {
        if (x->ev_price.size() < 2 * (x->n_price + 1)) {
            for (int k = 0; k < 2; ++k) {
                hipEvent_t e;
                HIP_TRY(hipEventCreate(&e));
                x->ev_price.push_back(e);
            }
        }
        if (x->ev_update.size() < 2 * (x->n_update + 1)) {
            for (int k = 0; k < 2; ++k) {
                hipEvent_t e;
                HIP_TRY(hipEventCreate(&e));
                x->ev_update.push_back(e);
            }
        }
        if (x->ev_xend.size() < x->n_price + 1) {
            hipEvent_t e;
            HIP_TRY(hipEventCreate(&e));
            x->ev_xend.push_back(e);
        }
        p0 = x->ev_price[2 * x->n_price];
        p1 = x->ev_price[2 * x->n_price + 1];
        u0 = x->ev_update[2 * x->n_update];
        u1 = x->ev_update[2 * x->n_update + 1];
        ++x->n_price;
        ++x->n_update;
    }
    const bool fold = fold_due(x);
    if (x->capturing) x->graph_folds += fold ? 1 : 0;
    else {
        ++x->n_eager;
        x->n_folds += fold ? 1 : 0;
    }
    if (fold) {
        hipEvent_t f0 = nullptr, f1 = nullptr;
        if (timed) SPX_TRY(fold_events(x, &f0, &f1));
        if (x->defer_tail) HIP_TRY(launch_apply_tail(x->P, x->stream));  // the fold reads the pivot's state
        if (f0) HIP_TRY(hipEventRecord(f0, x->stream));
        HIP_TRY(launch_fold(x->P, x->P.win, x->cus, x->stream));
        if (f1) HIP_TRY(hipEventRecord(f1, x->stream));
    }
    advance_window(x, fold);
    // steepest edge: after the fold, before pricing (k_se_part skipped when the
    // previous pass's FTRAN left its sums and no fold came between)
    HIP_TRY(launch_se_prep(x->P, x->stream, (x->se_fuse && x->se_chain && !fold) ? x->ucfg.grid : 0));
    Params Pp = x->P;  // loop passes: the pricing tail is reduced by k_update
    Pp.se_fused = x->se_fuse ? 1 : 0;
    Pp.defer_price = x->defer_ok ? 1 : 0;
    Pp.defer_tail = x->defer_tail ? 1 : 0;
    Pp.mbox_fused = (x->mbox_ready && x->mbox_fused) ? 1 : 0;
    HIP_TRY(launch_price(Pp, x->pcfg, x->stream, p0, p1));
    if (x->use_comm) {
        if (x->mbox_ready) {
            if (!Pp.mbox_fused) HIP_TRY(launch_exchange(x->P, x->stream));
        } else {
            if (!x->comm_ready) return fail(SPX_ERR_STATE, "nranks > 1 but neither spx_attach_comm nor spx_mbox_attach was called");
            NCCL_TRY(ncclAllGather(x->send, x->recv, sizeof(ArgMinEntry) * x->P.pr_stride, ncclUint8, x->comm,
                                   x->stream));
        }
    }
    if (timed) HIP_TRY(hipEventRecord(x->ev_xend[x->n_price - 1], x->stream));
    HIP_TRY(launch_update(Pp, x->ucfg, x->stream, u0, u1));
    x->se_chain = x->se_fuse;
    if (x->P.split_tail) HIP_TRY(launch_tail(x->P, x->ucfg.grid, x->stream));
    if (x->P.row_shard) {  // ratio-test all-gather (header + candidate row), then finalise
        if (!x->comm_ready) return fail(SPX_ERR_STATE, "row-sharded B^-1 needs spx_attach_comm");
        NCCL_TRY(ncclAllGather(x->P.rs_send, x->rs_recv, (size_t)x->P.rs_stride, ncclUint8, x->comm, x->stream));
        HIP_TRY(launch_finalize_rs(x->P, x->stream));
    }
    return SPX_OK;
}

int build_graph(spx_ctx* x) {
    if (x->graph_exec || x->batch <= 0) return SPX_OK;
    if (x->use_comm && !x->comm_ready && !x->mbox_ready)
        return fail(SPX_ERR_STATE, "nranks > 1 but neither spx_attach_comm nor spx_mbox_attach was called");
    HIP_TRY(hipStreamBeginCapture(x->stream, hipStreamCaptureModeThreadLocal));
    int rc = SPX_OK;
    const int nw_keep = x->nw;
    if (x->P.win) x->nw = x->P.win;  // a batch starts with a fold (see iterate)
    x->capturing = true;
    x->graph_folds = 0;
    for (int i = 0; i < x->batch && rc == SPX_OK; ++i) rc = enqueue_pass(x, false);
    x->capturing = false;
    x->se_chain = false;  // (nothing captured has run)
    x->nw = nw_keep;
    hipGraph_t g = nullptr;
    hipError_t e = hipStreamEndCapture(x->stream, &g);
    hipError_t ei = hipSuccess;
    if (rc == SPX_OK && e == hipSuccess) ei = hipGraphInstantiate(&x->graph_exec, g, nullptr, nullptr, 0);
    if (x->use_comm && (rc != SPX_OK || e != hipSuccess || ei != hipSuccess)) {
        // RCCL calls that cannot be captured: launch the passes eagerly
        if (g) (void)hipGraphDestroy(g);
        x->graph_exec = nullptr;
        x->batch = 0;
        x->graph_fallback = true;
        (void)hipGetLastError();
        return SPX_OK;
    }
    if (rc != SPX_OK) return rc;
    if (e != hipSuccess) return fail(SPX_ERR_HIP, "hipStreamEndCapture: %s", hipGetErrorString(e));
    x->graph = g;
    if (ei != hipSuccess) return fail(SPX_ERR_HIP, "hipGraphInstantiate: %s", hipGetErrorString(ei));
    ++x->n_graph_builds;
    // the first launch of a fresh graph pays its upload (measured 13 ms for a
    // 63-node graph): do it here, not inside somebody's timed loop
    HIP_TRY(hipGraphUpload(x->graph_exec, x->stream));
    HIP_TRY(hipStreamSynchronize(x->stream));
    return SPX_OK;
}

// The ticketed pricing tail's coverage (k_price, Params::price_dyn): each
// pass's workgroup 0 checks the previous pass's counters on the device
// (DevState::uncovered); the last pass of a call is checked here, from its
// counters and the slots each had to hand out (word 1 of its line).
int check_tickets(spx_ctx* x) {
    bool bad = x->st_host->uncovered != 0;
    if (!bad && x->P.price_dyn && (x->pcfg.wm == 2 || x->pcfg.tk)) {
        uint32_t t[TICKET_WORDS];
        HIP_TRY(hipMemcpy(t, x->P.tickets, sizeof(t), hipMemcpyDeviceToHost));
        for (int k = 0; k < 2 * x->P.tk_shards; ++k) bad = bad || t[32 * k + 1] > t[32 * k];
    }
    if (bad) {
        return fail(SPX_ERR_STATE, "pricing: ticketed list slots were left unpriced (tk_shards %d, grid %d): the "
                    "entering column may be wrong; call spx_reset", x->P.tk_shards, x->pcfg.grid);
    }
    return SPX_OK;
}

int read_state(spx_ctx* x) {
    HIP_TRY(hipMemcpyAsync(x->st_host, x->P.st, sizeof(DevState), hipMemcpyDeviceToHost, x->stream));
    HIP_TRY(hipStreamSynchronize(x->stream));
    x->pivots = x->st_host->iter;
    x->status = x->st_host->status;  // ST_RUNNING == SPX_STATUS_MAX_ITER
    x->nw = x->st_host->nw;
    if (x->status == ST_WINDOW_FULL) return fail(SPX_ERR_STATE, "internal error: eta window overflow");
    if (x->status == ST_HANDOFF_TIMEOUT) return fail(SPX_ERR_STATE, "internal error: ratio-test hand-off timed out");
    SPX_TRY(check_tickets(x));
    return SPX_OK;
}

// Apply the deferred y / x_b updates of the last pivot (spx_device.h) so the
// vectors in HBM are current.  Not valid between spx_price and spx_pivot.
int flush(spx_ctx* x) {
    if (x->stepped_price) return fail(SPX_ERR_STATE, "state readback between spx_price and spx_pivot");
    if (x->P.win) {  // fold every complete pivot: the explicit form the readback kernels expect
        HIP_TRY(launch_fold(x->P, 2, x->cus, x->stream));
        HIP_TRY(launch_tab_binv(x->P, x->stream));  // tableau without k_fold: B_w from T_w
        x->nw = std::min(x->nw, 1);
    }
    HIP_TRY(launch_flush(x->P, x->stream));
    return SPX_OK;
}

int reset_stamps(spx_ctx* x) {
    unsigned long long init[32] = {0};
    init[0] = init[4] = init[16] = init[20] = ~0ull;  // running minima
    HIP_TRY(hipMemcpy(x->P.stamps, init, sizeof(init), hipMemcpyHostToDevice));
    return SPX_OK;
}

// Row-sharded storage with a communicator: every rank's x_b rows to all
// ranks (in-place all-gather of ceil(m/G)-row slices).  Collective.
int gather_xb(spx_ctx* x) {
    if (!x->P.row_shard || !x->comm_ready) return SPX_OK;
    NCCL_TRY(ncclAllGather(x->P.x_b + x->P.r0, x->P.x_b, (size_t)x->mb, ncclFloat64, x->comm, x->stream));
    return SPX_OK;
}

int set_limit(spx_ctx* x, int64_t limit) {
    *x->limit_host = limit;
    HIP_TRY(hipMemcpyAsync(&x->P.st->limit, x->limit_host, sizeof(int64_t), hipMemcpyHostToDevice, x->stream));
    return SPX_OK;
}

int iterate_raw(spx_ctx* x, int64_t k);
int reinvert_current(spx_ctx* x);

// k passes, with a basis reinversion every opts.refactor_every pivots
int iterate(spx_ctx* x, int64_t k) {
    if (x->broken) return fail(SPX_ERR_STATE, "no valid basis (a failed spx_set_basis): call spx_reset");
    const int64_t K = x->opts.refactor_every;
    if (K <= 0) return iterate_raw(x, k);
    int64_t left = k;
    while (left > 0 && x->status == SPX_STATUS_MAX_ITER) {
        const int64_t chunk = std::min(left, std::max<int64_t>(1, x->refactor_base + K - x->pivots));
        const int64_t before = x->pivots;
        SPX_TRY(iterate_raw(x, chunk));
        left -= chunk;
        if (x->pivots == before) break;
        if (x->status == SPX_STATUS_MAX_ITER && x->pivots - x->refactor_base >= K) SPX_TRY(reinvert_current(x));
    }
    return SPX_OK;
}

// Persistent loop: one launch per window (k_loop, co-resident grid), folds between.
int iterate_persist(spx_ctx* x, int64_t k) {
    const int64_t target = x->pivots + k;
    int64_t left = k;
    int32_t launches = 0;
    while (left > 0) {
        const bool fold = fold_due(x);
        if (fold) {
            hipEvent_t f0 = nullptr, f1 = nullptr;
            if (x->timing) {
                SPX_TRY(fold_events(x, &f0, &f1));
                HIP_TRY(hipEventRecord(f0, x->stream));
            }
            HIP_TRY(launch_fold(x->P, x->P.win, x->cus, x->stream));
            if (f1) HIP_TRY(hipEventRecord(f1, x->stream));
            x->nw = 1;
            ++x->n_folds;
        }
        const int64_t np = std::min<int64_t>(left, x->P.win - x->nw);
        LoopArgs a = x->la;
        a.npasses = (int32_t)np;
        a.epoch = ++x->loop_epoch & 0x1ffffffu;  // 25 bits: the tag keeps 7 for pass and phase
        a.call_launch = launches++;
        if (!x->timing) a.clock = nullptr;
        HIP_TRY(hipMemsetAsync(a.ls, 0, LOOP_STATE_RESET, x->stream));
        hipEvent_t e0 = nullptr, e1 = nullptr;
        if (x->timing) {
            if (x->ev_loop.size() < 2 * (x->n_loop + 1)) {
                for (int i = 0; i < 2; ++i) {
                    hipEvent_t e;
                    HIP_TRY(hipEventCreate(&e));
                    x->ev_loop.push_back(e);
                }
                x->ev_loop_passes.push_back(0);
            }
            e0 = x->ev_loop[2 * x->n_loop];
            e1 = x->ev_loop[2 * x->n_loop + 1];
            x->ev_loop_passes[x->n_loop] = (int32_t)np;
            ++x->n_loop;
            HIP_TRY(hipEventRecord(e0, x->stream));
        }
        HIP_TRY(x->P.tab ? launch_tab_loop(x->P, a, x->lcfg, x->stream) : launch_loop(x->P, a, x->lcfg, x->stream));
        ++x->n_persist_launch;
        x->n_persist_pass += np;
        if (e1) HIP_TRY(hipEventRecord(e1, x->stream));
        if (x->timing) {  // phase split from workgroup 0's clock (s_memrealtime, 100 MHz)
            unsigned long long ck[3 * 64];
            LoopState ls{};
            HIP_TRY(hipStreamSynchronize(x->stream));
            HIP_TRY(hipMemcpy(&ls, a.ls, sizeof(ls), hipMemcpyDeviceToHost));
            const int done = std::min<int>(ls.passes, 64);
            HIP_TRY(hipMemcpy(ck, a.clock, sizeof(unsigned long long) * 3 * (size_t)done, hipMemcpyDeviceToHost));
            for (int i = 0; i < done; ++i) {
                x->loop_clock[0] += 1e-2 * (double)(ck[3 * i + 1] - ck[3 * i]);
                x->loop_clock[1] += 1e-2 * (double)(ck[3 * i + 2] - ck[3 * i + 1]);
                if (i + 1 < done) x->loop_clock[2] += 1e-2 * (double)(ck[3 * i + 3] - ck[3 * i + 2]);
            }
            x->loop_clock_passes += done;
        }
        x->nw += (int)np;
        left -= np;
    }
    SPX_TRY(read_state(x));
    LoopState ls{};
    HIP_TRY(hipMemcpy(&ls, x->la.ls, sizeof(ls), hipMemcpyDeviceToHost));
    if (ls.nores) {
        // some launch found its grid not co-resident (another stream or
        // process held CUs) and left the state untouched: from here on this
        // context runs two-kernel passes, and the passes those launches did
        // not make are made that way now
        HIP_TRY(hipMemsetAsync(x->la.ls, 0, sizeof(LoopState), x->stream));
        x->persist = false;
        ++x->n_persist_fallback;
        // k_loop never touches k_price's column tickets, and each two-kernel
        // pass only zeroes the other parity's: a stepped spx_price before the
        // persistent launches can have left this parity's counters used
        SPX_TRY(clear_tickets(x));
        x->nw = x->P.win ? x->st_host->nw : 0;
        const int64_t left = target - x->pivots;
        if (x->status == SPX_STATUS_MAX_ITER && left > 0) return iterate_raw(x, left);
        return SPX_OK;
    }
    if (ls.err) return fail(SPX_ERR_STATE, "persistent loop: a grid barrier timed out");
    return SPX_OK;
}

int iterate_raw(spx_ctx* x, int64_t k) {
    if (x->status != SPX_STATUS_MAX_ITER || k <= 0) return SPX_OK;
    if (x->persist && !x->stepped_price) {
        SPX_TRY(set_limit(x, x->pivots + k));
        return iterate_persist(x, k);
    }
    if (x->stepped_price) return fail(SPX_ERR_STATE, "spx_price was called without spx_pivot");
    SPX_TRY(set_limit(x, x->pivots + k));
    x->se_chain = false;  // (steepest edge: the fused sums are used within one call only)
    // exactly k passes: whole captured batches, then the remainder eagerly.
    // Eta window: batches are captured starting with a fold, so eager passes
    // first bring the window to nw == KW.
    int64_t left = k;
    if (x->batch > 0) {
        const int64_t lead = x->P.win ? std::max(0, x->P.win - x->nw) : 0;
        if (left >= lead + x->batch) {
            for (int64_t i = 0; i < lead; ++i) SPX_TRY(enqueue_pass(x, x->timing));
            left -= lead;
            SPX_TRY(build_graph(x));
            const int64_t reps = left / x->batch;
            for (int64_t i = 0; i < reps; ++i) HIP_TRY(hipGraphLaunch(x->graph_exec, x->stream));
            x->se_chain = false;
            x->n_graph_launch += reps;
            x->n_graph_pass += reps * x->batch;
            x->n_folds += reps * x->graph_folds;
            left -= reps * x->batch;  // a batch of whole windows leaves nw == KW again
        }
    }
    for (int64_t i = 0; i < left; ++i) SPX_TRY(enqueue_pass(x, x->timing));
    if (x->defer_tail) HIP_TRY(launch_apply_tail(x->P, x->stream));  // the last pass's tail, before any readback
    x->se_chain = false;
    return read_state(x);
}

// ---------------------------------------------------------------------------
// Basis reinversion (spx_reinv.h)
// ---------------------------------------------------------------------------
int rv_prepare(spx_ctx* x) {
    if (x->rv.X) return SPX_OK;
    RvParams& R = x->rv;
    const int64_t m = x->m, L = x->L;
    R.A = x->A;
    R.m = m;
    R.L = L;
    const int64_t tiles = (m + 63) / 64;
    int64_t S = std::max<int64_t>(1, std::min<int64_t>((1024 + tiles - 1) / tiles, L / 32));
    R.ks = round_up((L + S - 1) / S, 32);
    R.S = (int32_t)((L + R.ks - 1) / R.ks);
    SPX_TRY(x->alloc(&R.X, (size_t)(m * L)));
    SPX_TRY(x->alloc(&R.Ppart, (size_t)(R.S * RV_NB * L)));
    SPX_TRY(x->alloc(&x->rv_Pa, (size_t)(RV_NB * L)));
    SPX_TRY(x->alloc(&x->rv_Pb, (size_t)(RV_NB * L)));
    SPX_TRY(x->alloc(&R.U, (size_t)(m * RV_NB)));
    SPX_TRY(x->alloc(&R.Qrows, (size_t)(RV_NB * L)));
    SPX_TRY(x->alloc(&R.Urows, (size_t)(RV_NB * RV_NB)));
    SPX_TRY(x->alloc(&R.owner, (size_t)m));
    SPX_TRY(x->alloc(&x->rv_cols, (size_t)m));
    SPX_TRY(x->alloc(&x->rv_pos, (size_t)m));
    SPX_TRY(x->alloc(&R.qsel, (size_t)RV_NB));
    SPX_TRY(x->alloc(&R.parts, (size_t)rv_select_grid(m)));
    SPX_TRY(x->alloc(&R.rs, 1));
    SPX_TRY(x->alloc(&x->rv_Ypart, (size_t)(rv_y_splits(m) * L)));
    return SPX_OK;
}

// Rebuild B^-1 (and x_b, c_B, y) for `basis` (m distinct columns, basis order)
// on the device; nothing is left pending.  Host-validated basis.
int reinvert_basis(spx_ctx* x, const int64_t* basis) {
    if (x->P.row_shard) return fail(SPX_ERR_STATE, "basis reinversion needs replicated B^-1 (no row sharding)");
    SPX_TRY(rv_prepare(x));
    SPX_TRY(clear_tickets(x));
    RvParams& R = x->rv;
    const int64_t m = x->m, ns = x->ns, L = x->L;
    std::vector<int32_t> owner((size_t)m, -1);
    std::vector<int64_t> cols, pos;
    for (int64_t k = 0; k < m; ++k) {
        if (basis[k] >= ns) owner[(size_t)(basis[k] - ns)] = (int32_t)k;  // slacks keep their rows
        else { cols.push_back(basis[k]); pos.push_back(k); }
    }
    HIP_TRY(hipStreamSynchronize(x->stream));
    HIP_TRY(hipMemcpy(R.owner, owner.data(), (size_t)m * sizeof(int32_t), hipMemcpyHostToDevice));
    if (!cols.empty()) {
        HIP_TRY(hipMemcpy(x->rv_cols, cols.data(), cols.size() * sizeof(int64_t), hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(x->rv_pos, pos.data(), pos.size() * sizeof(int64_t), hipMemcpyHostToDevice));
    }
    HIP_TRY(hipMemcpy(x->P.b_ixs, basis, (size_t)m * sizeof(int64_t), hipMemcpyHostToDevice));
    HIP_TRY(hipMemsetAsync(R.rs, 0, sizeof(RvState), x->stream));
    HIP_TRY(hipMemsetAsync(R.X, 0, (size_t)(m * L) * sizeof(double), x->stream));
    HIP_TRY(rv_launch_identity(R, x->stream));
    const int64_t ncols = (int64_t)cols.size();
    for (int64_t b0 = 0; b0 < ncols; b0 += RV_NB) {
        R.nb = (int32_t)std::min<int64_t>(RV_NB, ncols - b0);
        R.cols = x->rv_cols + b0;
        R.pos = x->rv_pos + b0;
        HIP_TRY(rv_launch_gemm(R, x->stream));
        HIP_TRY(rv_launch_reduce(R, x->rv_Pa, x->stream));
        double* pin = x->rv_Pa;
        double* pout = x->rv_Pb;
        for (int tau = 0; tau < R.nb; ++tau) {
            HIP_TRY(rv_launch_step(R, tau, pin, pout, x->stream));
            std::swap(pin, pout);
        }
        HIP_TRY(rv_launch_fold(R, x->cus, x->stream));
    }
    RvState rs{};
    HIP_TRY(hipStreamSynchronize(x->stream));
    HIP_TRY(hipMemcpy(&rs, R.rs, sizeof(rs), hipMemcpyDeviceToHost));
    if (rs.singular)
        return fail(SPX_ERR_SINGULAR, "singular basis: no pivot above tolerance for column %lld (basis position %lld)",
                    (long long)basis[rs.bad_pos], (long long)rs.bad_pos);
    HIP_TRY(rv_launch_finish(x->P, R, x->rv_Ypart, x->stream));
    if (x->P.bc) {  // the new B_w's non-unit columns: rows whose slack is not basic in them
        std::vector<int32_t> left((size_t)x->L, 0);
        for (int64_t k = 0; k < m; ++k) left[(size_t)k] = basis[k] != ns + k ? 1 : 0;
        HIP_TRY(hipMemcpyAsync(x->P.rleft, left.data(), (size_t)x->L * sizeof(int32_t), hipMemcpyHostToDevice,
                               x->stream));
        HIP_TRY(hipMemsetAsync(x->P.rmap, 0xFF, (size_t)x->L * sizeof(int32_t), x->stream));
        HIP_TRY(hipMemsetAsync(x->P.bc_n, 0, BC_N_WORDS * sizeof(int32_t), x->stream));
        HIP_TRY(launch_compact(x->P, x->stream));
        HIP_TRY(hipStreamSynchronize(x->stream));  // (left is a host buffer)
    }
    SPX_TRY(tab_rebuild(x, false));
    x->nw = 0;
    return read_state(x);
}

int check_basis(const spx_ctx* x, const int64_t* basis) {
    if (!basis) return fail(SPX_ERR_ARG, "basis is NULL");
    std::vector<char> seen((size_t)x->n, 0);
    for (int64_t k = 0; k < x->m; ++k) {
        const int64_t j = basis[k];
        if (j < 0 || j >= x->n) return fail(SPX_ERR_ARG, "basis[%lld] = %lld out of range", (long long)k, (long long)j);
        if (seen[(size_t)j]) return fail(SPX_ERR_ARG, "column %lld repeated in the basis", (long long)j);
        seen[(size_t)j] = 1;
    }
    return SPX_OK;
}

int reinvert_current(spx_ctx* x) {
    if (x->stepped_price) return fail(SPX_ERR_STATE, "reinversion between spx_price and spx_pivot");
    std::vector<int64_t> basis((size_t)x->m);
    HIP_TRY(hipStreamSynchronize(x->stream));
    HIP_TRY(hipMemcpy(basis.data(), x->P.b_ixs, (size_t)x->m * sizeof(int64_t), hipMemcpyDeviceToHost));
    SPX_TRY(reinvert_basis(x, basis.data()));
    x->refactor_base = x->pivots;
    return SPX_OK;
}

// Window tableau without k_fold (Params::tab_slack): needs A[:, n-m:] = I
// exactly (the slack basis the reference's init assumes, v4:272-275).
// A == nullptr: generated [U | I].  SPX_TAB_BW=1 keeps B_w and k_fold.
bool env_on(const char* name) {
    const char* env = std::getenv(name);
    return env && env[0] == '1';
}
bool env_off(const char* name) {
    const char* env = std::getenv(name);
    return env && env[0] == '0';
}
bool slack_identity(const double* A, int64_t m, int64_t n) {
    if (!A) return true;
    for (int64_t i = 0; i < m; ++i) {
        const double* col = A + (n - m + i) * m;  // column-major m x n
        for (int64_t r = 0; r < m; ++r)
            if (col[r] != (r == i ? 1.0 : 0.0)) return false;
    }
    return true;
}
// the two uses of A[:, n-m:] = I (A == nullptr: generated [U | I]): the
// tableau's B_w from T_w, and k_price's unit slack columns (SPX_DENSE_SLACKS=1:
// stream them like any column)
int set_slack_flags(spx_ctx* x) {
    const bool ident = x->slack_ident;
    const int64_t m = x->m;
    if (x->P.tab) x->P.tab_slack = (ident && !env_on("SPX_TAB_BW")) ? 1 : 0;
    x->P.slack_unit = (ident && !env_on("SPX_DENSE_SLACKS")) ? 1 : 0;
    if (x->bc_want && ident) {  // compact FTRAN operand (do_reset initialises it)
        Params& P = x->P;
        // m x L more doubles (2.1 GB at C5), and a second buffer of that
        // shape for the compact fold (it writes the other one, spx_device.h).
        // No room for the first: the dense B_w stream is kept (every kernel
        // tests P.bc).  No room for the second: compact FTRAN with the dense
        // fold plus the gather (k_fold + k_bc_gather, bc_n[2] stays 0).
        const size_t bytes = (size_t)(m * x->L) * sizeof(double);
        void* d0 = nullptr;
        if (hipMalloc(&d0, bytes) != hipSuccess) {
            (void)hipGetLastError();
            x->bc_want = false;
            return SPX_OK;
        }
        x->allocs.push_back(d0);
        HIP_TRY(hipMemsetAsync(d0, 0, bytes, x->stream));
        P.bc = static_cast<double*>(d0);
        P.bc1 = nullptr;
        P.cfold = 0;
        if (!env_on("SPX_DENSE_FOLD")) {
            void* d1 = nullptr;
            if (hipMalloc(&d1, bytes) == hipSuccess) {
                x->allocs.push_back(d1);
                HIP_TRY(hipMemsetAsync(d1, 0, bytes, x->stream));
                P.bc1 = static_cast<double*>(d1);
                P.cfold = 1;
            } else {
                (void)hipGetLastError();
            }
        }
        SPX_TRY(x->alloc(&P.rlist, (size_t)x->L));
        SPX_TRY(x->alloc(&P.rmap, (size_t)x->L));
        SPX_TRY(x->alloc(&P.rleft, (size_t)x->L));
        SPX_TRY(x->alloc(&P.bc_n, BC_N_WORDS));
    }
    // deferred ratio-test tail (TailRec, spx_device.h): compact FTRAN passes
    // (k_ftran_bc, one row per wave) with 512- or 256-thread pricing -- the
    // reduction shape k_price (256 threads: two partials each,
    // reduce_partial_pair), k_apply_tail and the FTRAN tail share -- on one rank
    // with the pricing tail deferred as well; with G ranks (replicated B_w, so
    // every rank holds the same FTRAN partials) the pricing tail stays in
    // k_price for the exchange.  Measured at C3 (round-2 tools/fuse_est.py, in git history, the
    // timing-only estimate): 79.8 -> 73.9 us per pass.  SPX_DEFER_TAIL=0 keeps
    // the tail in the FTRAN pass.
    const UpdateCfg& uc = x->ucfg;
    const bool tail_ok = x->defer_ok || (x->use_comm && x->P.win && !x->P.split_tail && !x->P.row_shard &&
                                         !(x->opts.flags & SPX_FLAG_PRICE_TAIL));
    if (x->P.bc && tail_ok && !x->persist && !x->P.tab && uc.bc_entry && uc.rows == 1 &&
        uc.block == 512 && (x->pcfg.block == 512 || x->pcfg.block == 256) && !env_off("SPX_DEFER_TAIL")) {
        SPX_TRY(x->alloc(&x->P.trec, 1));
        HIP_TRY(hipMemset(x->P.trec, 0, sizeof(TailRec)));
        x->P.tail_parts = uc.grid;
        x->defer_tail = true;
    }
    // (measured: tools/r6_sefuse.sh; SPX_SE_FUSE=0 keeps k_se_part)
    x->se_fuse = x->P.steep && x->defer_tail && uc.bc_entry == 1 && uc.grid <= x->se_rows && !env_off("SPX_SE_FUSE");
    return SPX_OK;
}

int create_tail(spx_ctx* x) {
    SPX_TRY(do_reset(x));
    if (!x->use_comm && !x->persist) SPX_TRY(build_graph(x));  // capture + upload now (off any timed path)
    return SPX_OK;
}

}  // namespace

extern "C" {

int spx_create(spx_ctx** out, int64_t m, int64_t n, const double* A, const double* b, const double* c,
               const spx_opts* opts) {
    if (!out) return fail(SPX_ERR_ARG, "out is NULL");
    *out = nullptr;
    if (m <= 0 || n < m) return fail(SPX_ERR_ARG, "Either failed to read m and n, or m > n. (m=%lld n=%lld)",
                                     (long long)m, (long long)n);
    if (n > (int64_t)0x7fffffff) return fail(SPX_ERR_ARG, "n too large");
    if (!A || !b || !c) return fail(SPX_ERR_ARG, "NULL input array");
    spx_ctx* x = new spx_ctx();
    x->slack_ident = slack_identity(A, m, n);
    int rc = setup_common(x, m, n, opts);
    if (rc == SPX_OK) {
        // blocking copies from pageable memory, after the zero-fills queued on the stream
        hipError_t e = hipStreamSynchronize(x->stream);
        if (e == hipSuccess)
            e = hipMemcpy2D(x->A, (size_t)x->L * 8, A, (size_t)m * 8, (size_t)m * 8, (size_t)n, hipMemcpyHostToDevice);
        if (e == hipSuccess) e = hipMemcpy(x->b, b, (size_t)m * 8, hipMemcpyHostToDevice);
        if (e == hipSuccess) e = hipMemcpy(x->c, c, (size_t)n * 8, hipMemcpyHostToDevice);
        if (e != hipSuccess) rc = fail(SPX_ERR_HIP, "upload failed: %s", hipGetErrorString(e));
    }
    if (rc == SPX_OK) rc = set_slack_flags(x);
    if (rc == SPX_OK) rc = create_tail(x);
    if (rc != SPX_OK) {
        std::string keep = g_err;
        spx_destroy(x);
        g_err = keep;
        return rc;
    }
    *out = x;
    return SPX_OK;
}

int spx_create_generated(spx_ctx** out, int64_t m, int64_t n, uint64_t seed, const spx_opts* opts) {
    if (!out) return fail(SPX_ERR_ARG, "out is NULL");
    *out = nullptr;
    if (m <= 0 || n < m) return fail(SPX_ERR_ARG, "m must be in [1, n] (m=%lld n=%lld)", (long long)m, (long long)n);
    if (n > (int64_t)0x7fffffff) return fail(SPX_ERR_ARG, "n too large");
    spx_ctx* x = new spx_ctx();
    x->slack_ident = true;  // [U | I] by construction
    int rc = setup_common(x, m, n, opts);
    if (rc == SPX_OK) {
        hipError_t e = launch_generate(x->A, x->b, x->c, m, n, x->L, seed, x->stream);
        if (e != hipSuccess) rc = fail(SPX_ERR_HIP, "generate failed: %s", hipGetErrorString(e));
    }
    if (rc == SPX_OK) rc = set_slack_flags(x);
    if (rc == SPX_OK) rc = create_tail(x);
    if (rc != SPX_OK) {
        std::string keep = g_err;
        spx_destroy(x);
        g_err = keep;
        return rc;
    }
    *out = x;
    return SPX_OK;
}

void spx_destroy(spx_ctx* x) {
    if (!x) return;
    if (x->stream) (void)hipStreamSynchronize(x->stream);
    if (x->graph_exec) (void)hipGraphExecDestroy(x->graph_exec);
    if (x->graph) (void)hipGraphDestroy(x->graph);
    for (hipEvent_t e : {x->ev_sent, x->ev_recv, x->ev_sent2, x->ev_recv2})
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : x->ev_price) (void)hipEventDestroy(e);
    for (hipEvent_t e : x->ev_update) (void)hipEventDestroy(e);
    for (hipEvent_t e : x->ev_xend) (void)hipEventDestroy(e);
    for (hipEvent_t e : x->ev_loop) (void)hipEventDestroy(e);
    for (hipEvent_t e : x->ev_fold) (void)hipEventDestroy(e);
    if (x->comm) (void)ncclCommDestroy(x->comm);
    for (void* p : x->mbox_opened) (void)hipIpcCloseMemHandle(p);
    for (void* p : x->allocs) (void)hipFree(p);
    if (x->st_host) (void)hipHostFree(x->st_host);
    if (x->limit_host) (void)hipHostFree(x->limit_host);
    if (x->stream) (void)hipStreamDestroy(x->stream);
    delete x;
}

int spx_comm_unique_id(uint8_t id[SPX_COMM_ID_BYTES]) {
    if (!id) return fail(SPX_ERR_ARG, "id is NULL");
    static_assert(sizeof(ncclUniqueId) <= SPX_COMM_ID_BYTES, "ncclUniqueId too large");
    ncclUniqueId u;
    NCCL_TRY(ncclGetUniqueId(&u));
    std::memset(id, 0, SPX_COMM_ID_BYTES);
    std::memcpy(id, &u, sizeof(u));
    return SPX_OK;
}

int spx_attach_comm(spx_ctx* x, const uint8_t id[SPX_COMM_ID_BYTES]) {
    if (!x || !id) return fail(SPX_ERR_ARG, "NULL argument");
    if (!x->use_comm) return SPX_OK;
    if (x->comm_ready) return fail(SPX_ERR_STATE, "communicator already attached");
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    HIP_TRY(hipSetDevice(x->device));
    NCCL_TRY(ncclCommInitRank(&x->comm, x->opts.nranks, u, x->opts.rank));
    x->comm_ready = true;
    return SPX_OK;
}

int spx_comm_info(spx_ctx* x, int32_t out[SPX_COMM_INFO_FIELDS], char bus_id[SPX_BUS_ID_BYTES]) {
    if (!x || !out) return fail(SPX_ERR_ARG, "NULL argument");
    int cnt = -1, urank = -1, cdev = -1;
    if (x->comm_ready) {
        NCCL_TRY(ncclCommCount(x->comm, &cnt));
        NCCL_TRY(ncclCommUserRank(x->comm, &urank));
        NCCL_TRY(ncclCommCuDevice(x->comm, &cdev));
    }
    out[0] = cnt;
    out[1] = urank;
    out[2] = cdev;
    out[3] = x->device;
    out[4] = (x->graph_exec != nullptr && x->batch > 0) ? 1 : 0;
    out[5] = x->graph_fallback ? 1 : 0;
    out[6] = x->opts.nranks;
    out[7] = x->opts.rank;
    if (bus_id) {
        std::memset(bus_id, 0, SPX_BUS_ID_BYTES);
        HIP_TRY(hipDeviceGetPCIBusId(bus_id, SPX_BUS_ID_BYTES - 1, x->device));
    }
    return SPX_OK;
}

int spx_mbox_export(spx_ctx* x, uint8_t handle[SPX_MBOX_HANDLE_BYTES]) {
    if (!x || !handle) return fail(SPX_ERR_ARG, "NULL argument");
    if (!x->use_comm) return fail(SPX_ERR_STATE, "mailboxes need opts.nranks > 1 (or SPX_FLAG_COMM1)");
    static_assert(sizeof(hipIpcMemHandle_t) <= SPX_MBOX_HANDLE_BYTES, "hipIpcMemHandle_t too large");
    HIP_TRY(hipSetDevice(x->device));
    if (!x->mbox) {
        // [2 parities][nranks][pr_stride * 4 halves] tagged words, zeroed (seq starts at 1);
        // fine-grained and uncached: peers store into it over xGMI while k_exchange polls
        const size_t words = (size_t)2 * x->opts.nranks * x->P.pr_stride * (sizeof(ArgMinEntry) / 4);
        SPX_TRY(x->alloc(&x->mbox, words, hipDeviceMallocUncached));
        SPX_TRY(x->alloc(&x->mbox_seq, 1));
        HIP_TRY(hipStreamSynchronize(x->stream));
    }
    hipIpcMemHandle_t h;
    HIP_TRY(hipIpcGetMemHandle(&h, x->mbox));
    std::memset(handle, 0, SPX_MBOX_HANDLE_BYTES);
    std::memcpy(handle, &h, sizeof(h));
    return SPX_OK;
}

int spx_mbox_attach(spx_ctx* x, const uint8_t* handles) {
    if (!x || !handles) return fail(SPX_ERR_ARG, "NULL argument");
    if (!x->mbox) return fail(SPX_ERR_STATE, "spx_mbox_export first");
    if (x->mbox_ready) return fail(SPX_ERR_STATE, "mailboxes already attached");
    HIP_TRY(hipSetDevice(x->device));
    const int G = x->opts.nranks;
    std::vector<uint64_t*> peers((size_t)G);
    bool shared_device = false;  // a peer's mailbox on this context's own device (ranks sharing a GPU)
    for (int g = 0; g < G; ++g) {
        if (g == x->opts.rank) {
            peers[(size_t)g] = x->mbox;
            continue;
        }
        hipIpcMemHandle_t h;
        std::memcpy(&h, handles + (size_t)g * SPX_MBOX_HANDLE_BYTES, sizeof(h));
        void* p = nullptr;
        const hipError_t e = hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess);
        if (e != hipSuccess) return fail(SPX_ERR_HIP, "hipIpcOpenMemHandle(rank %d): %s", g, hipGetErrorString(e));
        x->mbox_opened.push_back(p);
        peers[(size_t)g] = static_cast<uint64_t*>(p);
        hipPointerAttribute_t a{};
        // (unknown counts as shared: the k_exchange path is safe everywhere)
        if (hipPointerGetAttributes(&a, p) != hipSuccess || a.device == x->device) shared_device = true;
    }
    SPX_TRY(x->alloc(&x->mbox_peer, (size_t)G));
    HIP_TRY(hipMemcpyAsync(x->mbox_peer, peers.data(), sizeof(uint64_t*) * (size_t)G, hipMemcpyHostToDevice,
                           x->stream));
    HIP_TRY(hipStreamSynchronize(x->stream));
    x->P.mbox_peer = x->mbox_peer;
    x->P.mbox = x->mbox;
    x->P.mbox_seq = x->mbox_seq;
    x->P.mbox_rank = x->opts.rank;
    // the fused exchange where the loop pass is k_price (tagged pricing tail)
    // + k_ftran_bc (compact window FTRAN, one row per wave), and no peer
    // shares this device: there, a rank's k_ftran_bc workgroups, spinning on
    // the mailbox, can hold every CU a peer's k_price needs to produce the
    // record (measured: two processes on one GPU at m = 2048 time out), so
    // ranks sharing a GPU keep the one-workgroup k_exchange launch.
    // SPX_MBOX_FUSED=0 keeps it everywhere
    x->mbox_fused = x->P.win && x->P.bc && x->P.price_tag && !x->P.row_shard && !x->P.split_tail &&
                    x->ucfg.rows == 1 && x->ucfg.bc_entry && G <= 64 && !shared_device &&
                    !env_off("SPX_MBOX_FUSED");
    // a graph captured before (with the RCCL exchange, or none) is rebuilt
    if (x->graph_exec) (void)hipGraphExecDestroy(x->graph_exec);
    if (x->graph) (void)hipGraphDestroy(x->graph);
    x->graph_exec = nullptr;
    x->graph = nullptr;
    x->mbox_ready = true;
    return SPX_OK;
}

int spx_reset(spx_ctx* x) {
    if (!x) return fail(SPX_ERR_ARG, "ctx is NULL");
    x->refactor_base = 0;
    x->broken = false;
    return do_reset(x);
}

int spx_reinvert(spx_ctx* x) {
    if (!x) return fail(SPX_ERR_ARG, "ctx is NULL");
    if (x->broken) return fail(SPX_ERR_STATE, "no valid basis (a failed spx_set_basis): call spx_reset");
    return reinvert_current(x);
}

int spx_set_basis(spx_ctx* x, const int64_t* basis) {
    if (!x) return fail(SPX_ERR_ARG, "ctx is NULL");
    if (x->stepped_price) return fail(SPX_ERR_STATE, "spx_set_basis between spx_price and spx_pivot");
    SPX_TRY(check_basis(x, basis));
    if (x->P.row_shard) return fail(SPX_ERR_STATE, "spx_set_basis needs replicated B^-1 (no row sharding)");
    // this rank's non-basic list (ascending, owned columns only) and positions
    std::vector<char> basic((size_t)x->n, 0);
    for (int64_t k = 0; k < x->m; ++k) basic[(size_t)basis[k]] = 1;
    std::vector<int32_t> list, posv((size_t)x->n, -1);
    for (int64_t j = 0; j < x->n; ++j) {
        if (basic[(size_t)j] || !owns_col(x->P, j)) continue;
        posv[(size_t)j] = (int32_t)list.size();
        list.push_back((int32_t)j);
    }
    HIP_TRY(hipStreamSynchronize(x->stream));
    if (!list.empty())
        HIP_TRY(hipMemcpy(x->P.nb_list, list.data(), list.size() * sizeof(int32_t), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(x->P.nb_pos, posv.data(), posv.size() * sizeof(int32_t), hipMemcpyHostToDevice));
    SPX_TRY(read_state(x));
    DevState st = *x->st_host;
    st.status = ST_RUNNING;
    st.nb_count = (int32_t)list.size();
    st.p = -1;
    st.min_e = 0.0;
    st.leave = -1;  // Devex: a fresh reference framework
    st.wp = 1.0;
    HIP_TRY(hipMemcpy(x->P.st, &st, sizeof(st), hipMemcpyHostToDevice));
    if (x->P.W && !x->P.steep) {
        const std::vector<double> ones((size_t)x->n, 1.0);
        HIP_TRY(hipMemcpy(x->P.W, ones.data(), ones.size() * sizeof(double), hipMemcpyHostToDevice));
    }
    // steepest edge: the slack-basis reference values 1 + ||A_j||^2 (exact
    // weights for an arbitrary basis would need B^-1 A in full)
    HIP_TRY(launch_se_init(x->P, x->stream));
    x->broken = true;  // until the inverse is rebuilt
    SPX_TRY(reinvert_basis(x, basis));
    x->broken = false;
    x->refactor_base = x->pivots;
    return SPX_OK;
}

int spx_iterate(spx_ctx* x, int64_t k, int32_t* status, int64_t* pivots) {
    if (!x) return fail(SPX_ERR_ARG, "ctx is NULL");
    SPX_TRY(iterate(x, k));
    if (status) *status = x->status;
    if (pivots) *pivots = x->pivots;
    return SPX_OK;
}

int spx_group_iterate(spx_ctx** cs, int32_t G, int64_t k, int32_t* status, int64_t* pivots) {
    if (!cs || G < 1) return fail(SPX_ERR_ARG, "bad group");
    for (int g = 0; g < G; ++g) {
        spx_ctx* x = cs[g];
        if (!x) return fail(SPX_ERR_ARG, "NULL context in group");
        if (x->opts.nranks != G || x->opts.rank != g)
            return fail(SPX_ERR_ARG, "context %d was created with rank %d / nranks %d", g, x->opts.rank, x->opts.nranks);
        if (x->comm_ready) return fail(SPX_ERR_STATE, "group contexts must not have a communicator");
        if (x->m != cs[0]->m || x->n != cs[0]->n) return fail(SPX_ERR_ARG, "group shape mismatch");
        if (x->status != cs[0]->status || x->pivots != cs[0]->pivots) return fail(SPX_ERR_STATE, "group out of step");
        if (x->P.row_shard != cs[0]->P.row_shard || x->P.win != cs[0]->P.win)
            return fail(SPX_ERR_ARG, "group mixes storage modes");
        if (!x->ev_sent) {
            HIP_TRY(hipSetDevice(x->device));
            HIP_TRY(hipEventCreateWithFlags(&x->ev_sent, hipEventDisableTiming));
            HIP_TRY(hipEventCreateWithFlags(&x->ev_recv, hipEventDisableTiming));
            HIP_TRY(hipEventCreateWithFlags(&x->ev_sent2, hipEventDisableTiming));
            HIP_TRY(hipEventCreateWithFlags(&x->ev_recv2, hipEventDisableTiming));
        }
    }
    if (cs[0]->status == SPX_STATUS_MAX_ITER && k > 0) {
        for (int g = 0; g < G; ++g) {
            HIP_TRY(hipSetDevice(cs[g]->device));
            SPX_TRY(set_limit(cs[g], cs[g]->pivots + k));
            cs[g]->se_chain = false;
        }
        for (int64_t it = 0; it < k; ++it) {
            for (int g = 0; g < G; ++g) {  // pricing on every shard
                spx_ctx* x = cs[g];
                HIP_TRY(hipSetDevice(x->device));
                const bool fold = fold_due(x);
                if (fold && x->defer_tail) HIP_TRY(launch_apply_tail(x->P, x->stream));
                if (fold) HIP_TRY(launch_fold(x->P, x->P.win, x->cus, x->stream));
                advance_window(x, fold);
                // steepest edge: after the fold, before pricing (as enqueue_pass)
                HIP_TRY(launch_se_prep(x->P, x->stream, (x->se_fuse && x->se_chain && !fold) ? x->ucfg.grid : 0));
                ++x->n_eager;
                x->n_folds += fold ? 1 : 0;
                Params Pp = x->P;  // the deferred ratio-test tail (each rank's own FTRAN partials)
                Pp.defer_tail = x->defer_tail ? 1 : 0;
                HIP_TRY(launch_price(Pp, x->pcfg, x->stream, nullptr, nullptr));
                HIP_TRY(hipEventRecord(x->ev_sent, x->stream));
            }
            for (int h = 0; h < G; ++h) {  // all-gather of the candidate records
                spx_ctx* x = cs[h];
                HIP_TRY(hipSetDevice(x->device));
                const int ps = x->P.pr_stride;
                for (int g = 0; g < G; ++g) {
                    HIP_TRY(hipStreamWaitEvent(x->stream, cs[g]->ev_sent, 0));
                    HIP_TRY(hipMemcpyAsync(x->recv + g * ps, cs[g]->send, sizeof(ArgMinEntry) * ps,
                                           hipMemcpyDefault, x->stream));
                }
                HIP_TRY(hipEventRecord(x->ev_recv, x->stream));
            }
            const bool rs = cs[0]->P.row_shard != 0;
            for (int g = 0; g < G; ++g) {  // fused update; next pricing waits for every reader
                spx_ctx* x = cs[g];
                HIP_TRY(hipSetDevice(x->device));
                Params Pp = x->P;
                Pp.defer_tail = x->defer_tail ? 1 : 0;
                Pp.se_fused = x->se_fuse ? 1 : 0;
                HIP_TRY(launch_update(Pp, x->ucfg, x->stream, nullptr, nullptr));
                x->se_chain = x->se_fuse;
                if (x->P.split_tail) HIP_TRY(launch_tail(x->P, x->ucfg.grid, x->stream));
                if (rs) HIP_TRY(hipEventRecord(x->ev_sent2, x->stream));
                else
                    for (int h = 0; h < G; ++h) HIP_TRY(hipStreamWaitEvent(x->stream, cs[h]->ev_recv, 0));
            }
            if (rs) {
                for (int h = 0; h < G; ++h) {  // ratio-test all-gather: headers + candidate rows
                    spx_ctx* x = cs[h];
                    HIP_TRY(hipSetDevice(x->device));
                    for (int g = 0; g < G; ++g) {
                        HIP_TRY(hipStreamWaitEvent(x->stream, cs[g]->ev_sent2, 0));
                        HIP_TRY(hipMemcpyAsync(x->rs_recv + g * x->P.rs_stride, cs[g]->P.rs_send,
                                               (size_t)x->P.rs_stride, hipMemcpyDefault, x->stream));
                    }
                    HIP_TRY(hipEventRecord(x->ev_recv2, x->stream));
                }
                for (int g = 0; g < G; ++g) {
                    spx_ctx* x = cs[g];
                    HIP_TRY(hipSetDevice(x->device));
                    HIP_TRY(launch_finalize_rs(x->P, x->stream));
                    for (int h = 0; h < G; ++h) {
                        HIP_TRY(hipStreamWaitEvent(x->stream, cs[h]->ev_recv, 0));
                        HIP_TRY(hipStreamWaitEvent(x->stream, cs[h]->ev_recv2, 0));
                    }
                }
            }
        }
        for (int g = 0; g < G; ++g) {
            HIP_TRY(hipSetDevice(cs[g]->device));
            if (cs[g]->defer_tail) HIP_TRY(launch_apply_tail(cs[g]->P, cs[g]->stream));  // the last pass's tail
            cs[g]->se_chain = false;
            SPX_TRY(read_state(cs[g]));
        }
        for (int g = 1; g < G; ++g)
            if (cs[g]->status != cs[0]->status || cs[g]->pivots != cs[0]->pivots)
                return fail(SPX_ERR_STATE, "shard %d diverged (status %d/%d, pivots %lld/%lld)", g, cs[g]->status,
                            cs[0]->status, (long long)cs[g]->pivots, (long long)cs[0]->pivots);
    }
    if (status) *status = cs[0]->status;
    if (pivots) *pivots = cs[0]->pivots;
    return SPX_OK;
}

int spx_group_sync(spx_ctx** cs, int32_t G) {
    if (!cs || G < 1) return fail(SPX_ERR_ARG, "bad group");
    for (int g = 0; g < G; ++g) {
        if (!cs[g] || cs[g]->opts.nranks != G || cs[g]->opts.rank != g) return fail(SPX_ERR_ARG, "bad group member");
        HIP_TRY(hipSetDevice(cs[g]->device));
        SPX_TRY(flush(cs[g]));
        HIP_TRY(hipStreamSynchronize(cs[g]->stream));
    }
    if (!cs[0]->P.row_shard) return SPX_OK;
    for (int h = 0; h < G; ++h)
        for (int g = 0; g < G; ++g)
            if (g != h && cs[g]->P.mloc > 0)
                HIP_TRY(hipMemcpyAsync(cs[h]->P.x_b + cs[g]->P.r0, cs[g]->P.x_b + cs[g]->P.r0,
                                       (size_t)cs[g]->P.mloc * 8, hipMemcpyDefault, cs[h]->stream));
    for (int h = 0; h < G; ++h) HIP_TRY(hipStreamSynchronize(cs[h]->stream));
    return SPX_OK;
}

int spx_objective(spx_ctx* x, double* z) {
    if (!x) return fail(SPX_ERR_ARG, "ctx is NULL");
    SPX_TRY(flush(x));
    SPX_TRY(gather_xb(x));
    HIP_TRY(launch_objective(x->P, x->stream));
    SPX_TRY(read_state(x));
    if (z) *z = x->st_host->z;
    return SPX_OK;
}

int spx_get_trace(spx_ctx* x, int64_t* p, int64_t* q, int64_t cap, int64_t* count) {
    if (!x) return fail(SPX_ERR_ARG, "ctx is NULL");
    if (cap < 0) return fail(SPX_ERR_ARG, "cap must be >= 0");
    if (!x->P.trace) return fail(SPX_ERR_STATE, "no pivot trace: create the context with opts.trace_cap > 0");
    SPX_TRY(read_state(x));
    const int64_t k = std::min(std::min<int64_t>(x->pivots, x->P.trace_cap), cap);
    std::vector<int64_t> buf((size_t)(2 * std::max<int64_t>(k, 1)));
    if (k > 0) HIP_TRY(hipMemcpy(buf.data(), x->P.trace, sizeof(int64_t) * 2 * (size_t)k, hipMemcpyDeviceToHost));
    for (int64_t i = 0; i < k; ++i) {
        if (p) p[i] = buf[2 * i];
        if (q) q[i] = buf[2 * i + 1];
    }
    if (count) *count = k;
    return SPX_OK;
}

int spx_wg_times(spx_ctx* x, uint64_t* out, int64_t cap, int64_t* count) {
    if (!x || !out) return fail(SPX_ERR_ARG, "NULL argument");
    if (!x->P.stamps) return fail(SPX_ERR_STATE, "context created without SPX_FLAG_STAMPS");
    HIP_TRY(hipStreamSynchronize(x->stream));
    // per parity: k_ftran_bc 4 per workgroup, k_price 4 per workgroup, the tail end, k_mark,
    // k_price workgroup 0's deferred bookkeeping issued
    const int64_t gu = std::min(x->ucfg.grid, 4096), gp = std::min(x->pcfg.grid, 4096);
    std::vector<uint64_t> h((size_t)STAMP_WORDS);
    HIP_TRY(hipMemcpy(h.data(), x->P.stamps, sizeof(uint64_t) * h.size(), hipMemcpyDeviceToHost));
    int64_t k = 0;
    for (int par = 0; par < 2; ++par) {
        for (int64_t i = 0; i < 4 * gu && k < cap; ++i) out[k++] = h[(size_t)(STAMP_FTRAN + par * 4 * 4096 + i)];
        for (int64_t i = 0; i < 4 * gp && k < cap; ++i) out[k++] = h[(size_t)(STAMP_PRICE + par * 4 * 4096 + i)];
        if (k < cap) out[k++] = h[(size_t)(STAMP_TAIL + par)];
        if (k < cap) out[k++] = h[(size_t)(STAMP_TAIL + 2 + par)];
        if (k < cap) out[k++] = h[(size_t)(STAMP_TAIL + 4 + par)];
    }
    if (count) *count = x->ucfg.grid;
    return SPX_OK;
}

int spx_fold_times(spx_ctx* x, uint64_t* out, int64_t cap, int64_t* count) {
    if (!x || !out) return fail(SPX_ERR_ARG, "NULL argument");
    if (!x->P.stamps) return fail(SPX_ERR_STATE, "context created without SPX_FLAG_STAMPS");
    HIP_TRY(hipStreamSynchronize(x->stream));
    const int64_t n = std::min<int64_t>(cap, (int64_t)STAMP_FOLD_PER * 1024);
    HIP_TRY(hipMemcpy(out, x->P.stamps + STAMP_FOLD, sizeof(uint64_t) * (size_t)n, hipMemcpyDeviceToHost));
    if (count) *count = n;
    return SPX_OK;
}

int spx_get_weights(spx_ctx* x, double* w) {
    if (!x || !w) return fail(SPX_ERR_ARG, "NULL argument");
    if (!x->P.W) return fail(SPX_ERR_STATE, "no pricing weights: the context runs Dantzig pricing");
    HIP_TRY(hipStreamSynchronize(x->stream));
    HIP_TRY(hipMemcpy(w, x->P.W, sizeof(double) * (size_t)x->n, hipMemcpyDeviceToHost));
    return SPX_OK;
}

int spx_get_state(spx_ctx* x, double* x_b, int64_t* b_ixs, double* y, double* c_b, double* binv, int32_t* status,
                  int64_t* pivots) {
    if (!x) return fail(SPX_ERR_ARG, "ctx is NULL");
    const size_t mb = (size_t)x->m * 8;
    SPX_TRY(flush(x));
    SPX_TRY(gather_xb(x));
    // Device work is enqueued and drained first; the copies into (pageable)
    // caller memory are then plain blocking copies: an async 2D D2H copy into
    // pageable memory was seen to overtake the materialising kernel.
    double* tmp = nullptr;
    if (binv) {
        const size_t rows = (size_t)std::max<int64_t>(x->m, (int64_t)x->opts.nranks * x->mb);
        HIP_TRY(hipMalloc(reinterpret_cast<void**>(&tmp), rows * x->L * 8));
        int rc = SPX_OK;
        hipError_t e = hipSuccess;
        if (x->P.row_shard) e = hipMemsetAsync(tmp, 0, rows * x->L * 8, x->stream);
        if (e == hipSuccess) e = launch_materialize(x->P, tmp, x->stream);
        if (e == hipSuccess && x->P.row_shard && x->comm_ready) {
            const ncclResult_t r = ncclAllGather(tmp + x->P.r0 * x->L, tmp, (size_t)(x->mb * x->L), ncclFloat64,
                                                 x->comm, x->stream);
            if (r != ncclSuccess) rc = fail(SPX_ERR_RCCL, "binv all-gather: %s", ncclGetErrorString(r));
        }
        if (e == hipSuccess) e = hipStreamSynchronize(x->stream);
        if (e == hipSuccess && rc == SPX_OK)
            e = hipMemcpy2D(binv, mb, tmp, (size_t)x->L * 8, mb, (size_t)x->m, hipMemcpyDeviceToHost);
        (void)hipFree(tmp);
        if (rc != SPX_OK) return rc;
        if (e != hipSuccess) return fail(SPX_ERR_HIP, "binv readback: %s", hipGetErrorString(e));
    }
    SPX_TRY(read_state(x));  // drains the stream; y_buf after the flush
    if (x_b) HIP_TRY(hipMemcpy(x_b, x->P.x_b, mb, hipMemcpyDeviceToHost));
    if (b_ixs) HIP_TRY(hipMemcpy(b_ixs, x->P.b_ixs, mb, hipMemcpyDeviceToHost));
    if (y) HIP_TRY(hipMemcpy(y, x->st_host->y_buf ? x->P.y1 : x->P.y0, mb, hipMemcpyDeviceToHost));
    if (c_b) HIP_TRY(hipMemcpy(c_b, x->P.c_B, mb, hipMemcpyDeviceToHost));
    if (status) *status = x->status;
    if (pivots) *pivots = x->pivots;
    return SPX_OK;
}

int spx_reduced_costs(spx_ctx* x, double* e) {
    if (!x || !e) return fail(SPX_ERR_ARG, "NULL argument");
    SPX_TRY(flush(x));
    double* tmp = nullptr;
    HIP_TRY(hipMalloc(reinterpret_cast<void**>(&tmp), (size_t)x->n * 8));
    hipError_t er = launch_reduced_costs(x->P, tmp, x->stream);
    if (er == hipSuccess) er = hipStreamSynchronize(x->stream);
    if (er == hipSuccess) er = hipMemcpy(e, tmp, (size_t)x->n * 8, hipMemcpyDeviceToHost);
    (void)hipFree(tmp);
    if (er != hipSuccess) return fail(SPX_ERR_HIP, "reduced costs: %s", hipGetErrorString(er));
    return SPX_OK;
}

int spx_solve(spx_ctx* x, int64_t max_iter, double* z, int64_t* b_ixs, double* x_b, int32_t* status,
              int64_t* pivots) {
    if (!x) return fail(SPX_ERR_ARG, "ctx is NULL");
    if (max_iter < 0) return fail(SPX_ERR_ARG, "max_iter < 0");
    int64_t chunk = 16;
    while (x->status == SPX_STATUS_MAX_ITER && x->pivots < max_iter) {
        const int64_t k = std::min(chunk, max_iter - x->pivots);
        SPX_TRY(iterate(x, k));
        chunk = std::min<int64_t>(chunk * 2, 2048);
    }
    if (z) SPX_TRY(spx_objective(x, z));
    SPX_TRY(spx_get_state(x, x_b, b_ixs, nullptr, nullptr, nullptr, status, pivots));
    return SPX_OK;
}

int spx_price(spx_ctx* x, int64_t* p, double* min_e, int32_t* optimal) {
    if (!x) return fail(SPX_ERR_ARG, "ctx is NULL");
    if (x->status != SPX_STATUS_MAX_ITER) return fail(SPX_ERR_STATE, "solve already terminated");
    SPX_TRY(set_limit(x, x->pivots + 1));
    const bool fold = fold_due(x);
    if (fold) HIP_TRY(launch_fold(x->P, x->P.win, x->cus, x->stream));
    ++x->n_eager;
    x->n_folds += fold ? 1 : 0;
    HIP_TRY(launch_se_prep(x->P, x->stream));
    SPX_TRY(clear_tickets(x));
    HIP_TRY(launch_price(x->P, x->pcfg, x->stream, nullptr, nullptr));
    const int ps = x->P.pr_stride;
    if (x->use_comm) {
        if (x->mbox_ready) {
            HIP_TRY(launch_exchange(x->P, x->stream));
        } else {
            if (!x->comm_ready) return fail(SPX_ERR_STATE, "nranks > 1 but neither spx_attach_comm nor spx_mbox_attach was called");
            NCCL_TRY(ncclAllGather(x->send, x->recv, sizeof(ArgMinEntry) * ps, ncclUint8, x->comm, x->stream));
        }
    }
    std::vector<ArgMinEntry> cand((size_t)x->opts.nranks * ps);
    HIP_TRY(hipStreamSynchronize(x->stream));
    HIP_TRY(hipMemcpy(cand.data(), x->P.price_in, sizeof(ArgMinEntry) * cand.size(), hipMemcpyDeviceToHost));
    ArgMinEntry best{INFINITY, INT64_MAX};
    int gbest = 0;
    for (int g = 0; g < x->opts.nranks; ++g) {
        const ArgMinEntry& e = cand[(size_t)g * ps];
        if (argmin_better(e.val, e.idx, best.val, best.idx)) {
            best = e;
            gbest = g;
        }
    }
    if (p) *p = (best.idx == INT64_MAX) ? -1 : best.idx;
    double e_enter = best.val;
    if (x->P.devex && x->opts.nranks > 1)  // the winner's record (dvx_payload)
        std::memcpy(&e_enter, &cand[(size_t)gbest * ps + 1 + x->P.win / 2], sizeof(double));
    else if (x->P.devex)
        HIP_TRY(hipMemcpy(&e_enter, x->P.dvx_e, sizeof(double), hipMemcpyDeviceToHost));
    if (min_e) *min_e = e_enter;
    if (optimal) *optimal = no_entering(x->P, best.val, best.idx) ? 1 : 0;
    x->stepped_price = true;
    return SPX_OK;
}

int spx_pivot(spx_ctx* x, int64_t* q, int32_t* status) {
    if (!x) return fail(SPX_ERR_ARG, "ctx is NULL");
    if (!x->stepped_price) return fail(SPX_ERR_STATE, "spx_pivot needs a preceding spx_price");
    x->stepped_price = false;
    HIP_TRY(launch_update(x->P, x->ucfg, x->stream, nullptr, nullptr));
    if (x->P.split_tail) HIP_TRY(launch_tail(x->P, x->ucfg.grid, x->stream));
    SPX_TRY(read_state(x));
    if (q) *q = (x->status == SPX_STATUS_UNBOUNDED) ? -1 : x->st_host->q;
    if (status) *status = x->status;
    return SPX_OK;
}

int spx_dispatch_stats(spx_ctx* x, int64_t out[SPX_DISPATCH_FIELDS]) {
    if (!x || !out) return fail(SPX_ERR_ARG, "NULL argument");
    out[0] = x->n_eager;
    out[1] = x->n_graph_launch;
    out[2] = x->n_graph_pass;
    out[3] = x->n_persist_launch;
    out[4] = x->n_persist_pass;
    out[5] = x->n_folds;
    out[6] = x->P.win ? x->nw : 0;
    out[7] = x->P.win;
    out[8] = x->n_persist_fallback;
    out[9] = x->n_graph_builds;
    return SPX_OK;
}

int spx_prepare(spx_ctx* x) {
    if (!x) return fail(SPX_ERR_ARG, "ctx is NULL");
    if (x->persist) return SPX_OK;  // one launch per window: nothing to capture
    return build_graph(x);
}

int spx_pass_times(spx_ctx* x, double out[3], int64_t* passes) {
    if (!x || !out) return fail(SPX_ERR_ARG, "NULL argument");
    HIP_TRY(hipStreamSynchronize(x->stream));
    double tp = 0.0, tx = 0.0, tu = 0.0;
    for (size_t i = 0; i < x->n_price; ++i) {
        float a = 0.f, b = 0.f;
        HIP_TRY(hipEventElapsedTime(&a, x->ev_price[2 * i], x->ev_price[2 * i + 1]));
        HIP_TRY(hipEventElapsedTime(&b, x->ev_price[2 * i], x->ev_xend[i]));
        tp += a;
        tx += b;
    }
    for (size_t i = 0; i < x->n_update; ++i) {
        float a = 0.f;
        HIP_TRY(hipEventElapsedTime(&a, x->ev_update[2 * i], x->ev_update[2 * i + 1]));
        tu += a;
    }
    out[0] = tp;
    out[1] = tx;
    out[2] = tu;
    if (passes) *passes = (int64_t)x->n_price;
    x->n_price = x->n_update = 0;
    return SPX_OK;
}

int spx_loop_times(spx_ctx* x, double out[SPX_LOOP_FIELDS], int64_t* passes) {
    if (!x || !out) return fail(SPX_ERR_ARG, "NULL argument");
    HIP_TRY(hipStreamSynchronize(x->stream));
    double ms = 0.0;
    int64_t np = 0;
    for (size_t i = 0; i < x->n_loop; ++i) {
        float t = 0.f;
        HIP_TRY(hipEventElapsedTime(&t, x->ev_loop[2 * i], x->ev_loop[2 * i + 1]));
        ms += t;
        np += x->ev_loop_passes[i];
    }
    x->n_loop = 0;
    double fms = 0.0;
    for (size_t i = 0; i < x->n_fold; ++i) {
        float t = 0.f;
        HIP_TRY(hipEventElapsedTime(&t, x->ev_fold[2 * i], x->ev_fold[2 * i + 1]));
        fms += t;
    }
    out[5] = fms;
    out[6] = (double)x->n_fold;
    x->n_fold = 0;
    out[0] = ms;
    out[1] = (double)np;
    out[2] = x->loop_clock[0];
    out[3] = x->loop_clock[1];
    out[4] = x->loop_clock[2];
    if (passes) *passes = x->loop_clock_passes;
    x->loop_clock[0] = x->loop_clock[1] = x->loop_clock[2] = 0.0;
    x->loop_clock_passes = 0;
    return SPX_OK;
}

int spx_kernel_times(spx_ctx* x, double* price_ms, int64_t* np, double* update_ms, int64_t* nu) {
    if (!x) return fail(SPX_ERR_ARG, "ctx is NULL");
    HIP_TRY(hipStreamSynchronize(x->stream));
    double tp = 0.0, tu = 0.0;
    for (size_t i = 0; i < x->n_price; ++i) {
        float ms = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, x->ev_price[2 * i], x->ev_price[2 * i + 1]));
        tp += ms;
    }
    for (size_t i = 0; i < x->n_update; ++i) {
        float ms = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, x->ev_update[2 * i], x->ev_update[2 * i + 1]));
        tu += ms;
    }
    if (price_ms) *price_ms = tp;
    if (update_ms) *update_ms = tu;
    if (np) *np = (int64_t)x->n_price;
    if (nu) *nu = (int64_t)x->n_update;
    x->n_price = x->n_update = 0;
    return SPX_OK;
}

int spx_phase_times(spx_ctx* x, double out[SPX_PHASES]) {
    if (!x || !out) return fail(SPX_ERR_ARG, "NULL argument");
    if (!x->P.stamps) return fail(SPX_ERR_STATE, "context created without SPX_FLAG_STAMPS");
    unsigned long long h[32];
    HIP_TRY(hipStreamSynchronize(x->stream));
    HIP_TRY(hipMemcpy(h, x->P.stamps, sizeof(h), hipMemcpyDeviceToHost));
    for (int k = 0; k < 5; ++k) out[4 + k] = h[8 + k] * 0.01;
    out[9] = h[18] * 0.01;   // update prologue
    out[10] = h[19] * 0.01;  // update drain
    out[11] = h[22] * 0.01;  // price prologue
    out[12] = h[23] * 0.01;  // price drain
    for (int k = 0; k < 5; ++k) out[13 + k] = h[24 + k] * 0.01;  // k_update workgroup 0 marks
    out[0] = h[1] * 0.01;  // 100 MHz ticks -> us
    out[1] = h[2] * 0.01;
    out[2] = h[5] * 0.01;
    out[3] = h[6] * 0.01;
    return reset_stamps(x);
}

int spx_info(spx_ctx* x, int64_t* m, int64_t* n, int64_t* ld, int64_t* local_nb, double* bp, double* bu) {
    if (!x) return fail(SPX_ERR_ARG, "ctx is NULL");
    SPX_TRY(read_state(x));
    if (m) *m = x->m;
    if (n) *n = x->n;
    if (ld) *ld = x->L;
    if (local_nb) *local_nb = x->st_host->nb_count;
    // pricing bytes: the streamed non-basic columns (with P.slack_unit the
    // non-basic slacks of this rank's block are priced without their column)
    int64_t streamed = x->st_host->nb_count;
    if (x->P.slack_unit) {
        std::vector<int64_t> bix((size_t)x->m);
        HIP_TRY(hipMemcpy(bix.data(), x->P.b_ixs, (size_t)x->m * sizeof(int64_t), hipMemcpyDeviceToHost));
        int64_t basic_slacks = 0;
        for (int64_t j : bix) basic_slacks += (j >= x->P.k_lo && j < x->P.k_hi) ? 1 : 0;
        streamed -= (x->P.k_hi - x->P.k_lo) - basic_slacks;
    }
    if (bp) *bp = 8.0 * (double)(x->m + 1) * (double)streamed;
    // update bytes per pivot: B^-1 read + write, or (eta window) the B_w
    // FTRAN stream (its non-unit columns with the compact operand) plus the
    // fold's read + write spread over its KW-1 pivots
    int32_t cols = 0;
    SPX_TRY(spx_ftran_cols(x, &cols));
    const double md = (double)x->m;
    // the fold per window: dense -- B_w read + written; compact (k_cfold) --
    // the operand's columns read, written and scattered into B_w, U read
    const double fold = (x->P.bc && x->P.cfold) ? 8.0 * md * (3.0 * cols + x->P.win) : 16.0 * md * md;
    if (bu) *bu = x->P.win ? 8.0 * md * (double)cols + fold / (x->P.win - 1) : 16.0 * md * md;
    return SPX_OK;
}

int spx_ftran_cols(spx_ctx* x, int32_t* cols) {
    if (!x || !cols) return fail(SPX_ERR_ARG, "NULL argument");
    *cols = (int32_t)x->m;
    if (x->P.win && x->P.bc) {
        HIP_TRY(hipStreamSynchronize(x->stream));
        HIP_TRY(hipMemcpy(cols, x->P.bc_n, sizeof(int32_t), hipMemcpyDeviceToHost));
    }
    return SPX_OK;
}

int spx_config(spx_ctx* x, int32_t out[SPX_CONFIG_FIELDS]) {
    if (!x || !out) return fail(SPX_ERR_ARG, "NULL argument");
    out[0] = x->P.win;
    out[1] = x->pcfg.block;
    out[2] = x->pcfg.grid;
    out[3] = !x->pcfg.lds_y ? 0 : (x->pcfg.wm == 1 ? 2 : 1);
    out[4] = x->ucfg.block;
    out[5] = x->ucfg.rows;
    out[6] = x->ucfg.grid;
    out[7] = x->batch;
    out[8] = x->persist ? 1 : 0;
    out[9] = x->persist ? x->lcfg.block : 0;
    out[10] = x->P.tab;
    out[11] = x->persist ? x->lcfg.grid : 0;
    out[12] = x->defer_tail ? 1 : 0;
    out[13] = (x->P.bc && x->P.cfold) ? 1 : 0;
    out[14] = (x->P.bc && x->ucfg.rows == 1 && x->ucfg.bc_entry) ? x->ucfg.bc_entry : 0;
    out[15] = (x->mbox_ready && x->mbox_fused) ? 1 : 0;
    return SPX_OK;
}

int spx_shard_range(int64_t m, int64_t n, int32_t rank, int32_t nranks, int64_t out[4]) {
    if (!out || m <= 0 || n < m || nranks < 1 || rank < 0 || rank >= nranks)
        return fail(SPX_ERR_ARG, "bad shard arguments");
    shard_range(m, n, rank, nranks, out);
    return SPX_OK;
}

int spx_minloc_merge(const double* vals, const int64_t* idx, int32_t count, double* best_val, int64_t* best_idx) {
    if ((count > 0 && (!vals || !idx)) || !best_val || !best_idx) return fail(SPX_ERR_ARG, "NULL argument");
    ArgMinEntry b{INFINITY, INT64_MAX};
    for (int32_t g = 0; g < count; ++g)
        if (argmin_better(vals[g], idx[g], b.val, b.idx)) b = ArgMinEntry{vals[g], idx[g]};
    *best_val = b.val;
    *best_idx = b.idx;
    return SPX_OK;
}

}  // extern "C"

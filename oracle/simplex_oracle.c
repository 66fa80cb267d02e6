/*
 * simplex_oracle.c — TEST INFRASTRUCTURE ONLY (see simplex_oracle.h).
 *
 * fp64 CPU restatement of the reference's revised-simplex loop.  Every step
 * cites the reference line it restates (src/v4_cub_reduction.cu unless noted).
 * It keeps the reference's data layout (A and B^-1 column-major, R2C at
 * v4:59-60), its reduction semantics (first index on ties, as CUB ArgMin at
 * v4:294,324) and its update formulas, with the intended init semantics
 * (the reference's init_I / init_D_from_A grids and the n-m copy at v4:277
 * are buggy beyond m,n <= 16).
 *
 * Parallel loops (OpenMP) only split independent outputs, so results do not
 * depend on the thread count.
 */
#include "simplex_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#ifdef _OPENMP
#include <omp.h>
#endif

uint64_t orc_splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

double orc_uniform(uint64_t seed, uint64_t stream, uint64_t idx) {
    uint64_t key = (seed * 0x9E3779B97F4A7C15ULL) ^ (stream << 56) ^ idx;
    return (double)(orc_splitmix64(key) >> 11) * 0x1.0p-53;
}

void orc_generate(int64_t m, int64_t n, uint64_t seed,
                  double* A, double* b, double* c) {
    const int64_t ns = n - m; /* structural columns; the last m are slacks */
#pragma omp parallel for schedule(static)
    for (int64_t j = 0; j < n; ++j) {
        double* col = A + j * m;
        if (j < ns) {
            for (int64_t i = 0; i < m; ++i)
                col[i] = orc_uniform(seed, 1, (uint64_t)(i + j * m));
        } else {
            for (int64_t i = 0; i < m; ++i) col[i] = 0.0;
            col[j - ns] = 1.0;
        }
    }
    const double scale = (double)ns / 4.0;
    for (int64_t i = 0; i < m; ++i)
        b[i] = scale * (1.0 + orc_uniform(seed, 2, (uint64_t)i));
    for (int64_t j = 0; j < n; ++j)
        c[j] = (j < ns) ? orc_uniform(seed, 3, (uint64_t)j) : 0.0;
}

int orc_max_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

static void set_threads(int threads) {
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#else
    (void)threads;
#endif
}

/* e = [1 y] * [-c; A]  (v4:288-290, D built at v4:278-279): -c_j first, then
 * y_i * A_ij accumulated down the column. */
void orc_price(int64_t m, int64_t n, const double* A, const double* c,
               const double* y, double* e, int threads) {
    set_threads(threads);
#pragma omp parallel for schedule(static)
    for (int64_t j = 0; j < n; ++j) {
        const double* col = A + j * m;
        double s = -c[j];
        for (int64_t i = 0; i < m; ++i) s += y[i] * col[i];
        e[j] = s;
    }
}

/* cub::DeviceReduce::ArgMin semantics (v4:294,324): smallest value, first
 * index on ties. */
static int64_t argmin_first(const double* v, int64_t len, double* minval) {
    int64_t best = 0;
    double bv = v[0];
    for (int64_t k = 1; k < len; ++k)
        if (v[k] < bv) { bv = v[k]; best = k; }
    *minval = bv;
    return best;
}

typedef struct {
    int64_t m, n;
    double *Binv, *c_b, *x_b, *y, *e, *alpha, *theta, *E, *r;
    int64_t* b_ixs;
} orc_state;

static int state_init(orc_state* s, int64_t m, int64_t n, const double* b,
                      const double* c) {
    memset(s, 0, sizeof(*s));
    s->m = m; s->n = n;
    s->Binv = (double*)malloc(sizeof(double) * (size_t)(m * m));
    s->c_b = (double*)malloc(sizeof(double) * (size_t)m);
    s->x_b = (double*)malloc(sizeof(double) * (size_t)m);
    s->y = (double*)malloc(sizeof(double) * (size_t)m);
    s->e = (double*)malloc(sizeof(double) * (size_t)n);
    s->alpha = (double*)malloc(sizeof(double) * (size_t)m);
    s->theta = (double*)malloc(sizeof(double) * (size_t)m);
    s->E = (double*)malloc(sizeof(double) * (size_t)m);
    s->r = (double*)malloc(sizeof(double) * (size_t)m);
    s->b_ixs = (int64_t*)malloc(sizeof(int64_t) * (size_t)m);
    if (!s->Binv || !s->c_b || !s->x_b || !s->y || !s->e || !s->alpha ||
        !s->theta || !s->E || !s->r || !s->b_ixs)
        return -1;
    /* init_I (v4:182-188, launch :272): B^-1 = I_m */
#pragma omp parallel for schedule(static)
    for (int64_t k = 0; k < m; ++k)
        for (int64_t i = 0; i < m; ++i) s->Binv[i + k * m] = (i == k) ? 1.0 : 0.0;
    for (int64_t i = 0; i < m; ++i) {
        s->c_b[i] = c[n - m + i];  /* v4:273 */
        s->x_b[i] = b[i];          /* v4:274 */
        s->b_ixs[i] = n - m + i;   /* init_b_ixs v4:190-193 */
        s->y[i] = s->c_b[i];       /* y_aug = [1, c_B] (v4:276-277, m elements) */
    }
    return 0;
}

static void state_free(orc_state* s) {
    free(s->Binv); free(s->c_b); free(s->x_b); free(s->y); free(s->e);
    free(s->alpha); free(s->theta); free(s->E); free(s->r); free(s->b_ixs);
}

/* One pass of the do-loop body (v4:286-357).  Returns ORC_MAX_ITER when a
 * pivot was made (loop continues), otherwise the terminating status. */
static int one_pass(orc_state* s, const double* A, const double* b,
                    const double* c, double eps, int64_t* p_out, int64_t* q_out) {
    const int64_t m = s->m, n = s->n;
    double min_val;

    /* pricing GEMM + entering ArgMin (v4:289-302) */
    orc_price(m, n, A, c, s->y, s->e, 0);
    const int64_t p = argmin_first(s->e, n, &min_val);
    if (min_val >= -eps) return ORC_OPTIMUM_FOUND;

    /* FTRAN: alpha = B_inv * A_p (cublasSgemv, v4:307-308) */
    const double* Ap = A + p * m;
    const int64_t CH = 256;
#pragma omp parallel for schedule(static)
    for (int64_t i0 = 0; i0 < m; i0 += CH) {
        const int64_t i1 = (i0 + CH < m) ? i0 + CH : m;
        double acc[256];
        for (int64_t i = i0; i < i1; ++i) acc[i - i0] = 0.0;
        for (int64_t k = 0; k < m; ++k) {
            const double a = Ap[k];
            const double* colk = s->Binv + k * m;
            for (int64_t i = i0; i < i1; ++i) acc[i - i0] += colk[i] * a;
        }
        for (int64_t i = i0; i < i1; ++i) s->alpha[i] = acc[i - i0];
    }

    /* compute_theta (v4:199-208): strict alpha_i > 0, no pivot tolerance */
    int64_t non_pos = 0;
    for (int64_t i = 0; i < m; ++i) {
        const int flag = s->alpha[i] > 0;
        s->theta[i] = flag ? s->x_b[i] / s->alpha[i] : INFINITY;
        non_pos += !flag;
    }
    if (non_pos == m) return ORC_UNBOUNDED; /* v4:317-322 */

    /* leaving ArgMin (v4:324-325) */
    const int64_t q = argmin_first(s->theta, m, &min_val);

    /* r = B_inv[q,:] (cublasScopy, v4:331); E_q (compute_E_q v4:210-215) */
    for (int64_t k = 0; k < m; ++k) s->r[k] = s->Binv[q + k * m];
    const double aq = s->alpha[q];
    for (int64_t i = 0; i < m; ++i)
        s->E[i] = (i != q) ? (-s->alpha[i] / aq) : (1.0 / aq - 1.0);

    /* rank-1 update B_inv += E_q r^T (cublasSger, v4:333) */
#pragma omp parallel for schedule(static)
    for (int64_t k = 0; k < m; ++k) {
        const double rk = s->r[k];
        double* colk = s->Binv + k * m;
        for (int64_t i = 0; i < m; ++i) colk[i] += s->E[i] * rk;
    }

    /* basis bookkeeping (v4:339-342) */
    const double c_bq = s->c_b[q];
    const double c_p = c[p];
    s->c_b[q] = c_p;
    s->b_ixs[q] = p;

    /* x_b += (r.b) E_q (cublasSdot + Saxpy, v4:347-348) */
    double sx = 0.0;
    for (int64_t k = 0; k < m; ++k) sx += s->r[k] * b[k];
    for (int64_t i = 0; i < m; ++i) s->x_b[i] += sx * s->E[i];

    /* y += (c_B.E_q + c_p - c_Bq) r (Sdot, compute_scalar, Saxpy, v4:354-356;
     * compute_scalar v4:195-197) */
    double sy = 0.0;
    for (int64_t i = 0; i < m; ++i) sy += s->c_b[i] * s->E[i];
    sy += c_p - c_bq;
    for (int64_t k = 0; k < m; ++k) s->y[k] += sy * s->r[k];

    *p_out = p;
    *q_out = q;
    return ORC_MAX_ITER;
}

int orc_solve(int64_t m, int64_t n, const double* A, const double* b,
              const double* c, int64_t max_iter, double eps, int threads,
              double* z, double* x_b, int64_t* b_ixs, int64_t* pivots,
              int64_t* trace_p, int64_t* trace_q, int64_t trace_cap,
              double* y_out, double* binv_out) {
    if (m <= 0 || n < m) return -1; /* CLI rejects m > n (v4:402-405) */
    set_threads(threads);
    orc_state s;
    if (state_init(&s, m, n, b, c) != 0) { state_free(&s); return -2; }

    int status = ORC_MAX_ITER;
    int64_t i = 0;
    if (max_iter > 0) {
        do { /* v4:286-359 */
            int64_t p = -1, q = -1;
            status = one_pass(&s, A, b, c, eps, &p, &q);
            if (status != ORC_MAX_ITER) break;
            if (i < trace_cap) {
                if (trace_p) trace_p[i] = p;
                if (trace_q) trace_q[i] = q;
            }
        } while (++i < max_iter);
    }

    if (z) { /* z = c_B . x_b (cublasSdot, v4:365) */
        double acc = 0.0;
        for (int64_t k = 0; k < m; ++k) acc += s.c_b[k] * s.x_b[k];
        *z = acc;
    }
    if (x_b) memcpy(x_b, s.x_b, sizeof(double) * (size_t)m);
    if (b_ixs) memcpy(b_ixs, s.b_ixs, sizeof(int64_t) * (size_t)m);
    if (pivots) *pivots = i;
    if (y_out) memcpy(y_out, s.y, sizeof(double) * (size_t)m);
    if (binv_out)
        for (int64_t r = 0; r < m; ++r)
            for (int64_t k = 0; k < m; ++k) binv_out[r * m + k] = s.Binv[r + k * m];
    state_free(&s);
    return status;
}

double orc_time_iterations(int64_t m, int64_t n, const double* A,
                           const double* b, const double* c, int64_t iters,
                           int threads, int64_t* done) {
    set_threads(threads);
    orc_state s;
    if (state_init(&s, m, n, b, c) != 0) { state_free(&s); return -1.0; }
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    int64_t k = 0;
    for (; k < iters; ++k) {
        int64_t p, q;
        if (one_pass(&s, A, b, c, -1.0e300, &p, &q) != ORC_MAX_ITER) break;
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    if (done) *done = k;
    state_free(&s);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

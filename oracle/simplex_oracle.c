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
    /* Devex pricing (orc_opts.pricing = 1): reference weights, basic mask and
     * the last pivot's data (r above is its pivot row of B^-1) */
    double* w;
    char* basic;
    int dvx_pend;
    double dvx_aq, dvx_wp;
    int64_t dvx_leave;
    /* steepest edge (orc_opts.pricing = 2): v = B^-T alpha of the last pivot
     * (B^-1 before it) and gamma_p = 1 + ||alpha||^2, exact */
    double* se_v;
    double se_gp;
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
    s->w = (double*)malloc(sizeof(double) * (size_t)n);
    s->basic = (char*)calloc((size_t)n, 1);
    s->se_v = (double*)malloc(sizeof(double) * (size_t)m);
    if (!s->Binv || !s->c_b || !s->x_b || !s->y || !s->e || !s->alpha ||
        !s->theta || !s->E || !s->r || !s->b_ixs || !s->w || !s->basic || !s->se_v)
        return -1;
    for (int64_t j = 0; j < n; ++j) s->w[j] = 1.0;
    for (int64_t j = n - m; j < n; ++j) s->basic[j] = 1;
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
    free(s->w); free(s->basic); free(s->se_v);
}

/* Steepest-edge reference weights at the slack basis (B = I):
 * gamma_j = 1 + ||A_j||^2, k ascending, for the structural columns (the slack
 * columns are basic; their weights are set when they leave). */
static void se_init(orc_state* s, const double* A) {
    const int64_t m = s->m, n = s->n;
#pragma omp parallel for schedule(static)
    for (int64_t j = 0; j < n - m; ++j) {
        const double* col = A + j * m;
        double a = 0.0;
        for (int64_t k = 0; k < m; ++k) a = fma(col[k], col[k], a);
        s->w[j] = 1.0 + a;
    }
}

/* One pass of the do-loop body (v4:286-357).  Returns ORC_MAX_ITER when a
 * pivot was made (loop continues), otherwise the terminating status. */
/* Leaving row under the SPX_RATIO_* rules (include/simplex.h).  rule 0 is the
 * reference: compute_theta (v4:199-208, strict alpha_i > 0, no filter) + the
 * first-index ArgMin (v4:324-325).  Returns -1 when no row is a candidate
 * (Unbounded, v4:317-322). */
static int64_t ratio_test(const orc_state* s, int rule, double piv_tol,
                          double feas_tol) {
    const int64_t m = s->m;
    const double pt = rule == 0 ? 0.0 : piv_tol;
    int64_t non_pos = 0;
    for (int64_t i = 0; i < m; ++i) {
        const double a = s->alpha[i], xb = s->x_b[i];
        const int flag = a > pt;
        double th = INFINITY;
        if (flag) {
            if (rule == 0) th = xb / a;
            else {
                const double xc = xb > 0.0 ? xb : 0.0;
                th = rule == 2 ? (xc + feas_tol) / a : xc / a;
            }
        }
        s->theta[i] = th;
        non_pos += !flag;
    }
    if (non_pos == m) return -1;
    double thmax;
    int64_t q = argmin_first(s->theta, m, &thmax);
    if (rule == 2) {
        /* Harris second pass: largest alpha_i among rows whose clamped ratio
         * is within theta_max, first index on ties */
        double best = -INFINITY;
        q = -1;
        for (int64_t i = 0; i < m; ++i) {
            const double a = s->alpha[i];
            if (!(a > pt)) continue;
            const double xc = s->x_b[i] > 0.0 ? s->x_b[i] : 0.0;
            if (xc / a <= thmax && a > best) { best = a; q = i; }
        }
    }
    return q;
}

/* Devex entering column (README.md:16-17 "steepest edge"; the reference
 * framework of Forrest & Goldfarb's Devex).  First the weights of the
 * non-basic columns take the last pivot into account: with alpha_rj = r.A_j
 * its pivot-row entries (r = row q of B^-1 before that pivot), alpha_q its
 * pivot and w_p the entering column's weight,
 *   w_j = max(w_j, (alpha_rj / alpha_q)^2 w_p),  w_leave = max(w_p / alpha_q^2, 1).
 * Then p = argmin over non-basic j with e_j < -eps of -(e_j^2) / w_j (first
 * index on ties); -1 when there is none (optimal). */
static int64_t devex_choose(orc_state* s, const double* A, double eps) {
    const int64_t m = s->m, n = s->n;
    if (s->dvx_pend) {
        const double aq = s->dvx_aq, wp = s->dvx_wp;
#pragma omp parallel for schedule(static)
        for (int64_t j = 0; j < n; ++j) {
            if (s->basic[j]) continue;
            if (j == s->dvx_leave) {
                const double v = wp / (aq * aq);
                s->w[j] = v > 1.0 ? v : 1.0;
                continue;
            }
            const double* col = A + j * m;
            double a = 0.0;
            for (int64_t k = 0; k < m; ++k) a += s->r[k] * col[k];
            const double g = a / aq;
            const double v = g * g * wp;
            if (v > s->w[j]) s->w[j] = v;
        }
    }
    int64_t p = -1;
    double best = INFINITY;
    for (int64_t j = 0; j < n; ++j) {
        if (s->basic[j] || !(s->e[j] < -eps)) continue;
        const double key = -(s->e[j] * s->e[j]) / s->w[j];
        if (key < best) { best = key; p = j; }
    }
    return p;
}

/* Steepest-edge entering column (README.md:16-17 "Steepest edge with a
 * recurrence"): exact reference weights gamma_j = 1 + ||B^-1 A_j||^2, kept by
 * Goldfarb & Reid's recurrence.  After a pivot with entering p, leaving row q,
 * alpha = B^-1 A_p, alpha_q = alpha[q], pivot row alpha_rj = r.A_j (r = row q
 * of B^-1 before the pivot), v = B^-T alpha and gamma_p = 1 + ||alpha||^2
 * (both before the pivot), every non-basic column j but the leaving one takes
 *   g = alpha_rj / alpha_q,  d_j = v.A_j,
 *   gamma_j = max(gamma_j - 2 g d_j + g^2 gamma_p, 1 + g^2)
 *           = fmax(fma(g*g, gamma_p, fma(-2*g, d_j, gamma_j)), fma(g, g, 1)),
 * and the leaving column gamma = max(gamma_p / alpha_q^2, 1).  Then p =
 * argmin over non-basic j with e_j < -eps of -(e_j^2) / gamma_j (first index
 * on ties); -1 when there is none (optimal).  Weights start at the slack basis
 * (se_init) and persist across reinversions. */
static void se_apply_pending(orc_state* s, const double* A) {
    const int64_t m = s->m, n = s->n;
    if (s->dvx_pend) {
        const double aq = s->dvx_aq, gp = s->se_gp;
#pragma omp parallel for schedule(static)
        for (int64_t j = 0; j < n; ++j) {
            if (s->basic[j]) continue;
            if (j == s->dvx_leave) {
                const double v = gp / (aq * aq);
                s->w[j] = v > 1.0 ? v : 1.0;
                continue;
            }
            const double* col = A + j * m;
            double a = 0.0, d = 0.0;
            for (int64_t k = 0; k < m; ++k) {
                a = fma(s->r[k], col[k], a);
                d = fma(s->se_v[k], col[k], d);
            }
            const double g = a / aq;
            const double t = fma(g * g, gp, fma(-2.0 * g, d, s->w[j]));
            const double lo = fma(g, g, 1.0);
            s->w[j] = t > lo ? t : lo;
        }
        s->dvx_pend = 0;
    }
}

static int64_t se_choose(orc_state* s, const double* A, double eps) {
    const int64_t n = s->n;
    se_apply_pending(s, A);
    int64_t p = -1;
    double best = INFINITY;
    for (int64_t j = 0; j < n; ++j) {
        if (s->basic[j] || !(s->e[j] < -eps)) continue;
        const double key = -(s->e[j] * s->e[j]) / s->w[j];
        if (key < best) { best = key; p = j; }
    }
    return p;
}

static int one_pass(orc_state* s, const double* A, const double* b,
                    const double* c, double eps, int rule, double piv_tol,
                    double feas_tol, int pricing, int64_t* p_out, int64_t* q_out) {
    const int64_t m = s->m, n = s->n;
    double min_val;

    /* pricing GEMM + entering ArgMin (v4:289-302), or Devex */
    orc_price(m, n, A, c, s->y, s->e, 0);
    int64_t p;
    if (pricing == 1 || pricing == 2) {
        p = pricing == 1 ? devex_choose(s, A, eps) : se_choose(s, A, eps);
        if (p < 0) return ORC_OPTIMUM_FOUND;
    } else {
        p = argmin_first(s->e, n, &min_val);
        if (min_val >= -eps) return ORC_OPTIMUM_FOUND;
    }

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

    /* compute_theta + leaving ArgMin (v4:199-208,317-325), or a variant */
    const int64_t q = ratio_test(s, rule, piv_tol, feas_tol);
    if (q < 0) return ORC_UNBOUNDED;

    /* steepest edge: v = B^-T alpha and gamma_p = 1 + ||alpha||^2 with the
     * B^-1 of before this pivot (se_choose applies them at the next pass) */
    if (pricing == 2) {
        double a2 = 0.0;
        for (int64_t i = 0; i < m; ++i) a2 = fma(s->alpha[i], s->alpha[i], a2);
        s->se_gp = 1.0 + a2;
#pragma omp parallel for schedule(static)
        for (int64_t k = 0; k < m; ++k) {
            const double* colk = s->Binv + k * m;
            double v = 0.0;
            for (int64_t i = 0; i < m; ++i) v = fma(colk[i], s->alpha[i], v);
            s->se_v[k] = v;
        }
    }

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
    s->dvx_leave = s->b_ixs[q];
    s->basic[s->dvx_leave] = 0;
    s->basic[p] = 1;
    s->dvx_pend = 1;
    s->dvx_aq = aq;
    s->dvx_wp = s->w[p];
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

/* Pivot-in reinversion (orc_reinvert).  Binv_cm: m x m COLUMN-major output
 * (the oracle's layout), already in the given basis order. */
static int reinvert_core(int64_t m, int64_t n, const double* A,
                         const int64_t* basis, double* Binv_cm) {
    const int64_t ns = n - m;
    double* X = (double*)malloc(sizeof(double) * (size_t)(m * m)); /* col-major */
    double* alpha = (double*)malloc(sizeof(double) * (size_t)m);
    double* eta = (double*)malloc(sizeof(double) * (size_t)m);
    double* xq = (double*)malloc(sizeof(double) * (size_t)m);
    int64_t* owner = (int64_t*)malloc(sizeof(int64_t) * (size_t)m); /* row -> basis position */
    char* seen = (char*)calloc((size_t)n, 1);
    int rc = 0;
    if (!X || !alpha || !eta || !xq || !owner || !seen) { rc = -2; goto out; }
    for (int64_t k = 0; k < m; ++k) {
        if (basis[k] < 0 || basis[k] >= n || seen[basis[k]]) { rc = -1; goto out; }
        seen[basis[k]] = 1;
    }
#pragma omp parallel for schedule(static)
    for (int64_t k = 0; k < m; ++k)
        for (int64_t i = 0; i < m; ++i) X[i + k * m] = (i == k) ? 1.0 : 0.0;
    for (int64_t i = 0; i < m; ++i) owner[i] = -1;
    for (int64_t k = 0; k < m; ++k) /* slack columns keep their rows */
        if (basis[k] >= ns) owner[basis[k] - ns] = k;
    for (int64_t k = 0; k < m; ++k) {
        const int64_t j = basis[k];
        if (j >= ns) continue;
        const double* Aj = A + j * m;
        /* alpha = X A_j (FTRAN) */
#pragma omp parallel for schedule(static)
        for (int64_t i = 0; i < m; ++i) {
            double acc = 0.0;
            for (int64_t l = 0; l < m; ++l) acc += X[i + l * m] * Aj[l];
            alpha[i] = acc;
        }
        double amax = 0.0, best = -1.0;
        int64_t q = -1;
        for (int64_t i = 0; i < m; ++i) {
            const double v = fabs(alpha[i]);
            if (v > amax) amax = v;
            if (owner[i] < 0 && v > best) { best = v; q = i; }
        }
        if (q < 0 || !(best > 1e-11 * amax)) { rc = -7; goto out; }
        const double aq = alpha[q];
        for (int64_t i = 0; i < m; ++i) eta[i] = (i != q) ? -alpha[i] / aq : 1.0 / aq - 1.0;
        for (int64_t l = 0; l < m; ++l) xq[l] = X[q + l * m];
#pragma omp parallel for schedule(static)
        for (int64_t l = 0; l < m; ++l) {
            const double r = xq[l];
            double* col = X + l * m;
            for (int64_t i = 0; i < m; ++i) col[i] += eta[i] * r;
        }
        owner[q] = k;
    }
    /* B^-1[k,:] = X[row owned by k,:] */
    for (int64_t i = 0; i < m; ++i) {
        const int64_t k = owner[i];
        for (int64_t l = 0; l < m; ++l) Binv_cm[k + l * m] = X[i + l * m];
    }
out:
    free(X); free(alpha); free(eta); free(xq); free(owner); free(seen);
    return rc;
}

/* x_b = B^-1 b and y = c_B B^-1 from a column-major B^-1 (the v2 formulas,
 * v2_quadratic_B_inv.cu:337-338,396-397). */
static void basis_vectors(int64_t m, const double* Binv_cm, const double* b,
                          const double* c_b, double* x_b, double* y) {
    for (int64_t i = 0; i < m; ++i) x_b[i] = 0.0;
    for (int64_t l = 0; l < m; ++l) {
        const double* col = Binv_cm + l * m;
        for (int64_t i = 0; i < m; ++i) x_b[i] += col[i] * b[l];
    }
#pragma omp parallel for schedule(static)
    for (int64_t l = 0; l < m; ++l) {
        const double* col = Binv_cm + l * m;
        double acc = 0.0;
        for (int64_t i = 0; i < m; ++i) acc += c_b[i] * col[i];
        y[l] = acc;
    }
}

int orc_reinvert(int64_t m, int64_t n, const double* A, const double* b,
                 const double* c, const int64_t* basis, int threads,
                 double* binv_out, double* x_b, double* y) {
    if (m <= 0 || n < m) return -1;
    set_threads(threads);
    double* Bi = (double*)malloc(sizeof(double) * (size_t)(m * m));
    double* cb = (double*)malloc(sizeof(double) * (size_t)m);
    double* xb = (double*)malloc(sizeof(double) * (size_t)m);
    double* yy = (double*)malloc(sizeof(double) * (size_t)m);
    int rc = (Bi && cb && xb && yy) ? reinvert_core(m, n, A, basis, Bi) : -2;
    if (rc == 0) {
        for (int64_t k = 0; k < m; ++k) cb[k] = c[basis[k]];
        basis_vectors(m, Bi, b, cb, xb, yy);
        if (x_b) memcpy(x_b, xb, sizeof(double) * (size_t)m);
        if (y) memcpy(y, yy, sizeof(double) * (size_t)m);
        if (binv_out)
            for (int64_t r = 0; r < m; ++r)
                for (int64_t k = 0; k < m; ++k) binv_out[r * m + k] = Bi[r + k * m];
    }
    free(Bi); free(cb); free(xb); free(yy);
    return rc;
}

void orc_default_opts(orc_opts* o) {
    o->max_iter = (int64_t)1 << 40;
    o->eps = 1e-7;
    o->threads = 0;
    o->ratio = 0;
    o->piv_tol = 1e-9;
    o->feas_tol = 1e-9;
    o->refactor_every = 0;
    o->pricing = 0;
    o->w_out = NULL;
}

int orc_solve_ex(int64_t m, int64_t n, const double* A, const double* b,
                 const double* c, const orc_opts* o, double* z, double* x_b,
                 int64_t* b_ixs, int64_t* pivots, int64_t* trace_p,
                 int64_t* trace_q, int64_t trace_cap, double* y_out,
                 double* binv_out) {
    if (m <= 0 || n < m) return -1; /* CLI rejects m > n (v4:402-405) */
    set_threads(o->threads);
    orc_state s;
    if (state_init(&s, m, n, b, c) != 0) { state_free(&s); return -2; }
    if (o->pricing == 2) se_init(&s, A);

    int status = ORC_MAX_ITER;
    int64_t i = 0;
    if (o->max_iter > 0) {
        do { /* v4:286-359 */
            int64_t p = -1, q = -1;
            status = one_pass(&s, A, b, c, o->eps, o->ratio, o->piv_tol, o->feas_tol, o->pricing, &p, &q);
            if (status != ORC_MAX_ITER) break;
            if (i < trace_cap) {
                if (trace_p) trace_p[i] = p;
                if (trace_q) trace_q[i] = q;
            }
            if (o->refactor_every > 0 && (i + 1) % o->refactor_every == 0) {
                const int rc = reinvert_core(m, n, A, s.b_ixs, s.Binv);
                if (rc != 0) { state_free(&s); return rc; }
                basis_vectors(m, s.Binv, b, s.c_b, s.x_b, s.y);
            }
        } while (++i < o->max_iter);
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
    if (o->w_out) {  /* the current weights: the last pivot's update applied */
        if (o->pricing == 2) se_apply_pending(&s, A);
        memcpy(o->w_out, s.w, sizeof(double) * (size_t)n);
    }
    state_free(&s);
    return status;
}

int orc_solve(int64_t m, int64_t n, const double* A, const double* b,
              const double* c, int64_t max_iter, double eps, int threads,
              double* z, double* x_b, int64_t* b_ixs, int64_t* pivots,
              int64_t* trace_p, int64_t* trace_q, int64_t trace_cap,
              double* y_out, double* binv_out) {
    orc_opts o;
    orc_default_opts(&o);
    o.max_iter = max_iter;
    o.eps = eps;
    o.threads = threads;
    return orc_solve_ex(m, n, A, b, c, &o, z, x_b, b_ixs, pivots, trace_p,
                        trace_q, trace_cap, y_out, binv_out);
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
        if (one_pass(&s, A, b, c, -1.0e300, 0, 0.0, 0.0, 0, &p, &q) != ORC_MAX_ITER) break;
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    if (done) *done = k;
    state_free(&s);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

/* slq_ref.c -- CPU oracle / CPU baseline for the probe-Lanczos trace path.
 *
 * TEST INFRASTRUCTURE ONLY: loaded by tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py (kind "port").  The product never links it.
 *
 * Plain-C restatement of the reference's single-vector Lanczos recurrence as
 * the north star composes it (SURVEY.md §8a rows a4 + a10):
 *   - start:   v1 = z/||z||                     (lanczos_krylov.m:48, qr(b,0))
 *   - step:    w = A v_j                        (lanczos_krylov.m:81)
 *              CGS2 against the 2-vector window (lanczos_krylov.m:88,109-115)
 *              beta = ||w||, v_{j+1} = w/beta    (lanczos_krylov.m:90)
 *              lucky breakdown if beta < 1e-8    (lanczos_krylov.m:91-93)
 *   - T_m = (H + H')/2 of the m x m projected block (trace_fun_update.m:78-81)
 *   - z' f(A) z ~= ||z||^2 sum_k tau_k^2 f(theta_k)   (Gauss quadrature)
 * Probes are the build-defined splitmix64 Rademacher stream,
 * identical to oracle/krylov_oracle.py:rademacher and the HIP generator.
 * OpenMP parallelises over probes; each probe runs a scalar CSR SpMV.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <float.h>
#ifdef _OPENMP
#include <omp.h>
#endif

static inline uint64_t sm64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

double slq_ref_rademacher(uint64_t seed, uint64_t probe, uint64_t row) {
    uint64_t key = sm64(sm64(seed) + probe);
    return (sm64(key + row) >> 63) ? -1.0 : 1.0;
}

static double fscalar(int fun, double x) {
    switch (fun) {
    case 0: return exp(x);
    case 1: return sinh(x);
    case 2: return cosh(x);
    case 3: return sin(x);
    case 4: return cos(x);
    case 5: return log(x);
    case 6: return sqrt(x);
    default: return NAN;
    }
}

/* Implicit-shift QL on a symmetric tridiagonal (d[0..m-1], e[0..m-2]).
 * Source: EISPACK IMTQL2 / TQL2 (public domain; Bowdler, Martin, Reinsch &
 * Wilkinson, Numer. Math. 11 (1968), Handbook vol. II contribution II/3),
 * rotating only the first row of the eigenvector matrix (Golub & Welsch 1969).
 * On exit d holds the eigenvalues and z the FIRST components of the
 * normalised eigenvectors (only row 0 of the eigenvector matrix is rotated). */
static void tql_first_row(int m, double *d, const double *e_in, double *z) {
    double e[256];
    for (int i = 0; i < m - 1; ++i) e[i] = e_in[i];
    e[m - 1] = 0.0;
    for (int i = 0; i < m; ++i) z[i] = (i == 0) ? 1.0 : 0.0;
    for (int l = 0; l < m; ++l) {
        int iter = 0, mm;
        for (;;) {
            for (mm = l; mm < m - 1; ++mm) {
                double dd = fabs(d[mm]) + fabs(d[mm + 1]);
                if (fabs(e[mm]) <= DBL_EPSILON * dd) break;
            }
            if (mm == l) break;
            if (iter++ == 100) break;
            double g = (d[l + 1] - d[l]) / (2.0 * e[l]);
            double r = hypot(g, 1.0);
            g = d[mm] - d[l] + e[l] / (g + copysign(r, g));
            double s = 1.0, c = 1.0, p = 0.0;
            int i, early = 0;
            for (i = mm - 1; i >= l; --i) {
                double f = s * e[i], b = c * e[i];
                r = hypot(f, g);
                e[i + 1] = r;
                if (r == 0.0) { d[i + 1] -= p; e[mm] = 0.0; early = 1; break; }
                s = f / r; c = g / r;
                g = d[i + 1] - p;
                r = (d[i] - g) * s + 2.0 * c * b;
                p = s * r;
                d[i + 1] = g + p;
                g = c * r - b;
                double zf = z[i + 1];
                z[i + 1] = s * z[i] + c * zf;
                z[i] = c * z[i] - s * zf;
            }
            if (early) continue;
            d[l] -= p; e[l] = g; e[mm] = 0.0;
        }
    }
}

double slq_ref_tridiag_quad(int m, const double *alpha, const double *off, int fun) {
    double d[256], z[256];
    if (m <= 0) return 0.0;
    if (m > 256) m = 256;
    for (int i = 0; i < m; ++i) d[i] = alpha[i];
    tql_first_row(m, d, off, z);
    double q = 0.0;
    for (int i = 0; i < m; ++i) q += z[i] * z[i] * fscalar(fun, d[i]);
    return q;
}

static void spmv(int64_t n, const int64_t *rp, const int32_t *ci, const double *va,
                 const double *x, double *y) {
    for (int64_t i = 0; i < n; ++i) {
        double acc = 0.0;
        for (int64_t k = rp[i]; k < rp[i + 1]; ++k) acc += va[k] * x[ci[k]];
        y[i] = acc;
    }
}

/* One probe: m-step Lanczos (CGS2 window) -> alpha[0..m'-1], off[0..m'-2].
 * Returns m' (<= m). */
int slq_ref_lanczos(int64_t n, const int64_t *rp, const int32_t *ci, const double *va,
                    const double *z, int m, double *alpha, double *off) {
    double *v0 = (double *)calloc((size_t)n, sizeof(double));
    double *v1 = (double *)malloc((size_t)n * sizeof(double));
    double *w = (double *)malloc((size_t)n * sizeof(double));
    double up[256];  /* H(j-1,j): CGS coefficient on v_{j-1} */
    double low[256]; /* H(j+1,j): QR factor */
    double nz = 0.0;
    for (int64_t i = 0; i < n; ++i) nz += z[i] * z[i];
    nz = sqrt(nz);
    for (int64_t i = 0; i < n; ++i) v1[i] = z[i] / nz;
    int have_prev = 0, steps = 0;
    for (int j = 0; j < m; ++j) {
        spmv(n, rp, ci, va, v1, w);
        double h0 = 0.0, h1 = 0.0;
        for (int pass = 0; pass < 2; ++pass) {           /* CGS2: lanczos_krylov.m:109-115 */
            double g0 = 0.0, g1 = 0.0;
            for (int64_t i = 0; i < n; ++i) { g0 += v0[i] * w[i]; g1 += v1[i] * w[i]; }
            if (!have_prev) g0 = 0.0;
            for (int64_t i = 0; i < n; ++i) w[i] -= g0 * v0[i] + g1 * v1[i];
            h0 += g0; h1 += g1;
        }
        double beta = 0.0;
        for (int64_t i = 0; i < n; ++i) beta += w[i] * w[i];
        beta = sqrt(beta);
        alpha[j] = h1;
        up[j] = h0;
        low[j] = beta;
        steps = j + 1;
        if (beta < 1e-8) break;                         /* lucky breakdown */
        for (int64_t i = 0; i < n; ++i) { v0[i] = v1[i]; v1[i] = w[i] / beta; }
        have_prev = 1;
    }
    for (int j = 0; j + 1 < steps; ++j) off[j] = 0.5 * (low[j] + up[j + 1]);  /* (H+H')/2 */
    free(v0); free(v1); free(w);
    return steps;
}

/* Hutchinson over probes [probe_offset, probe_offset+nprobes): returns mean of
 * z' f(A) z; per-probe quadratic forms in quad_out (may be NULL). */
double slq_ref_trace(int64_t n, const int64_t *rp, const int32_t *ci, const double *va,
                     int nprobes, int64_t probe_offset, int m, uint64_t seed, int fun,
                     int nthreads, double *quad_out) {
    double total = 0.0;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
#pragma omp parallel reduction(+ : total)
    {
        double *z = (double *)malloc((size_t)n * sizeof(double));
        double alpha[256], off[256];
#pragma omp for schedule(dynamic, 1)
        for (int p = 0; p < nprobes; ++p) {
            uint64_t key = sm64(sm64(seed) + (uint64_t)(probe_offset + p));
            for (int64_t i = 0; i < n; ++i) z[i] = (sm64(key + (uint64_t)i) >> 63) ? -1.0 : 1.0;
            int steps = slq_ref_lanczos(n, rp, ci, va, z, m, alpha, off);
            double q = (double)n * slq_ref_tridiag_quad(steps, alpha, off, fun);
            if (quad_out) quad_out[p] = q;
            total += q;
        }
        free(z);
    }
    return nprobes > 0 ? total / nprobes : 0.0;
}

/* Diagonal entries e_i' exp(t_k A) e_i for rows i in [row0, row0 + nrows),
 * k < nt: one m-step Lanczos run started from the unit vector e_i (the same
 * recurrence as the probes: lanczos_krylov.m:30-115 with bs = 1) and the
 * Gauss quadrature of its tridiagonal, sum_j tau_j^2 exp(t_k theta_j).
 * Summed over every row this is tr(exp(t A)) with no sampling error: only
 * the quadrature error of m nodes (for exp on a spectrum of width w it is
 * below exp(t lambda_max) (t w)^{2m} / (2^{4m-1} (2m)!)) and rounding.
 * out[(i - row0) * nt + k].  Used to pin config 2 (tests/golden/
 * make_config2_fixture.py): t = 1 gives tr(exp A), t = 2 gives ||exp A||_F^2,
 * from which the Rademacher Hutchinson variance follows exactly. */
void slq_ref_unit_quad(int64_t n, const int64_t *rp, const int32_t *ci, const double *va,
                       int64_t row0, int64_t nrows, int m, const double *t, int nt, int nthreads,
                       double *out) {
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
#pragma omp parallel
    {
        double *z = (double *)calloc((size_t)n, sizeof(double));
        double alpha[256], off[256], d[256], zz[256];
#pragma omp for schedule(dynamic, 4)
        for (int64_t r = 0; r < nrows; ++r) {
            const int64_t i = row0 + r;
            z[i] = 1.0;
            int steps = slq_ref_lanczos(n, rp, ci, va, z, m, alpha, off);
            z[i] = 0.0;
            for (int k = 0; k < nt; ++k) {
                for (int j = 0; j < steps; ++j) d[j] = alpha[j];
                tql_first_row(steps, d, off, zz);
                double q = 0.0;
                for (int j = 0; j < steps; ++j) q += zz[j] * zz[j] * exp(t[k] * d[j]);
                out[r * nt + k] = q;
            }
        }
        free(z);
    }
}

int slq_ref_max_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

/* mctrace_ref.c -- CPU restatement (C + OpenMP) of the reference's OWN
 * trace_exp composition, for the CPU baseline of bench.py's
 * `mc_trace.reference_composition` leg.
 *
 * TEST INFRASTRUCTURE ONLY: loaded by tests/ and bench.py's CPU-baseline leg
 * (through oracle/mctrace_ref.py).  The product never links it.
 *
 *   trace_exp.m:5-6     tr = mc_trace(@(x) expmv(1, A, x, [], 'double'), n, 1e-4, 1000, 1)
 *   mc_trace.m:36-58    block Hutchinson, m = 10 columns per round, K = ceil(maxit/30)
 *                       rounds; S, G Rademacher (:43-44, the build's counter RNG
 *                       in place of sign(randn)), Q = qr(Afun(S), 0) (:45),
 *                       tr += trace(Q' Afun(Q)) (:46), Afun <- P Afun P with
 *                       P = I - Q Q' nested (:47-48), tr_new = tr +
 *                       trace(G' Afun(G)) / m (:49), relative-change stop (:50-56)
 *   expmv.m:31-92       shift mu = trace(A)/n, degree selection, s stages of <= m
 *                       Taylor terms b = (t/(s k)) (A - mu I) b with the
 *                       infinity-norm early stop c1 + c2 <= 2^-53 ||f||_inf
 *   select_taylor_degree.m:16-68, normAm.m:17-23
 *                       ||A||_1, or alpha_p from ||A^(p+1)||_1 = max(A'^(p+1) 1)
 *                       for nonnegative A - mu I, one normAm call (p + 1
 *                       products) per p as the reference does (44 products).
 *
 * Scope: A symmetric (every trace_exp caller's adjacency) with
 * A - mu I >= 0 (no self loops: mu = 0) -- normAm.m's exact branch; the
 * normest1 branch (:25-26) is restated in oracle/krylov_oracle.py only.
 * Blocks are n x b ROW-major (a row's b columns contiguous: one gathered
 * row per nonzero in the SpMM).  qr(., 0) is Householder with LAPACK's
 * reflector signs; traces do not depend on the signs.  OpenMP over rows.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef struct {
    int64_t n;
    const int64_t *rp;
    const int32_t *ci;
    const double *va;
} csr_t;

typedef struct {
    int64_t calls, terms, mv;       /* expmv calls, Taylor terms (A b products), expmv.m's mv */
    double t_select, t_terms;       /* seconds in select_taylor_degree / in the Taylor loops */
    double t_qr, t_proj, t_total;   /* seconds in qr(., 0), in the projections, in all */
} mct_stats;

static double now(void) {
#ifdef _OPENMP
    return omp_get_wtime();
#else
    return 0.0;
#endif
}

static inline uint64_t sm64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

/* Y = (A - mu I) X scaled by c: Y = c (A X - mu X) */
static void spmm10(const csr_t *A, double c, double mu, const double *X, double *Y) {
#pragma omp parallel for schedule(dynamic, 2048)
    for (int64_t i = 0; i < A->n; ++i) {
        double a0 = 0, a1 = 0, a2 = 0, a3 = 0, a4 = 0, a5 = 0, a6 = 0, a7 = 0, a8 = 0, a9 = 0;
        const int64_t kb = A->rp[i], ke = A->rp[i + 1];
        for (int64_t k = kb; k < ke; ++k) {
            if (k + 8 < ke) __builtin_prefetch(X + (int64_t)A->ci[k + 8] * 10, 0, 0);
            const double a = A->va[k];
            const double *x = X + (int64_t)A->ci[k] * 10;
            a0 += a * x[0]; a1 += a * x[1]; a2 += a * x[2]; a3 += a * x[3]; a4 += a * x[4];
            a5 += a * x[5]; a6 += a * x[6]; a7 += a * x[7]; a8 += a * x[8]; a9 += a * x[9];
        }
        const double *xi = X + i * 10;
        double *yi = Y + i * 10;
        yi[0] = c * (a0 - mu * xi[0]); yi[1] = c * (a1 - mu * xi[1]); yi[2] = c * (a2 - mu * xi[2]);
        yi[3] = c * (a3 - mu * xi[3]); yi[4] = c * (a4 - mu * xi[4]); yi[5] = c * (a5 - mu * xi[5]);
        yi[6] = c * (a6 - mu * xi[6]); yi[7] = c * (a7 - mu * xi[7]); yi[8] = c * (a8 - mu * xi[8]);
        yi[9] = c * (a9 - mu * xi[9]);
    }
}

static void spmm(const csr_t *A, int b, double c, double mu, const double *X, double *Y) {
    if (b == 10) {  /* the mc_trace blocks (m = 10, mc_trace.m:36) */
        spmm10(A, c, mu, X, Y);
        return;
    }
#pragma omp parallel for schedule(dynamic, 2048)
    for (int64_t i = 0; i < A->n; ++i) {
        double acc[64];
        for (int j = 0; j < b; ++j) acc[j] = 0.0;
        for (int64_t k = A->rp[i]; k < A->rp[i + 1]; ++k) {
            const double a = A->va[k];
            const double *x = X + (int64_t)A->ci[k] * b;
            for (int j = 0; j < b; ++j) acc[j] += a * x[j];
        }
        const double *xi = X + i * b;
        double *yi = Y + i * b;
        for (int j = 0; j < b; ++j) yi[j] = c * (acc[j] - mu * xi[j]);
    }
}

/* norm(X, inf) = max row sum of |X| (n x b) */
static double inf_norm(int64_t n, int b, const double *X) {
    double m = 0.0;
#pragma omp parallel for schedule(static, 4096) reduction(max : m)
    for (int64_t i = 0; i < n; ++i) {
        double s = 0.0;
        for (int j = 0; j < b; ++j) s += fabs(X[i * b + j]);
        if (s > m) m = s;
    }
    return m;
}

/* normAm.m:17-23: ||(t(A - mu I))^m||_1 = max(((t(A - mu I))')^m ones), A symmetric */
static double normAm_nonneg(const csr_t *A, double t, double mu, int m, double *e, double *w) {
    const int64_t n = A->n;
    for (int64_t i = 0; i < n; ++i) e[i] = 1.0;
    for (int k = 0; k < m; ++k) {
        spmm(A, 1, t, mu, e, w);
        memcpy(e, w, sizeof(double) * (size_t)n);
    }
    double c = 0.0;
    for (int64_t i = 0; i < n; ++i)
        if (fabs(e[i]) > c) c = fabs(e[i]);
    return c;
}

/* select_taylor_degree.m:16-68 (prec 'double', p_max = 8, m_max = 55) and the
 * cost minimisation of expmv.m:53-68: s, m, and the products it took */
static int select_degree(const csr_t *A, double t, double mu, int ncols, const double *theta, int *s_out,
                         int *m_out, int *mv_out) {
    const int64_t n = A->n;
    const int m_max = 55, p_max = 8;
    double normA = 0.0;  /* norm(t (A - mu I), 1): column sums = row sums (symmetric) */
#pragma omp parallel for schedule(static, 4096) reduction(max : normA)
    for (int64_t i = 0; i < n; ++i) {
        double s = 0.0;
        int diag = 0;
        for (int64_t k = A->rp[i]; k < A->rp[i + 1]; ++k) {
            const int d = A->ci[k] == i;
            diag |= d;
            s += fabs(t * (A->va[k] - (d ? mu : 0.0)));
        }
        if (!diag) s += fabs(t * mu);
        if (s > normA) normA = s;
    }
    double alpha[8];
    int mv = 0;
    if (normA <= 4.0 * theta[m_max - 1] * p_max * (p_max + 3) / ((double)m_max * ncols)) {
        for (int p = 0; p < p_max - 1; ++p) alpha[p] = normA;
    } else {
        double *e = (double *)malloc(sizeof(double) * (size_t)n);
        double *w = (double *)malloc(sizeof(double) * (size_t)n);
        if (!e || !w) {
            free(e);
            free(w);
            return -1;
        }
        double eta[8];
        for (int p = 1; p <= p_max; ++p) {
            eta[p - 1] = pow(normAm_nonneg(A, t, mu, p + 1, e, w), 1.0 / (p + 1));
            mv += p + 1;
        }
        for (int p = 1; p < p_max; ++p) alpha[p - 1] = fmax(eta[p - 1], eta[p]);
        free(e);
        free(w);
    }
    double cost = INFINITY;
    int m_best = 0;
    for (int mm = 1; mm <= m_max; ++mm) {
        double cm = INFINITY;
        for (int p = 2; p <= p_max; ++p) {
            if (mm < p * (p - 1) - 1) continue;
            double c = ceil(alpha[p - 2] / theta[mm - 1]) * mm;
            if (c == 0.0) c = INFINITY;
            if (c < cm) cm = c;
        }
        if (cm < cost) {
            cost = cm;
            m_best = mm;
        }
    }
    if (t == 0.0) m_best = 0;
    if (cost == INFINITY) cost = 0.0;
    *m_out = m_best;
    *s_out = (int)fmax(cost / (m_best > 0 ? m_best : 1), 1.0);
    *mv_out = mv;
    return 0;
}

/* F = expmv(t, A, B, [], 'double') on an n x b row-major block (expmv.m:1-94) */
int mct_expmv(const csr_t *A, double t, int b, const double *B, double *F, const double *theta, int *s_out,
              int *m_out, int *mv_out, mct_stats *st) {
    const int64_t n = A->n;
    if (b < 1 || b > 64) return -1;
    double trA = 0.0;  /* :31-36 shift */
    for (int64_t i = 0; i < n; ++i)
        for (int64_t k = A->rp[i]; k < A->rp[i + 1]; ++k)
            if (A->ci[k] == i) trA += A->va[k];
    const double mu = n ? trA / (double)n : 0.0;
    const double t0 = now();
    int s = 1, m = 0, mv = 0;
    if (select_degree(A, t, mu, b, theta, &s, &m, &mv) != 0) return -2;
    const double t1 = now();
    const double tol = ldexp(1.0, -53), eta = exp(t * mu / s);
    double *bb = (double *)malloc(sizeof(double) * (size_t)n * b);
    double *ab = (double *)malloc(sizeof(double) * (size_t)n * b);
    if (!bb || !ab) {
        free(bb);
        free(ab);
        return -2;
    }
    memcpy(bb, B, sizeof(double) * (size_t)n * b);
    memcpy(F, B, sizeof(double) * (size_t)n * b);
    int64_t terms = 0;
    for (int i = 0; i < s; ++i) {  /* :73-92 */
        double c1 = inf_norm(n, b, bb);
        for (int k = 1; k <= m; ++k) {
            spmm(A, b, t / ((double)s * k), mu, bb, ab);  /* b = (t/(s k)) (A - mu I) b */
            double *tmp = bb;
            bb = ab;
            ab = tmp;
            ++mv;
            ++terms;
            double c2 = 0.0, nf = 0.0;
#pragma omp parallel for schedule(static, 4096) reduction(max : c2, nf)
            for (int64_t r = 0; r < n; ++r) {  /* f = f + b; norm(b, inf), norm(f, inf) */
                double sb = 0.0, sf = 0.0;
                for (int j = 0; j < b; ++j) {
                    const double v = F[r * b + j] + bb[r * b + j];
                    F[r * b + j] = v;
                    sb += fabs(bb[r * b + j]);
                    sf += fabs(v);
                }
                if (sb > c2) c2 = sb;
                if (sf > nf) nf = sf;
            }
            if (c1 + c2 <= tol * nf) break;
            c1 = c2;
        }
#pragma omp parallel for schedule(static, 4096)
        for (int64_t r = 0; r < n * b; ++r) {  /* f = eta f; b = f */
            F[r] *= eta;
            bb[r] = F[r];
        }
    }
    free(bb);
    free(ab);
    if (s_out) *s_out = s;
    if (m_out) *m_out = m;
    if (mv_out) *mv_out = mv;
    if (st) {
        st->calls += 1;
        st->terms += terms;
        st->mv += mv;
        st->t_select += t1 - t0;
        st->t_terms += now() - t1;
    }
    return 0;
}

/* column dot products G (p x q, row-major p rows) = X' Y for n x p, n x q row-major blocks */
static void gram(int64_t n, int p, const double *X, int q, const double *Y, double *G) {
    for (int a = 0; a < p * q; ++a) G[a] = 0.0;
#pragma omp parallel
    {
        double loc[64 * 64];
        for (int a = 0; a < p * q; ++a) loc[a] = 0.0;
#pragma omp for schedule(static, 4096)
        for (int64_t r = 0; r < n; ++r)
            for (int i = 0; i < p; ++i)
                for (int j = 0; j < q; ++j) loc[i * q + j] += X[r * p + i] * Y[r * q + j];
#pragma omp critical
        for (int a = 0; a < p * q; ++a) G[a] += loc[a];
    }
}

/* X <- X - Q (Q' X), Q n x b orthonormal, X n x b (mc_trace.m:47 aux) */
static void project(int64_t n, int b, const double *Q, double *X) {
    double G[64 * 64];
    gram(n, b, Q, b, X, G);
#pragma omp parallel for schedule(static, 4096)
    for (int64_t r = 0; r < n; ++r)
        for (int j = 0; j < b; ++j) {
            double s = 0.0;
            for (int i = 0; i < b; ++i) s += Q[r * b + i] * G[i * b + j];
            X[r * b + j] -= s;
        }
}

/* w[c] = sum_{r >= r0} v[r] W[r, c] for c in [c0, b): one pass over the rows */
static void col_dots(int64_t n, int b, int64_t r0, int c0, const double *V, int j, const double *W, double *w) {
    for (int c = 0; c < b; ++c) w[c] = 0.0;
#pragma omp parallel
    {
        double loc[64] = {0};
#pragma omp for schedule(static, 4096)
        for (int64_t r = r0; r < n; ++r) {
            const double v = V[r * b + j];
            for (int c = c0; c < b; ++c) loc[c] += v * W[r * b + c];
        }
#pragma omp critical
        for (int c = c0; c < b; ++c) w[c] += loc[c];
    }
}

/* [Q, ~] = qr(W, 0): Householder (LAPACK signs), Q n x b row-major over W's
 * storage; each reflector's dots and update are one pass over the rows */
static int householder_qr(int64_t n, int b, double *W) {
    double *V = (double *)malloc(sizeof(double) * (size_t)n * b);  /* reflectors, row-major */
    double tau[64], w[64];
    if (!V) return -2;
    for (int j = 0; j < b; ++j) {
        double nrm2 = 0.0;
#pragma omp parallel for schedule(static, 4096) reduction(+ : nrm2)
        for (int64_t r = j; r < n; ++r) nrm2 += W[r * b + j] * W[r * b + j];
        const double alpha = W[(int64_t)j * b + j];
        const double xn = sqrt(fmax(nrm2 - alpha * alpha, 0.0));
        const double beta = -copysign(sqrt(nrm2), alpha);
        tau[j] = xn == 0.0 ? 0.0 : (beta - alpha) / beta;  /* tau = 0: H = I (dlarfg) */
        const double sc = xn == 0.0 ? 0.0 : 1.0 / (alpha - beta);
#pragma omp parallel for schedule(static, 4096)
        for (int64_t r = 0; r < n; ++r) V[r * b + j] = (r < j) ? 0.0 : (r == j) ? 1.0 : W[r * b + j] * sc;
        if (tau[j] == 0.0 || j + 1 == b) continue;
        col_dots(n, b, j, j + 1, V, j, W, w);  /* apply H_j to the trailing columns */
#pragma omp parallel for schedule(static, 4096)
        for (int64_t r = j; r < n; ++r) {
            const double tv = tau[j] * V[r * b + j];
            for (int c = j + 1; c < b; ++c) W[r * b + c] -= tv * w[c];
        }
    }
    /* Q = H_0 ... H_{b-1} [I; 0]: apply the reflectors in reverse to e_1..e_b */
#pragma omp parallel for schedule(static, 4096)
    for (int64_t r = 0; r < n; ++r)
        for (int c = 0; c < b; ++c) W[r * b + c] = (r == c) ? 1.0 : 0.0;
    for (int j = b - 1; j >= 0; --j) {
        if (tau[j] == 0.0) continue;
        col_dots(n, b, j, 0, V, j, W, w);
#pragma omp parallel for schedule(static, 4096)
        for (int64_t r = j; r < n; ++r) {
            const double tv = tau[j] * V[r * b + j];
            for (int c = 0; c < b; ++c) W[r * b + c] -= tv * w[c];
        }
    }
    free(V);
    return 0;
}

/* The mc_trace round's Afun on block X (n x 10): Y = P_{k-1}..P_0 F(P_0..P_{k-1} X),
 * P_i = I - Q_i Q_i', F = expmv(1, A, .) (mc_trace.m:47-48 nesting) */
static int afun(const csr_t *A, int nq, double *const *Qs, const double *X, double *Y, double *tmp,
                const double *theta, mct_stats *st) {
    const int64_t n = A->n;
    const int b = 10;
    memcpy(tmp, X, sizeof(double) * (size_t)n * b);
    double tp = now();
    for (int i = nq - 1; i >= 0; --i) project(n, b, Qs[i], tmp);
    st->t_proj += now() - tp;
    int s, m, mv;
    if (mct_expmv(A, 1.0, b, tmp, Y, theta, &s, &m, &mv, st) != 0) return -2;
    tp = now();
    for (int i = 0; i < nq; ++i) project(n, b, Qs[i], Y);
    st->t_proj += now() - tp;
    return 0;
}

static double block_trace(int64_t n, const double *X, const double *Y) {
    double G[100];
    gram(n, 10, X, 10, Y, G);
    double t = 0.0;
    for (int i = 0; i < 10; ++i) t += G[i * 10 + i];
    return t;
}

static void rademacher(int64_t n, uint64_t seed, int64_t base, double *X) {
    uint64_t key[10];
    for (int c = 0; c < 10; ++c) key[c] = sm64(sm64(seed) + (uint64_t)(base + c));
#pragma omp parallel for schedule(static, 4096)
    for (int64_t r = 0; r < n; ++r)
        for (int c = 0; c < 10; ++c) X[r * 10 + c] = (sm64(key[c] + (uint64_t)r) >> 63) ? -1.0 : 1.0;
}

/* [tr, res, it] = mc_trace(@(x) expmv(1, A, x, [], 'double'), n, tol, maxit, 1);
 * rounds_max > 0 stops after that many rounds (a bounded sample of the loop).
 * Returns 0, or < 0 on an allocation failure / bad argument. */
int mct_trace_exp(int64_t n, const int64_t *rp, const int32_t *ci, const double *va, double tol, int maxit,
                  uint64_t seed, const double *theta, int nthreads, int rounds_max, double *tr_out,
                  double *res_out, int *it_out, mct_stats *st) {
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
    const csr_t A = {n, rp, ci, va};
    const int mb = 10;
    const int K = (maxit + 3 * mb - 1) / (3 * mb);  /* :41 */
    const size_t blk = sizeof(double) * (size_t)n * mb;
    double *S = malloc(blk), *G = malloc(blk), *Y = malloc(blk), *Z = malloc(blk), *tmp = malloc(blk);
    double **Qs = calloc((size_t)K + 1, sizeof(double *));
    int rc = 0, nq = 0, it = 0;
    double tr = 0.0, tr_old = 0.0, tr_new = 0.0, res = 1.0;
    const double t0 = now();
    memset(st, 0, sizeof(*st));
    if (!S || !G || !Y || !Z || !tmp || !Qs) {
        rc = -2;
        goto done;
    }
    for (it = 1; it <= K; ++it) {  /* :42 */
        const int64_t base = (int64_t)(it - 1) * 2 * mb;
        rademacher(n, seed, base, S);       /* :43 */
        rademacher(n, seed, base + mb, G);  /* :44 */
        if ((rc = afun(&A, nq, Qs, S, Y, tmp, theta, st)) != 0) goto done;   /* :45 */
        double tq = now();
        if ((rc = householder_qr(n, mb, Y)) != 0) goto done;
        st->t_qr += now() - tq;
        if ((rc = afun(&A, nq, Qs, Y, Z, tmp, theta, st)) != 0) goto done;   /* :46 */
        tr += block_trace(n, Y, Z);
        Qs[nq++] = Y;                                                       /* :47-48 */
        Y = malloc(blk);
        if (!Y) {
            rc = -2;
            goto done;
        }
        if ((rc = afun(&A, nq, Qs, G, Z, tmp, theta, st)) != 0) goto done;   /* :49 */
        tr_new = tr + block_trace(n, G, Z) / mb;
        res = fabs(tr_new - tr_old) / fmax(fabs(tr_new), fabs(tr_old));    /* :50 */
        if (res < tol) break;                                               /* :54-56 */
        tr_old = tr_new;
        if (rounds_max > 0 && it >= rounds_max) break;
    }
    if (it > K) it = K;
done:
    st->t_total = now() - t0;
    if (Qs)
        for (int i = 0; i < nq; ++i) free(Qs[i]);
    free(Qs);
    free(S);
    free(G);
    free(Y);
    free(Z);
    free(tmp);
    if (tr_out) *tr_out = tr_new;
    if (res_out) *res_out = res;
    if (it_out) *it_out = it;
    return rc;
}

/* expmv on a row-major block with its own thread count (tests / timing) */
int mct_expmv_block(int64_t n, const int64_t *rp, const int32_t *ci, const double *va, double t, int b,
                    const double *B, double *F, const double *theta, int nthreads, int *s, int *m, int *mv,
                    mct_stats *st) {
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
    const csr_t A = {n, rp, ci, va};
    if (st) memset(st, 0, sizeof(*st));
    return mct_expmv(&A, t, b, B, F, theta, s, m, mv, st);
}

/* Seconds of one qr(W, 0) of an n x 10 Rademacher block and of one
 * projection X - Q (Q' X) against its Q (mc_trace.m:45, :47): the host-side
 * work of a round, for extrapolating a bounded CPU sample */
int mct_round_host_times(int64_t n, uint64_t seed, int nthreads, double *t_qr, double *t_proj) {
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
    const size_t blk = sizeof(double) * (size_t)n * 10;
    double *W = malloc(blk), *X = malloc(blk);
    if (!W || !X) {
        free(W);
        free(X);
        return -2;
    }
    rademacher(n, seed, 0, W);
    rademacher(n, seed, 10, X);
    double t0 = now();
    if (householder_qr(n, 10, W) != 0) {
        free(W);
        free(X);
        return -2;
    }
    double t1 = now();
    project(n, 10, W, X);
    double t2 = now();
    *t_qr = t1 - t0;
    *t_proj = t2 - t1;
    free(W);
    free(X);
    return 0;
}

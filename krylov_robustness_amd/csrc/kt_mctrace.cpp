// kt_mctrace.cpp -- mc_trace.m / trace_exp.m / expmv.m on the device.
//
//   mc_trace.m  -> kt_mc_trace: block Hutchinson with Hutch++-style nested
//                  deflation (m = 10 columns per round, K = ceil(maxit/30)).
//                  Afun is one of: the matrix itself (mc_trace.m:32-34), the
//                  Lanczos-f action, or expmv (trace_exp.m:5).
//   trace_exp.m -> kt_trace_exp: mc_trace(Afun, n, 1e-4, 1000, 1).
//   expmv.m     -> kt_expmv (+ select_taylor_degree.m, normAm.m).
// Probes S, G of round it are Rademacher columns (it-1)*20 + [0,10) and
// [10,20) of the build's counter RNG (oracle/krylov_oracle.py:mc_trace).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <thread>

#include "kt_krylov.h"
#include "kt_worker.h"
#include "kt_launch.h"
#include "kt_slq.h"

namespace kt {

// theta_m for m = 1..100, prec = 'double' (functions/theta_taylor.mat,
// Al-Mohy & Higham 2011, Table; loaded by select_taylor_degree.m:31).
static const double kTheta[100] = {
2.2204460492503131e-16, 2.5809568029946243e-08, 1.3863478661191185e-05, 0.00033971688399768305,
0.0024008763578872742, 0.0090656564075951018, 0.023844555325002736, 0.049912288711153226,
0.08957760203223343, 0.1441829761614378, 0.21423580684517107, 0.29961589138115802,
0.3997775336316795, 0.51391469361242936, 0.64108352330411988, 0.78028742566265763,
0.93053284607865683, 1.0908637192900361, 1.2603810606426387, 1.4382525968043369,
1.6237159502358214, 1.8160778162150852, 2.0147107809446161, 2.2190488693650896,
2.4285825244428265, 2.6428534574594353, 2.8614496339342641, 3.0840005449891619,
3.3101728398902708, 3.5396663487436895, 3.772210495681751, 4.0075610861180397,
4.2454974425796959, 4.4858198594473686, 4.728347345793539, 4.9729156261919814,
5.219375371084058, 5.4675906305245441, 5.7174374475720127, 5.9688026300418491,
6.221582661689891, 6.4756827360799845, 6.731015898381024, 6.9875022821306301,
7.2450684295979526, 7.5036466857888637, 7.763174657377987, 8.0235947289399796,
8.2848536298039175, 8.5469020456849325, 8.8096942699713221, 9.0731878901761451,
9.3373435056120133, 9.6021244728265565, 9.8674966757534008, 10.133428317897478,
10.399889734191031, 10.666853220434106, 10.934292878475777, 11.202184475504579,
11.470505316002537, 11.739234125080184, 12.008350942053168, 12.277837023246892,
12.547674753126438, 12.817847562946627, 13.088339856203294, 13.359136940242903,
13.630224963455026, 13.901590857531859, 14.173222284331819, 14.445107586931254,
14.717235744490083, 14.989596330594328, 15.262179474771679, 15.534975826905702,
15.807976524300871, 16.081173161174046, 16.354557760369328, 16.628122747112073,
16.901860924634942, 17.175765451524093, 17.449829820647437, 17.724047839539214,
17.998413612126303, 18.27292152169181, 18.54756621498051, 18.822342587358953,
19.09724576895055, 19.372271111672617, 19.647414177108576, 19.922670725154251,
20.198036703383082, 20.473508237083141, 20.749081619935929, 21.024753305356054,
21.300519898663481, 21.576378150721375, 21.85232495499011, 22.128357353464594
};

enum { AFUN_MATRIX = 0, AFUN_LANCZOS = 1, AFUN_EXPMV = 2 };

// B = A - mu I (expmv.m:33-36 shift; A symmetric, so B' = B): y = B x on one
// column, as the SpMV of A followed by y -= mu x.
static void shifted_spmv(kt_matrix_s* A, double mu, const double* x, double* y) {
    spmm(A, x, 1, y, 1, 1);
    if (mu != 0.0) KT_HIP(launch_axpby((int)A->n, 1, -mu, x, 1, 1.0, y, 1, A->ctx->stream));
}

// normAm.m: ||A^m||_1 for A - mu I >= 0 (exact: e = A'^m ones, c = ||e||_inf), for
// every m = 2..mmax at once: select_taylor_degree.m:48-53 asks for
// m = p + 1, p = 1..p_max, each from ones -- the same vectors A^m ones, so
// one chain of mmax SpMVs gives them all (one host round trip).
static std::vector<double> normAm_chain(kt_matrix_s* A, double mu, int mmax) {
    kt_context_s* ctx = A->ctx;
    const int64_t n = A->n;
    const int nb = inf_norm_blocks();
    DevMat e, t;
    e.alloc(ctx, n, 1);
    t.alloc(ctx, n, 1);
    DevBuf& part = ctx->ws.norm_part;
    part.ensure(sizeof(double) * (size_t)nb * (mmax + 1));
    KT_HIP(launch_fill(e.col(0), (int)n, 1.0, ctx->stream));
    for (int j = 1; j <= mmax; ++j) {  // B' e = B e
        shifted_spmv(A, mu, e.col(0), t.col(0));
        copy_cols(ctx, n, t.col(0), 1, e.col(0), 1, 1);
        KT_HIP(launch_inf_norm((int)n, 1, e.col(0), 1, part.as<double>() + (size_t)j * nb, ctx->stream));
    }
    std::vector<double> h((size_t)nb * (mmax + 1));
    KT_HIP(hipMemcpyAsync(h.data() + nb, part.as<double>() + nb, sizeof(double) * (size_t)nb * mmax,
                          hipMemcpyDeviceToHost, ctx->stream));
    KT_HIP(hipStreamSynchronize(ctx->stream));
    std::vector<double> c(mmax + 1, 0.0);
    for (int j = 1; j <= mmax; ++j)
        c[j] = *std::max_element(h.begin() + (size_t)j * nb, h.begin() + (size_t)(j + 1) * nb);
    return c;
}

// normAm.m:25-26 for a matrix with negative entries: [c,~,~,it] =
// normest1(@afun_power, t = 1), the Higham-Tisseur estimator (Algorithm 2.4)
// of ||C^m||_1, C = t (A - mu I), with one column -- deterministic: start
// ones/n, then unit vectors e_ind at the largest |Z| (smallest index on
// ties), stop on no improvement, parallel signs, a repeated best index or
// after itmax = 5 (oracle/krylov_oracle.py normest1_t1).  C is symmetric,
// so the transposed products are the same chain.  Products and reductions
// run on the device; the host reads 2-3 partial vectors per iteration.
// Returns {c, mv = it(2) * m}.
static std::pair<double, int> normest1_power(kt_matrix_s* A, double mu, double t, int m) {
    kt_context_s* ctx = A->ctx;
    hipStream_t st = ctx->stream;
    const int64_t n = A->n;
    DevMat X, Y, T, S0, S1;
    X.alloc(ctx, n, 1);
    Y.alloc(ctx, n, 1);
    T.alloc(ctx, n, 1);
    S0.alloc(ctx, n, 1);  // S_old (zero before the first sign vector)
    S1.alloc(ctx, n, 1);
    auto apply = [&](const double* in, double* out) {  // out = C^m in (in kept)
        const double* src = in;
        for (int i = 0; i < m; ++i) {
            double* dst = (i % 2 == m % 2) ? T.col(0) : out;  // the last product lands in out
            shifted_spmv(A, mu, src, dst);
            if (t != 1.0) KT_HIP(launch_axpby((int)n, 1, t, dst, 1, 0.0, dst, 1, st));
            src = dst;
        }
    };
    auto unit = [&](double* x, int64_t i) {
        static const double one = 1.0;
        KT_HIP(hipMemsetAsync(x, 0, sizeof(double) * (size_t)n, st));
        KT_HIP(hipMemcpyAsync(x + i, &one, sizeof(double), hipMemcpyHostToDevice, st));
    };
    const int nb = normest1_blocks((int)n);
    DevBuf& part = ctx->ws.norm_part;
    part.ensure(std::max(sizeof(double) * 2 * nb, (sizeof(double) + sizeof(int)) * nb));
    std::vector<double> hp(2 * nb);
    std::vector<int> hi(nb);
    if (n <= 4) {  // exact: the identity's columns (normest1's small-n branch)
        double est = 0.0;
        std::vector<double> y(n);
        for (int64_t j = 0; j < n; ++j) {
            unit(X.col(0), j);
            apply(X.col(0), Y.col(0));
            KT_HIP(hipMemcpyAsync(y.data(), Y.col(0), sizeof(double) * n, hipMemcpyDeviceToHost, st));
            KT_HIP(hipStreamSynchronize(st));
            double s = 0.0;
            for (double v : y) s += std::fabs(v);
            est = std::max(est, s);
        }
        return {est, 0};
    }
    KT_HIP(launch_fill(X.col(0), (int)n, 1.0 / (double)n, st));
    double* S = S1.col(0);
    double* S_old = S0.col(0);
    const int itmax = 5;
    double est = 0.0, est_old = 0.0;
    int64_t ind = -1, ind_best = -1;
    int k = 1, it2 = 0;
    while (true) {
        apply(X.col(0), Y.col(0));                                       // (1) Y = C^m X
        KT_HIP(launch_normest1_y((int)n, Y.col(0), S_old, S, part.as<double>(), st));
        KT_HIP(hipMemcpyAsync(hp.data(), part.ptr, sizeof(double) * 2 * nb, hipMemcpyDeviceToHost, st));
        KT_HIP(hipStreamSynchronize(st));
        double ssum = 0.0, dot = 0.0;
        for (int b = 0; b < nb; ++b) {
            ssum += hp[b];
            dot += hp[nb + b];
        }
        est = ssum;
        if ((est > est_old || k == 2) && k >= 2) ind_best = ind;
        if (k >= 2 && est <= est_old) {                                  // (2)
            est = est_old;
            break;
        }
        est_old = est;
        if (k > itmax) break;
        if (std::fabs(dot) == (double)n) break;                          // (3) S parallel to S_old
        apply(S, Y.col(0));                                              // (4) Z = C^m S (into Y)
        ++it2;
        double* pv = part.as<double>();
        int* pi = reinterpret_cast<int*>(pv + nb);
        KT_HIP(launch_absmax_idx((int)n, Y.col(0), pv, pi, st));
        double zbest = 0.0;
        KT_HIP(hipMemcpyAsync(hp.data(), pv, sizeof(double) * nb, hipMemcpyDeviceToHost, st));
        KT_HIP(hipMemcpyAsync(hi.data(), pi, sizeof(int) * nb, hipMemcpyDeviceToHost, st));
        if (k >= 2)
            KT_HIP(hipMemcpyAsync(&zbest, Y.col(0) + ind_best, sizeof(double), hipMemcpyDeviceToHost, st));
        KT_HIP(hipStreamSynchronize(st));
        double hmax = -1.0;
        int imax = 0x7fffffff;
        for (int b = 0; b < nb; ++b)
            if (hp[b] > hmax || (hp[b] == hmax && hi[b] < imax)) {
                hmax = hp[b];
                imax = hi[b];
            }
        if (k >= 2 && hmax == std::fabs(zbest)) break;                   // (5)
        ind = imax;
        unit(X.col(0), ind);                                             // X = e_ind
        std::swap(S, S_old);
        ++k;
    }
    return {est, it2 * m};
}

struct Expmv {
    int s = 1, m = 0, mv = 0;
};

// expmv.m:1-94 with prec = 'double', shift = true, bal = false, M = [] ;
// F = exp(t A) B on nc columns of the device block B (ld), written to F.
static Expmv expmv_device(kt_matrix_s* A, double t, const double* Bsrc, int ld, int nc, double* F) {
    kt_context_s* ctx = A->ctx;
    const int64_t n = A->n;
    hipStream_t st = ctx->stream;
    Expmv r;
    ctx->expmv_calls += 1;
    // shift + degree selection, cached per (A version, t, block width): the
    // reference recomputes them every call from the same inputs; the
    // selection's matrix products still count in mv, as expmv.m's mv does
    if (A->expmv_sel_ok && A->expmv_sel_version == A->version && A->expmv_sel_t == t &&
        A->expmv_sel_nc == nc) {
        r.s = A->expmv_sel_s;
        r.m = A->expmv_sel_m;
        r.mv = A->expmv_sel_mv;
    } else {
        // shift: mu = trace(A)/n   (:31-36)
        double trA = 0.0;
        for (int64_t i = 0; i < n; ++i)
            for (int64_t k = A->h_rowptr[i]; k < A->h_rowptr[i + 1]; ++k)
                if (A->h_col[k] == i) trA += A->h_val[k];
        const double mu = n ? trA / (double)n : 0.0;
        // select_taylor_degree(t*(A - mu I), b)   (:41; select_taylor_degree.m:16-68)
        const int m_max = 55, p_max = 8;
        std::vector<double> colsum(n, 0.0);
        for (int64_t i = 0; i < n; ++i)
            for (int64_t k = A->h_rowptr[i]; k < A->h_rowptr[i + 1]; ++k)
                colsum[A->h_col[k]] += std::fabs(t * (A->h_val[k] - (A->h_col[k] == i ? mu : 0.0)));
        for (int64_t i = 0; i < n; ++i) {  // diagonal entries absent from the CSR still get -mu
            bool has = false;
            for (int64_t k = A->h_rowptr[i]; k < A->h_rowptr[i + 1]; ++k) has |= (A->h_col[k] == i);
            if (!has) colsum[i] += std::fabs(t * mu);
        }
        const double normA = n ? *std::max_element(colsum.begin(), colsum.end()) : 0.0;
        std::vector<double> alpha(p_max - 1);
        if (normA <= 4.0 * kTheta[m_max - 1] * p_max * (p_max + 3) / ((double)m_max * nc)) {
            std::fill(alpha.begin(), alpha.end(), normA);  // unA = 1
        } else {
            // normAm.m:17 isequal(A, abs(A)) on t (A - mu I): every stored entry
            // and every diagonal (absent ones are -mu) times t is >= 0
            bool nonneg = true;
            for (int64_t i = 0; i < n && nonneg; ++i) {
                bool has = false;
                for (int64_t k = A->h_rowptr[i]; k < A->h_rowptr[i + 1]; ++k) {
                    const bool dg = A->h_col[k] == i;
                    has |= dg;
                    if (t * (A->h_val[k] - (dg ? mu : 0.0)) < 0.0) nonneg = false;
                }
                if (!has && t * -mu < 0.0) nonneg = false;
            }
            std::vector<double> eta(p_max);
            if (nonneg) {
                const std::vector<double> nAm = normAm_chain(A, mu, p_max + 1);
                for (int p = 1; p <= p_max; ++p) {
                    const double c = nAm[p + 1] * std::pow(std::fabs(t), p + 1);
                    r.mv += p + 1;  // as normAm.m counts them (one chain per m)
                    eta[p - 1] = std::pow(c, 1.0 / (p + 1));
                }
            } else {
                for (int p = 1; p <= p_max; ++p) {  // :25-26 normest1, mv = it(2) * m
                    const std::pair<double, int> cm = normest1_power(A, mu, t, p + 1);
                    r.mv += cm.second;
                    eta[p - 1] = std::pow(cm.first, 1.0 / (p + 1));
                }
            }
            for (int p = 1; p < p_max; ++p) alpha[p - 1] = std::max(eta[p - 1], eta[p]);
        }
        // M(m, p-1) = alpha(p-1) / theta(m); cost = min over (m, p) of m * ceil(M)   (expmv.m:57-67)
        double cost = INFINITY;
        int m_best = 0;
        for (int mm = 1; mm <= m_max; ++mm) {
            double cm = INFINITY;
            for (int p = 2; p <= p_max; ++p) {
                if (mm < p * (p - 1) - 1) continue;
                const double Mv = alpha[p - 2] / kTheta[mm - 1];
                double c = std::ceil(Mv) * mm;
                if (c == 0.0) c = INFINITY;
                cm = std::min(cm, c);
            }
            if (cm < cost) {
                cost = cm;
                m_best = mm;
            }
        }
        if (t == 0.0) m_best = 0;
        if (cost == INFINITY) cost = 0.0;
        r.m = m_best;
        r.s = (int)std::max(cost / std::max(m_best, 1), 1.0);
        A->expmv_sel_ok = true;
        A->expmv_sel_version = A->version;
        A->expmv_sel_t = t;
        A->expmv_sel_nc = nc;
        A->expmv_sel_mu = mu;
        A->expmv_sel_s = r.s;
        A->expmv_sel_m = r.m;
        A->expmv_sel_mv = r.mv;
    }
    const double mu = A->expmv_sel_mu;
    const double tol = std::ldexp(1.0, -53);
    const double eta = std::exp(t * mu / r.s);  // :70
    // f = b; b = (t/(s k)) (A - mu I) b ...   (:71-92)
    DevMat b, Ab;
    b.alloc(ctx, n, ld);
    Ab.alloc(ctx, n, ld);
    copy_cols(ctx, n, Bsrc, ld, b.col(0), ld, nc);
    copy_cols(ctx, n, Bsrc, ld, F, ld, nc);
    // The stop test `c1 + c2 <= tol*norm(f, inf)` runs on the device
    // (k_expmv_check clears state.active; the remaining terms of the stage
    // are no-ops), so a stage is queued without host round trips.  Same
    // arithmetic as the host-tested loop: b = (t/(s k)) (A b - mu b),
    // f = f + b, row sums of |.| in column order.
    const int nb = inf_norm_blocks();
    ctx->ws.norm_part.ensure(sizeof(double) * 2 * nb);
    ctx->ws.expmv_state.ensure(expmv_state_bytes());
    double* part = ctx->ws.norm_part.as<double>();
    void* state = ctx->ws.expmv_state.ptr;
    KT_HIP(hipMemsetAsync(state, 0, expmv_state_bytes(), st));
    const int P = pow2_at_least(std::max(nc, 1));
    if (P <= 32 && ld >= P && !std::getenv("KT_EXPMV_UNFUSED")) {
        // One launch per term (k_expmv_step: the previous term's stop test,
        // SpMM, update, the term's norm maxima); b ping-pongs, the maxima
        // rotate through three slots of the state.  Every row sums its
        // gathers in the order of the reference's A*b (natural CSR order).
        const DevCSR& M0 = natural_csr(A);
        // KT_EXPMV_SPLIT=0 / 1 forces the fused / split term form (read per call)
        const char* spe = std::getenv("KT_EXPMV_SPLIT");
        const bool split = spe ? spe[0] == '1' : expmv_split_check((int)n, P, M0.n_long, M0.n_med);
        // the split form runs row-blocked (k_expmv_rows, resident workgroups)
        // with each term's kernel first testing the previous term's stop
        // (form 3); KT_EXPMV_ROWS=0 selects the workgroup-per-row-class split
        // kernel, KT_EXPMV_ROWCHECK=0 the row-blocked one with the separate
        // slot-check launch (A/B)
        const char* rwe = std::getenv("KT_EXPMV_ROWS");
        const char* rce = std::getenv("KT_EXPMV_ROWCHECK");
        int form = !split ? 0 : (rwe && rwe[0] == '0') ? 1 : (rce && rce[0] == '0') ? 2 : 3;
        if (form >= 2 && !(M0.short_tasks && M0.med_tasks)) form = 1;  // (the launcher's own fallback)
        // (Measured and dropped, round 6: the Taylor loop on hubs-first copies
        // of b and f with each row in natural column order -- bit-identical --
        // ran 16 % slower than the natural table, profiles/r06/expmv_rows_ab.)
        const DevCSR& M = M0;
        const CsrView V{M.rowptr, M.col, M.val, (int)n, M.long_rows, M.n_long, A->long_thresh,
                        kSplitThresh, M.ck_beg, M.ck_end, M.n_chunks, M.sp_rows, M.sp_first, M.n_split,
                        M.short_tasks, M.n_short, M.med_tasks, M.n_heavy};
        // The launch that finds a stage's stop test satisfied also stores the
        // stage index into a coherent host flag; the host, which queues terms
        // only slightly ahead of the device here, stops queueing that stage's
        // remaining (no-op) terms once it sees it.  KT_EXPMV_STOPFLAG=0 queues
        // all s * m terms.
        const char* sf = std::getenv("KT_EXPMV_STOPFLAG");
        const bool use_flag = !(sf && sf[0] == '0');
        int* hflag = nullptr;
        if (use_flag) {
            ctx->ws.expmv_stop.ensure();
            __atomic_store_n(ctx->ws.expmv_stop.host, -1, __ATOMIC_RELEASE);
            hflag = ctx->ws.expmv_stop.dev;
        }
        // Split form (large grids, terms of ~0.4 ms): the host keeps at most
        // 3 terms queued past the last finished one, so it sees a stage's
        // stop flag before it has queued the stage's remaining terms (each a
        // launch that returns at once, ~19 us with its check; ~2,000 of them
        // per config-4 trace_exp).
        const int ahead = (split && use_flag) ? 3 : 0;
        std::vector<hipEvent_t> ring(ahead, nullptr);
        for (auto& e : ring) KT_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        struct RingGuard {
            std::vector<hipEvent_t>& r;
            ~RingGuard() {
                for (hipEvent_t e : r)
                    if (e) (void)hipEventDestroy(e);
            }
        } ring_guard{ring};
        int64_t queued = 0;
        for (int i = 0; i < r.s; ++i) {
            KT_HIP(launch_inf_norm((int)n, nc, b.col(0), ld, part, st));   // c1 = norm(b, inf)
            KT_HIP(launch_expmv_begin(part, nb, state, st));
            double* cur = b.col(0);
            double* nxt = Ab.col(0);
            for (int k = 1; k <= r.m; ++k) {
                if (ahead && queued >= ahead) KT_HIP(hipEventSynchronize(ring[queued % ahead]));
                if (use_flag && k > 2 && __atomic_load_n(ctx->ws.expmv_stop.host, __ATOMIC_ACQUIRE) >= i) break;
                prof_begin(ctx, PROF_EXPMV, st, form);
                KT_HIP(launch_expmv_step(P, A->unit_values, V, M.med_rows, M.n_med, nc, ld, mu,
                                         t / ((double)r.s * k), tol, k, cur, nxt, F, state, st, form, hflag, i));
                prof_end(ctx, PROF_EXPMV, st);
                if ((form == 1 || form == 2) && k < r.m) KT_HIP(launch_expmv_slot_check(state, k, tol, st, hflag, i));
                if (ahead) KT_HIP(hipEventRecord(ring[queued % ahead], st));
                ++queued;
                std::swap(cur, nxt);
            }
            KT_HIP(launch_axpby((int)n, nc, eta, F, ld, 0.0, F, ld, st));  // f = eta f
            copy_cols(ctx, n, F, ld, b.col(0), ld, nc);                    // b = f
        }
        int hstate[2] = {0, 0};  // {active, mv}
        KT_HIP(hipMemcpyAsync(hstate, state, sizeof(hstate), hipMemcpyDeviceToHost, st));
        KT_HIP(hipStreamSynchronize(st));
        r.mv += hstate[1];
        ctx->expmv_terms += hstate[1];
        return r;
    }
    for (int i = 0; i < r.s; ++i) {
        KT_HIP(launch_inf_norm((int)n, nc, b.col(0), ld, part, st));   // c1 = norm(b, inf)
        KT_HIP(launch_expmv_begin(part, nb, state, st));
        for (int k = 1; k <= r.m; ++k) {
            spmm_slices(A, b.col(0), ld, Ab.col(0), ld, nc, static_cast<const int*>(state));
            KT_HIP(launch_expmv_term((int)n, nc, mu, t / ((double)r.s * k), Ab.col(0), b.col(0), F, ld,
                                     part, state, st));
            KT_HIP(launch_expmv_check((int)n, part, tol, state, st));
        }
        KT_HIP(launch_axpby((int)n, nc, eta, F, ld, 0.0, F, ld, st));  // f = eta f
        copy_cols(ctx, n, F, ld, b.col(0), ld, nc);                    // b = f
    }
    int hstate[2] = {0, 0};  // {active, mv}
    KT_HIP(hipMemcpyAsync(hstate, state, sizeof(hstate), hipMemcpyDeviceToHost, st));
    KT_HIP(hipStreamSynchronize(st));
    r.mv += hstate[1];
    ctx->expmv_terms += hstate[1];
    return r;
}

// The Afun handle of mc_trace on device blocks (n x ld, nc <= ld columns).
struct AfunDev {
    kt_matrix_s* A;
    int kind, fun, m;
    void apply(const double* X, int ld, int nc, double* Y) {
        switch (kind) {
        case AFUN_MATRIX: spmm(A, X, ld, Y, ld, nc); break;
        case AFUN_LANCZOS: lanczos_columns(A, X, ld, nc, m, fun, nullptr, Y, ld); break;
        default: expmv_device(A, 1.0, X, ld, nc, Y); break;
        }
    }
    // q[c] = x_c' F(x_c), c < nc
    void quad_cols(const double* X, int ld, int nc, double* q) {
        if (kind == AFUN_LANCZOS) {
            lanczos_columns(A, X, ld, nc, m, fun, q, nullptr, 0);
            return;
        }
        DevMat Y;
        Y.alloc(A->ctx, A->n, ld);
        apply(X, ld, nc, Y.col(0));
        std::vector<double> G;
        gram(A->ctx, A->n, X, ld, nc, Y.col(0), ld, nc, G);
        for (int c = 0; c < nc; ++c) q[c] = G[c + (size_t)c * nc];
    }
    // sum_c x_c' F(x_c), summed in column order
    double trace_quad(const double* X, int ld, int nc) {
        std::vector<double> q(nc);
        quad_cols(X, ld, nc, q.data());
        double s = 0.0;
        for (double v : q) s += v;
        return s;
    }
};

// Multi-GPU form of mc_trace: every rank recomputes S, Q
// and tr(Q' Afun Q) from the shared seed; the G term's columns are dealt
// round-robin (column c to rank c % world) and their quadratic forms
// summed by one all-reduce of the 10-vector, then added in column order
// on every rank.  expmv picks its Taylor degree from the whole block
// (expmv.m:41), so that Afun stays replicated.
struct Shard {
    int rank = 0, world = 1;
    kt_reduce_fn allreduce = nullptr;
    void* user = nullptr;
};

// X <- X - Q (Q' X) with separate leading dimensions for Q and X (the
// deflation aux of mc_trace.m:47): the Gram block stays on the device and
// the combine reads it in stream order -- no host round trip per projection
static void project_ld(kt_context_s* ctx, int64_t n, const double* Q, int ldq, int nq, double* X, int ldx,
                       int nc) {
    if (nc <= 0 || nq <= 0) return;
    const double* dG = gram_device(ctx, n, Q, ldq, nq, X, ldx, nc);
    combine_device(ctx, n, Q, ldq, nq, dG, nc, -1.0, 1.0, X, ldx);
}

// X <- X - Q (Q' X)  on nc columns, one leading dimension
static void project(kt_context_s* ctx, int64_t n, const double* Q, int ld, int nq, double* X, int nc) {
    project_ld(ctx, n, Q, ld, nq, X, ld, nc);
}

// mc_trace.m:42-58 with the Lanczos-f Afun, one batch of sweeps per round.
// The round's Q term (:46), its G term (:49) and the NEXT round's S term
// (:43-45, which needs only Q_1..Q_it) are independent Afun calls, so their
// 30 columns are queued together on two lanes: the 10 S columns, whose
// f(A) x feeds the next qr (:45), by the explicit sweep with its basis, 16
// wide, its 6 spare slots taking Q's leading columns (Q_1's first column is
// the top eigenvector to rounding: a lucky breakdown the y-form's guard
// would send to a redo); Q's other 4 columns and G -- quadratic forms only --
// by a 16-wide y-form sweep beside it.  Config 4: 41.8 ms per trace_exp vs
// 43.1 with all 30 columns in two explicit sweeps and 46.6 in one 32-wide
// explicit sweep, whose 256 MB gathered table fills the Infinity Cache
// (profiles/r05/mc_ahead_ab, profiles/r05/sweep_plan_ab).  Round 1's S term
// runs alone.
//
// The next round's S term is computed ahead in round `it` unless the round
// is expected to stop the loop: |trace(G' Afun G)/m| of the previous round
// below tol |tr_new| (the deflated remainder is already below the stopping
// tolerance; on the config-4 graph, rank one to 1e-23, round 2 always
// stops).  Such a round runs only its Q and G terms (:46, :49), quadratic
// forms both, by y-form sweeps (one pass per Lanczos step, no K2 stream) on
// two lanes.  A wrong guess moves the S term to the start of the next round;
// mc_trace never stops in round 1 (tr_old = 0), so round 2's S term is always
// computed ahead.
//
// Multi-GPU (sh.allreduce set): S and Q replicated, G column c on rank
// c % world in one of 10 fixed G slots (the others zero), the 10 G forms
// all-reduced once per round and summed in column order.  The sweep widths
// depend only on the slot layout and on the guess (made from all-reduced
// sums, the same on every rank), never on the rank count, so every world size
// gives the world-1 estimate bit for bit.
// y-form sweep chunk of a round that does not compute the next S term (its
// 10 Q and 10 G columns, forms only): KT_MC_YCHUNK (A/B), default 16 (16 + 4)
static int mc_final_chunk() {
    const char* e = getenv("KT_MC_YCHUNK");
    return e ? std::max(1, std::min(16, atoi(e))) : 16;
}

static void mc_trace_batched(kt_matrix_s* A, const AfunDev& F, double tol, int maxit, uint64_t seed,
                             double* tr_out, double* res_out, int* it_out, const Shard& sh) {
    kt_context_s* ctx = A->ctx;
    hipStream_t st = ctx->stream;
    const int64_t n = A->n;
    const int mb = 10, ld = 16, LB = 32;
    const int K = (maxit + 3 * mb - 1) / (3 * mb);  // :41
    double tr = 0.0, tr_old = 0.0, tr_new = 0.0, res = 1.0;
    std::vector<DevMat> Qs;
    DevMat Bk, Yb;
    Bk.alloc(ctx, n, LB);  // [S_{it+1} | P..P Q_it | P..P G_it (10 slots) | 0 0]
    Yb.alloc(ctx, n, ld);  // Afun_it(S_it), then Q_it in place
    auto rademacher_into = [&](int64_t base, double* dst) {  // probes base .. base + 9 into their slots
        KT_HIP(launch_rademacher_cols((int)n, mb, seed, base, dst, LB, st));
    };
    // S term of round itx: Y = F(P_{itx-1}..P_1 S_itx) into Yb (unprojected)
    // The S term alone (round 1, or a round whose guess was wrong): its 10
    // columns need f(A) x, so their sweep keeps the Lanczos basis.
    // KT_MC_YBASIS=1 forms it with the y-form pass itself (KF_VB: one gather
    // pass per step instead of K1 + K2; a tripped column redoes the sweep
    // explicitly).  Measured at config 4 (round 6, profiles/r06/mc_ybasis_ab):
    // 42.1 vs 41.7 ms per trace_exp -- the three basis streams and the
    // P-wide slots' weighted sum cost what K2 saved on a lone sweep -- so the
    // explicit sweep stays the default.
    const char* ybe = getenv("KT_MC_YBASIS");
    const int yb_cols = (ybe && ybe[0] == '1') ? mb : 0;
    auto s_term = [&](int itx) {
        rademacher_into((int64_t)(itx - 1) * 2 * mb, Bk.col(0));
        for (int k = (int)Qs.size() - 1; k >= 0; --k) project_ld(ctx, n, Qs[k].col(0), ld, mb, Bk.col(0), LB, mb);
        lanczos_columns_split(A, Bk.col(0), LB, mb, mb, mb, F.m, F.fun, nullptr, Yb.col(0), ld, 16, 16, yb_cols);
    };
    s_term(1);                                                             // :43-45
    std::vector<double> q(3 * mb);
    double gprev = INFINITY;  // |trace(G' Afun G)/m| of the previous round
    // KT_MC_AHEAD (tests): 1 always compute the next S term ahead, 0 never
    // (each round starts with its own), unset: the guess above
    const char* ae = getenv("KT_MC_AHEAD");
    const int ahead_mode = ae ? (ae[0] == '1' ? 1 : 0) : -1;
    int it = 0;
    for (it = 1; it <= K; ++it) {
        const int64_t base = (int64_t)(it - 1) * 2 * mb;
        std::vector<double> R;
        householder_qr(ctx, n, Yb.col(0), ld, mb, R);                      // [Q, ~] = qr(Afun(S), 0)
        // Q term input: P_{it-1}..P_1 Q_it                                   :46
        copy_cols(ctx, n, Yb.col(0), ld, Bk.col(mb), LB, mb);
        for (int k = (int)Qs.size() - 1; k >= 0; --k) project_ld(ctx, n, Qs[k].col(0), ld, mb, Bk.col(mb), LB, mb);
        Qs.emplace_back();                                                 // :47-48
        Qs.back().alloc(ctx, n, ld);
        copy_cols(ctx, n, Yb.col(0), ld, Qs.back().col(0), ld, mb);
        // G term input: P_it..P_1 G_it.  G column c sits in slot 2 mb + c at
        // every world size; a rank zeroes the slots of the other ranks' columns
        // (c % world != rank; a zero column's form is 0), so every column runs
        // in the same sweep at the same width whatever the rank count   :44, :49
        rademacher_into(base + mb, Bk.col(2 * mb));
        if (sh.world > 1)
            for (int c = 0; c < mb; ++c)
                if (c % sh.world != sh.rank) zero_cols(ctx, n, Bk.col(2 * mb + c), LB, 1);
        for (int k = (int)Qs.size() - 1; k >= 0; --k)
            project_ld(ctx, n, Qs[k].col(0), ld, mb, Bk.col(2 * mb), LB, mb);
        // next round's S term input: P_it..P_1 S_{it+1}, unless this round is
        // expected to stop
        const bool ahead = it < K && (ahead_mode == 1 || (ahead_mode < 0 && (it == 1 || !(gprev < tol * std::fabs(tr_new)))));
        if (ahead) {
            rademacher_into(base + 2 * mb, Bk.col(0));
            for (int k = (int)Qs.size() - 1; k >= 0; --k) project_ld(ctx, n, Qs[k].col(0), ld, mb, Bk.col(0), LB, mb);
            // [S | Q_0..5] explicit (16 wide, the basis for S) beside
            // [Q_6..9 | G] as a y-form sweep on a second lane
            lanczos_columns_split(A, Bk.col(0), LB, 3 * mb, mb, 16, F.m, F.fun, q.data(), Yb.col(0), ld, 16);
        } else {
            // no S term: the Q and G columns need quadratic forms only, so
            // both go through y-form sweeps (no K2, no basis), 16 wide on two
            // lanes.  (Round 1's Q_1 column 0 is the top eigenvector to
            // rounding -- a lucky breakdown at step 1 that the y-form guard
            // sends to the explicit redo -- but round 1 always computes the
            // S term ahead, so its Q columns ride the explicit sweeps.)
            lanczos_columns_split(A, Bk.col(mb), LB, 2 * mb, 0, 0, F.m, F.fun, q.data() + mb, nullptr, 0, 16,
                                  mc_final_chunk());
        }
        std::vector<double> qv(mb, 0.0);
        for (int c = sh.rank; c < mb; c += sh.world) qv[c] = q[2 * mb + c];
        if (sh.allreduce && sh.allreduce(qv.data(), mb, sh.user) != 0)
            fail(KT_ERR_CALLBACK, "mc_trace: all-reduce callback failed");
        double qsum = 0.0, gsum = 0.0;  // column order, as trace_quad sums
        for (int c = 0; c < mb; ++c) qsum += q[mb + c];
        for (double v : qv) gsum += v;
        tr += qsum;
        tr_new = tr + gsum / mb;                                           // :49
        gprev = std::fabs(gsum / mb);
        res = std::fabs(tr_new - tr_old) / std::max(std::fabs(tr_new), std::fabs(tr_old));  // :50
        if (res < tol) break;                                              // :54-56
        tr_old = tr_new;
        if (it < K) {
            if (!ahead) s_term(it + 1);  // the guess was wrong: the S term now
            // Y_{it+1} = P_1..P_it F(P_it..P_1 S_{it+1})                     :45, :48
            for (size_t k = 0; k < Qs.size(); ++k) project_ld(ctx, n, Qs[k].col(0), ld, mb, Yb.col(0), ld, mb);
        }
    }
    if (it > K) it = K;
    *tr_out = tr_new;
    if (res_out) *res_out = res;
    if (it_out) *it_out = it;
}

// mc_trace.m:1-63
//
// Round it + 1's S term -- Afun_{it+1}(S_{it+1}) = P_it..P_1 F(P_1..P_it S_{it+1})
// (:43-45) -- needs only the Q blocks up to round it, not the round's trace
// sums, so it runs speculatively on a third device copy of A (the twin's
// twin: own stream, workspace and matrix) on a third host thread while the
// round's Q and G terms run (:46, :49).  mc_trace never stops in round 1
// (tr_old = 0), so round 2's S term is never wasted; a later one is discarded
// when the round's relative change stops the loop.  Same kernels on the same
// data: the estimate is bit-identical to the serial order (KT_MC_SPEC=0).
void mc_trace_impl(kt_matrix_s* A, AfunDev& F, double tol, int maxit, int isAreal, uint64_t seed,
                   double* tr_out, double* res_out, int* it_out, const Shard& sh = Shard()) {
    kt_context_s* ctx = A->ctx;
    const int64_t n = A->n;
    const char* be = getenv("KT_MC_BATCH");
    if (F.kind == AFUN_LANCZOS && !(be && be[0] == '0')) {
        mc_trace_batched(A, F, tol, maxit, seed, tr_out, res_out, it_out, sh);
        return;
    }
    const int mb = 10, ld = 16;                    // :36
    const int K = (maxit + 3 * mb - 1) / (3 * mb);  // :41 ceil(maxit/30)
    double tr = 0.0, tr_old = 0.0, tr_new = 0.0, res = 1.0;
    std::vector<DevMat> Qs;
    DevMat S, G, Z, Y, Zg2;
    // G columns dealt over the ranks whenever the caller supplied the
    // all-reduce (at world 1 too: rank 0 takes every column, the sums still
    // travel through the collective); expmv stays replicated
    const bool sharded = sh.allreduce != nullptr && F.kind != AFUN_EXPMV;
    const char* se = getenv("KT_MC_SPEC");
    kt_matrix_s* A3 = nullptr;  // the speculative S terms' matrix
    if (!sharded && K > 1 && !(se && se[0] == '0')) {
        kt_matrix_s* A2 = twin_of(A);
        if (A2) A3 = twin_of(A2);
    }
    // the S-term output blocks (round parity) and the speculative run's
    // scratch, allocated once on A3's context: never re-allocated while the
    // speculative thread may use that context's pool
    DevMat Yb[2], S3, Z3;
    if (A3) {
        for (auto& b : Yb) b.alloc(A3->ctx, n, ld);
        S3.alloc(A3->ctx, n, ld);
        Z3.alloc(A3->ctx, n, ld);
        KT_HIP(hipStreamSynchronize(A3->ctx->stream));
        KT_HIP(hipSetDevice(ctx->device));
    }
    // Y = Afun_itx(S_itx) into Yx on AX's stream (the matrix F works on)
    auto s_term = [&](kt_matrix_s* AX, int itx, DevMat& Sx, DevMat& Zx, double* Yx) {
        kt_context_s* cx = AX->ctx;
        const int64_t base = (int64_t)(itx - 1) * 2 * mb;
        KT_HIP(launch_rademacher(ld, (int)n, seed, base, nullptr, Sx.col(0), cx->stream));  // :43
        zero_cols(cx, n, Sx.col(mb), ld, ld - mb);
        copy_cols(cx, n, Sx.col(0), ld, Zx.col(0), ld, mb);
        for (int q = itx - 2; q >= 0; --q) project(cx, n, Qs[q].col(0), ld, mb, Zx.col(0), mb);
        AfunDev FX{AX, F.kind, F.fun, F.m};
        FX.apply(Zx.col(0), ld, mb, Yx);
        for (int q = 0; q <= itx - 2; ++q) project(cx, n, Qs[q].col(0), ld, mb, Yx, mb);
    };
    bool spec_ready = false;  // this round's S term was computed by the speculative thread
    int it = 0;
    for (it = 1; it <= K; ++it) {
        const int64_t base = (int64_t)(it - 1) * 2 * mb;
        G.alloc(ctx, n, ld);
        KT_HIP(launch_rademacher(ld, (int)n, seed, base + mb, nullptr, G.col(0), ctx->stream));  // :44
        zero_cols(ctx, n, G.col(mb), ld, ld - mb);
        Z.alloc(ctx, n, ld);
        double* Yc;
        if (A3) {
            Yc = Yb[it & 1].col(0);
        } else {
            Y.alloc(ctx, n, ld);
            Yc = Y.col(0);
        }
        if (!spec_ready) {  // Y = Afun_it(S) = P_{it-1}..P_1 F(P_1..P_{it-1} S)          :45
            S.alloc(ctx, n, ld);
            s_term(A, it, S, Z, Yc);
        }
        spec_ready = false;
        std::vector<double> R;
        householder_qr(ctx, n, Yc, ld, mb, R);                                     // [Q, ~] = qr(.,0)
        // tr += trace(Q' Afun_it(Q)) = sum quadforms of P_1..P_{it-1} Q          :46
        copy_cols(ctx, n, Yc, ld, Z.col(0), ld, mb);
        for (int q = (int)Qs.size() - 1; q >= 0; --q) project(ctx, n, Qs[q].col(0), ld, mb, Z.col(0), mb);
        const bool split = !sharded;  // the G term is local
        kt_matrix_s* A2 = split ? twin_of(A) : nullptr;
        if (!A2) tr += F.trace_quad(Z.col(0), ld, mb);
        Qs.emplace_back();                                                         // :47-48
        Qs.back().alloc(ctx, n, ld);
        copy_cols(ctx, n, Yc, ld, Qs.back().col(0), ld, mb);
        // tr_new = tr + trace(G' Afun_{it+1}(G)) / m                              :49
        DevMat& Zg = A2 ? Zg2 : Z;
        if (A2) Zg.alloc(ctx, n, ld);
        copy_cols(ctx, n, G.col(0), ld, Zg.col(0), ld, mb);
        for (int q = (int)Qs.size() - 1; q >= 0; --q) project(ctx, n, Qs[q].col(0), ld, mb, Zg.col(0), mb);
        double gsum = 0.0;
        if (A2) {
            // The two quadratures of the round are independent Afun calls:
            // the G term runs on the matrix's twin (own stream, workspace and
            // device copy; kt_krylov.cpp twin_of) on a second host thread
            // while the Q term runs here -- same kernels on the same data,
            // so the sums are bit-identical to the serial order.  The next
            // round's S term (see above) starts on a third thread.
            KT_HIP(hipStreamSynchronize(ctx->stream));  // Z, Zg and Q_it are ready for every stream
            Status gerr{KT_OK, ""}, serr{KT_OK, ""};
            // persistent threads of this context (kt_worker.h): finished on
            // every exit path before the captured locals go out of scope
            RunWorker tg, ts;
            tg.reset(ctx_worker(ctx, kWorkerTwin));
            tg->submit([&] {
                try {
                    KT_HIP(hipSetDevice(A2->ctx->device));
                    AfunDev F2{A2, F.kind, F.fun, F.m};
                    gsum = F2.trace_quad(Zg.col(0), ld, mb);
                    KT_HIP(hipStreamSynchronize(A2->ctx->stream));
                } catch (const Status& e) {
                    gerr = e;
                } catch (...) {
                    gerr = Status{KT_ERR_HIP, "mc_trace: G term on the twin failed"};
                }
            });
            if (A3 && it < K) {
                ts.reset(ctx_worker(ctx, kWorkerSpec));
                ts->submit([&] {
                    try {
                        KT_HIP(hipSetDevice(A3->ctx->device));
                        s_term(A3, it + 1, S3, Z3, Yb[(it + 1) & 1].col(0));
                        KT_HIP(hipStreamSynchronize(A3->ctx->stream));
                    } catch (const Status& e) {
                        serr = e;
                    } catch (...) {
                        serr = Status{KT_ERR_HIP, "mc_trace: speculative S term failed"};
                    }
                });
            }
            const double qsum = F.trace_quad(Z.col(0), ld, mb);  // (on a throw, tg / ts finish first)
            tg->wait(0);
            if (ts) {
                ts->wait(0);
                if (serr.code == KT_OK) {
                    spec_ready = true;
                } else if (serr.code != KT_ERR_ALLOC) {
                    throw serr;
                }  // out of memory: the next round computes its S term here
                (void)hipGetLastError();
                KT_HIP(hipSetDevice(ctx->device));
            }
            if (gerr.code == KT_ERR_ALLOC) {
                // the twin's workspace did not fit: give its idle blocks back
                // and run the G term in the serial order on A (as
                // fun_and_grad_krylov_fun does, kt_krylov.cpp)
                (void)hipGetLastError();
                A2->ctx->pool.clear();
                KT_HIP(hipSetDevice(ctx->device));
                gsum = F.trace_quad(Zg.col(0), ld, mb);
            } else if (gerr.code != KT_OK) {
                throw gerr;
            }
            tr += qsum;
        } else if (sharded) {
            std::vector<double> qv(mb, 0.0), qm;
            int nm = 0;
            for (int c = sh.rank; c < mb; c += sh.world) copy_cols(ctx, n, Z.col(c), ld, Yc + nm++, ld, 1);
            if (nm > 0) {
                zero_cols(ctx, n, Yc + nm, ld, ld - nm);
                qm.assign(nm, 0.0);
                F.quad_cols(Yc, ld, nm, qm.data());
                for (int c = sh.rank, t = 0; c < mb; c += sh.world, ++t) qv[c] = qm[t];
            }
            if (sh.allreduce(qv.data(), mb, sh.user) != 0) fail(KT_ERR_CALLBACK, "mc_trace: all-reduce callback failed");
            for (double v : qv) gsum += v;
        } else {
            gsum = F.trace_quad(Z.col(0), ld, mb);
        }
        tr_new = tr + gsum / mb;
        res = std::fabs(tr_new - tr_old) / std::max(std::fabs(tr_new), std::fabs(tr_old));  // :50
        if (res < tol) break;                                                      // :54-56
        tr_old = tr_new;
    }
    if (it > K) it = K;
    (void)isAreal;  // :60-62 real part: the device estimator is real
    *tr_out = tr_new;
    if (res_out) *res_out = res;
    if (it_out) *it_out = it;
}

}  // namespace kt

using namespace kt;

#define KT_TRY try {
#define KT_CATCH                                  \
    }                                             \
    catch (const kt::Status& s) {                 \
        kt::set_error(s.msg);                     \
        return s.code;                            \
    }                                             \
    catch (const std::exception& e) {             \
        kt::set_error(e.what());                  \
        return KT_ERR_ARG;                        \
    }                                             \
    return KT_OK;

extern "C" {

int kt_mc_trace(kt_matrix_t A, int afun, int fun, int m, double tol, int maxit, int isAreal,
                uint64_t seed, double* tr, double* res, int* it) {
    KT_TRY
    if (!A || !tr) fail(KT_ERR_ARG, "NULL argument");
    if (afun < AFUN_MATRIX || afun > AFUN_EXPMV) fail(KT_ERR_ARG, "unknown Afun kind");
    if (fun < KT_FUN_EXP || fun > KT_FUN_SQRT) fail(KT_ERR_ARG, "unknown fun code");
    if (afun == AFUN_LANCZOS && (m < 1 || m > 256)) fail(KT_ERR_ARG, "m must be in [1, 256]");
    if (maxit < 1) fail(KT_ERR_ARG, "maxit must be >= 1");
    if (A->n < 10) fail(KT_ERR_UNSUPPORTED, "mc_trace needs n >= 10 (qr of an n x 10 block)");
    KT_HIP(hipSetDevice(A->ctx->device));
    AfunDev F{A, afun, fun, m};
    mc_trace_impl(A, F, tol, maxit, isAreal, seed, tr, res, it);
    KT_CATCH
}

int kt_mc_trace_sharded(kt_matrix_t A, int afun, int fun, int m, double tol, int maxit, int isAreal,
                        uint64_t seed, int rank, int world, kt_reduce_fn allreduce, void* user,
                        double* tr, double* res, int* it) {
    KT_TRY
    if (!A || !tr) fail(KT_ERR_ARG, "NULL argument");
    if (world < 1 || rank < 0 || rank >= world) fail(KT_ERR_ARG, "bad rank / world");
    if (world > 1 && !allreduce) fail(KT_ERR_ARG, "world > 1 needs an all-reduce callback");
    if (afun < AFUN_MATRIX || afun > AFUN_EXPMV) fail(KT_ERR_ARG, "unknown Afun kind");
    if (fun < KT_FUN_EXP || fun > KT_FUN_SQRT) fail(KT_ERR_ARG, "unknown fun code");
    if (afun == AFUN_LANCZOS && (m < 1 || m > 256)) fail(KT_ERR_ARG, "m must be in [1, 256]");
    if (maxit < 1) fail(KT_ERR_ARG, "maxit must be >= 1");
    if (A->n < 10) fail(KT_ERR_UNSUPPORTED, "mc_trace needs n >= 10 (qr of an n x 10 block)");
    KT_HIP(hipSetDevice(A->ctx->device));
    AfunDev F{A, afun, fun, m};
    Shard sh{rank, world, allreduce, user};
    mc_trace_impl(A, F, tol, maxit, isAreal, seed, tr, res, it, sh);
    KT_CATCH
}

int kt_trace_exp(kt_matrix_t A, int afun, int m, uint64_t seed, double* tr) {
    KT_TRY
    if (!A || !tr) fail(KT_ERR_ARG, "NULL argument");
    if (afun != AFUN_LANCZOS && afun != AFUN_EXPMV) fail(KT_ERR_ARG, "trace_exp: Afun must be Lanczos or expmv");
    if (A->n < 10) fail(KT_ERR_UNSUPPORTED, "trace_exp needs n >= 10");
    KT_HIP(hipSetDevice(A->ctx->device));
    AfunDev F{A, afun, KT_FUN_EXP, m};
    mc_trace_impl(A, F, 1e-4, 1000, 1, seed, tr, nullptr, nullptr);  // trace_exp.m:5-6
    KT_CATCH
}

int kt_expmv(kt_matrix_t A, double t, int64_t ncols, const double* B, double* F, int* s, int* mdeg,
             int* mv) {
    KT_TRY
    if (!A || !B || !F || ncols < 1 || ncols > 128) fail(KT_ERR_ARG, "bad argument (1 <= ncols <= 128)");
    KT_HIP(hipSetDevice(A->ctx->device));
    const int ld = pow2_at_least((int)ncols);
    DevMat Bd, Fd;
    Bd.alloc(A->ctx, A->n, ld);
    Fd.alloc(A->ctx, A->n, ld);
    upload_rows(A, B, (int)ncols, Bd.col(0), ld);
    Expmv r = expmv_device(A, t, Bd.col(0), ld, (int)ncols, Fd.col(0));
    download_block(A, Fd.col(0), ld, (int)ncols, F);
    if (s) *s = r.s;
    if (mdeg) *mdeg = r.m;
    if (mv) *mv = r.mv;
    KT_CATCH
}

int kt_lanczos_fmv(kt_matrix_t A, int fun, int m, int64_t ncols, const double* X, double* Y) {
    KT_TRY
    if (!A || !X || !Y || ncols < 1 || ncols > 128) fail(KT_ERR_ARG, "bad argument (1 <= ncols <= 128)");
    if (fun < KT_FUN_EXP || fun > KT_FUN_SQRT) fail(KT_ERR_ARG, "unknown fun code");
    if (m < 1 || m > 256) fail(KT_ERR_ARG, "m must be in [1, 256]");
    KT_HIP(hipSetDevice(A->ctx->device));
    const int ld = pow2_at_least((int)ncols);
    DevMat Xd, Yd;
    Xd.alloc(A->ctx, A->n, ld);
    Yd.alloc(A->ctx, A->n, ld);
    upload_rows(A, X, (int)ncols, Xd.col(0), ld);
    lanczos_columns(A, Xd.col(0), ld, (int)ncols, m, fun, nullptr, Yd.col(0), ld);
    download_block(A, Yd.col(0), ld, (int)ncols, Y);
    KT_CATCH
}

}  // extern "C"

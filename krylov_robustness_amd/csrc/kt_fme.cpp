// kt_fme.cpp -- function_multiple_entries.m on the device, and the
// column-batched single-vector Arnoldi engine (ColArnoldi) it shares with
// multiple_frechet_eval.m (kt_frechet.cpp).
//
// f(A)(i, j) for every (i, j) of omega by one single-vector Arnoldi run per
// distinct row index i (arnoldi_krylov.m with bs = 1, started at e_i), all
// runs of a group of <= 128 rows advanced together: one SpMM over the group's
// columns per step, column-batched CGS2 / Householder / reorthogonalisation
// kernels (kt_colbatch.hip), and per-entry host work on the j x j projected
// matrices with the reference's lag-3 stopping rule
// (function_multiple_entries.m:112-156).
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <unordered_map>

#include "kt_colarnoldi.h"
#include "kt_pool.h"
#include "kt_launch.h"

namespace kt {

void ColArnoldi::init_buffers() {
    if (C_ < 1 || C_ > 128) fail(KT_ERR_UNSUPPORTED, "ColArnoldi: 1..128 columns");
    P_ = pow2_at_least(C_);
    vs_ = n_ * (int64_t)P_;
    basis_.ensure(sizeof(double) * (size_t)vs_ * (it_ + 1));
    W_.ensure(sizeof(double) * (size_t)vs_);
    nrb_ = col_nrb((int)n_, ctx_->num_cu, rpb_lo_);
    part_.ensure(sizeof(double) * (size_t)nrb_ * P_ * (it_ + 1));
    // red: h1 | h2 | hh (it x P each) | s (P) | r (P)
    red_.ensure(sizeof(double) * ((size_t)3 * it_ * P_ + 2 * P_));
    KT_HIP(hipMemsetAsync(basis_.ptr, 0, sizeof(double) * (size_t)vs_, ctx_->stream));
    H_.assign(C_, std::vector<double>((size_t)(it_ + 1) * it_, 0.0));
}

// [V, ~] = qr(start block, 0)   (arnoldi_krylov.m:50)
void ColArnoldi::start_qr() {
    double* V = basis_.as<double>();
    double* sq = red_.as<double>() + (size_t)3 * it_ * P_;
    double* rr = sq + P_;
    KT_HIP(launch_col_dots((int)n_, P_, 1, 0, V, V, 1, ctx_->num_cu, part_.as<double>(), sq, ctx_->stream, rpb_lo_));
    KT_HIP(launch_col_householder((int)n_, P_, sq, V, V, rr, ctx_->stream));
}

ColArnoldi::ColArnoldi(kt_matrix_s* A, const std::vector<int64_t>& starts, int it)
    : A_(A), ctx_(A->ctx), n_(A->n), C_((int)starts.size()), it_(it), rpb_lo_(32) {
    init_buffers();
    std::vector<int> ridx(starts.begin(), starts.end());
    idx_.ensure(sizeof(int) * ridx.size());
    double* V = basis_.as<double>();
    KT_HIP(hipMemcpyAsync(idx_.ptr, ridx.data(), sizeof(int) * ridx.size(), hipMemcpyHostToDevice,
                          ctx_->stream));
    KT_HIP(launch_col_select(C_, P_, idx_.as<int>(), V, ctx_->stream));
    start_qr();
    std::vector<int64_t> off(C_);
    for (int c = 0; c < C_; ++c) off[c] = starts[c] * P_ + c;
    download_elems(ctx_, V, off, uaux_);
}

ColArnoldi::ColArnoldi(kt_matrix_s* A, const double* X, int C, int it)
    : A_(A), ctx_(A->ctx), n_(A->n), C_(C), it_(it) {
    init_buffers();
    std::vector<double> rm((size_t)n_ * P_, 0.0);
    for (int c = 0; c < C_; ++c)
        for (int64_t i = 0; i < n_; ++i) rm[(size_t)i * P_ + c] = X[i + (size_t)c * n_];
    KT_HIP(hipMemcpyAsync(basis_.ptr, rm.data(), sizeof(double) * rm.size(), hipMemcpyHostToDevice,
                          ctx_->stream));
    start_qr();
    uaux_.assign(C_, 0.0);
    KT_HIP(hipStreamSynchronize(ctx_->stream));
}

void ColArnoldi::combine(const std::vector<double>& y, int nk, double* out) {
    // W = 0; W -= V (-y)  (the column update kernel with negated weights)
    std::vector<double> hy((size_t)nk * P_, 0.0);
    for (int k = 0; k < nk; ++k)
        for (int c = 0; c < C_; ++c) hy[(size_t)k * P_ + c] = -y[(size_t)k * C_ + c];
    double* dh = red_.as<double>();  // h1 slab, it x P >= nk x P
    if (nk > it_) fail(KT_ERR_ARG, "ColArnoldi::combine: too many blocks");
    KT_HIP(hipMemcpyAsync(dh, hy.data(), sizeof(double) * hy.size(), hipMemcpyHostToDevice, ctx_->stream));
    KT_HIP(hipMemsetAsync(W_.ptr, 0, sizeof(double) * (size_t)vs_, ctx_->stream));
    KT_HIP(launch_col_update((int)n_, P_, nk, vs_, basis_.as<double>(), dh, W_.as<double>(), ctx_->stream));
    std::vector<double> rm((size_t)n_ * P_);
    KT_HIP(hipMemcpyAsync(rm.data(), W_.ptr, sizeof(double) * rm.size(), hipMemcpyDeviceToHost, ctx_->stream));
    KT_HIP(hipStreamSynchronize(ctx_->stream));
    for (int c = 0; c < C_; ++c)
        for (int64_t i = 0; i < n_; ++i) out[i + (size_t)c * n_] = rm[(size_t)i * P_ + c];
}

void ColArnoldi::step_launch() {
    if (pending_) fail(KT_ERR_UNSUPPORTED, "ColArnoldi: a step is already in flight");
    if (j_ >= it_) fail(KT_ERR_UNSUPPORTED, "ColArnoldi: step budget exhausted");
    const int j = ++j_;
    const int n = (int)n_;
    double* V = basis_.as<double>();
    double* W = W_.as<double>();
    double* h1 = red_.as<double>();
    double* h2 = h1 + (size_t)it_ * P_;
    double* hh = h2 + (size_t)it_ * P_;
    double* sq = hh + (size_t)it_ * P_;
    double* rr = sq + P_;
    double* part = part_.as<double>();
    double* Vj1 = V + (size_t)(j - 1) * vs_;
    double* Vj = V + (size_t)j * vs_;
    hipStream_t st = ctx_->stream;
    spmm(A_, Vj1, P_, W, P_, C_);  // w = A * V(:, end)   (arnoldi_krylov.m:86)
    // CGS2 against the whole basis (arnoldi_krylov.m:119-125)
    KT_HIP(launch_col_dots(n, P_, j, vs_, V, W, 0, ctx_->num_cu, part, h1, st, rpb_lo_));
    KT_HIP(launch_col_update(n, P_, j, vs_, V, h1, W, st));
    KT_HIP(launch_col_dots(n, P_, j, vs_, V, W, 0, ctx_->num_cu, part, h2, st, rpb_lo_));
    KT_HIP(launch_col_update(n, P_, j, vs_, V, h2, W, st));
    // [w, r] = qr(w, 0)   (:99)
    KT_HIP(launch_col_dots(n, P_, 1, 0, W, W, 1, ctx_->num_cu, part, sq, st, rpb_lo_));
    KT_HIP(launch_col_householder(n, P_, sq, W, Vj, rr, st));
    // reorthogonalise: hh = V' w; w = w - V hh   (:104-106)
    KT_HIP(launch_col_dots(n, P_, j, vs_, V, Vj, 0, ctx_->num_cu, part, hh, st, rpb_lo_));
    KT_HIP(launch_col_update(n, P_, j, vs_, V, hh, Vj, st));
    // h1 | h2 | hh (j x P each) | r (P) into pinned staging (one buffer: the
    // previous step was finished before this one was launched)
    const size_t jp = (size_t)j * P_;
    PinnedBuf& sg = ctx_->ws.pin_colarn;
    sg.ensure(sizeof(double) * (3 * jp + P_));
    double* s = sg.as<double>();
    KT_HIP(hipMemcpyAsync(s, h1, sizeof(double) * jp, hipMemcpyDeviceToHost, st));
    KT_HIP(hipMemcpyAsync(s + jp, h2, sizeof(double) * jp, hipMemcpyDeviceToHost, st));
    KT_HIP(hipMemcpyAsync(s + 2 * jp, hh, sizeof(double) * jp, hipMemcpyDeviceToHost, st));
    KT_HIP(hipMemcpyAsync(s + 3 * jp, rr, sizeof(double) * P_, hipMemcpyDeviceToHost, st));
    pending_ = true;
}

void ColArnoldi::step_finish() {
    if (!pending_) return;
    KT_HIP(hipStreamSynchronize(ctx_->stream));
    pending_ = false;
    const int j = j_;
    const size_t jp = (size_t)j * P_;
    const double* hb1 = ctx_->ws.pin_colarn.as<double>();
    const double* hb2 = hb1 + jp;
    const double* hbh = hb2 + jp;
    const double* rb = hbh + jp;
    const int Hld = it_ + 1;
    for (int c = 0; c < C_; ++c) {
        std::vector<double>& Hc = H_[c];
        const double r = rb[c];
        for (int k = 0; k < j; ++k)  // H(1:end-1, end) = h + hh * r   (:96, :106)
            Hc[k + (size_t)(j - 1) * Hld] =
                (hb1[(size_t)k * P_ + c] + hb2[(size_t)k * P_ + c]) + hbh[(size_t)k * P_ + c] * r;
        Hc[j + (size_t)(j - 1) * Hld] = r;  // H(end, end) = r   (:108)
    }
    done_ = j;
}

void ColArnoldi::gm(int c, std::vector<double>& G) const {
    const int j = done_, Hld = it_ + 1;
    G.resize((size_t)j * j);
    for (int b = 0; b < j; ++b)
        for (int a = 0; a < j; ++a) G[a + (size_t)b * j] = H_[c][a + (size_t)b * Hld];
}

void ColArnoldi::rows(const std::vector<int64_t>& rr, int nk, std::vector<double>& out) const {
    // one gather of every (row, block, column) element instead of a copy and
    // a sync per row
    std::vector<int64_t> off(rr.size() * (size_t)nk * C_);
    for (size_t ri = 0; ri < rr.size(); ++ri)
        for (int k = 0; k < nk; ++k)
            for (int c = 0; c < C_; ++c) off[(ri * nk + k) * C_ + c] = rr[ri] * P_ + (int64_t)k * vs_ + c;
    download_elems(ctx_, static_cast<const double*>(basis_.ptr), off, out);
}

void sym_eig_small(int j, const std::vector<double>& G, std::vector<double>& w,
                   std::vector<double>& V) {
    std::vector<double> S((size_t)j * j);
    for (int b = 0; b < j; ++b)
        for (int a = 0; a < j; ++a)
            S[a + (size_t)b * j] = 0.5 * (G[a + (size_t)b * j] + G[b + (size_t)a * j]);
    w.resize(j);
    V.resize((size_t)j * j);
    sym_eig_host(j, S.data(), w.data(), V.data());
}

namespace {

struct Entry {
    int64_t h;    // position in omega
    int col;      // column (distinct row index) within the group
    int64_t j2;   // omega(h, 2), 0-based
    std::vector<double> Xm;  // f(Gm) e1 at convergence / last step
    std::vector<double> stop[3];
    bool conv = false;
};

// f(G) e1 for the j x j Arnoldi projection G (column-major); G is symmetric
// up to rounding for symmetric A and is symmetrised first (the reference's
// expm/funm of the Hessenberg G agree to that rounding).
std::vector<double> fun_e1(int j, const std::vector<double>& G, int fun) {
    std::vector<double> w, V;
    sym_eig_small(j, G, w, V);
    std::vector<double> out(j, 0.0);
    for (int k = 0; k < j; ++k) {
        const double coef = fscalar(fun, w[k]) * V[0 + (size_t)k * j];
        for (int i = 0; i < j; ++i) out[i] += V[i + (size_t)k * j] * coef;
    }
    return out;
}

int run_group(kt_matrix_s* A, const std::vector<int64_t>& rows, std::vector<Entry>& ents, int fun,
              double tol, int it) {
    ColArnoldi ca(A, rows, it);
    const int C = ca.cols();
    std::vector<char> col_live(C, 1);
    const int d = 3;  // lag (function_multiple_entries.m:63)
    int j = 0;
    // step j's projections, f(G_c) e1 and the stop test run on the host while
    // the device runs step j + 1 (launched first; when step j says stop, that
    // step's basis block is never read: X uses blocks 0..j).  Same arithmetic
    // and order as step-then-host (KT_FME_PIPE=0), so the same results.
    const char* pe = getenv("KT_FME_PIPE");
    const bool pipe = !(pe && pe[0] == '0');
    if (pipe) ca.step();
    for (j = 1; j <= it; ++j) {
        if (!pipe) ca.step();
        else if (j < it) ca.step_launch();
        std::vector<std::vector<double>> F(C);
        std::vector<int> lc;  // live columns: f(G_c) e1 each, on the host worker pool
        for (int c = 0; c < C; ++c)
            if (col_live[c]) lc.push_back(c);
        HostPool::get().run((int)lc.size(), [&](int i) {
            std::vector<double> Gc;
            ca.gm(lc[i], Gc);
            F[lc[i]] = fun_e1(j, Gc, fun);
        }, 4);
        bool stop = true;  // :113-156
        for (Entry& e : ents) {
            if (e.conv) continue;
            e.Xm = F[e.col];
            if (j <= d) {
                e.stop[j - 1] = e.Xm;
                stop = false;
            } else {
                const std::vector<double>& old = e.stop[0];
                double err = 0.0;
                for (int i = 0; i < j; ++i) {
                    const double o = i < (int)old.size() ? old[i] : 0.0;
                    err += (e.Xm[i] - o) * (e.Xm[i] - o);
                }
                err = std::sqrt(err);
                if (err > tol) stop = false;
                else e.conv = true;
                e.stop[0] = std::move(e.stop[1]);
                e.stop[1] = std::move(e.stop[2]);
                e.stop[2] = e.Xm;
            }
        }
        if (stop) break;
        std::fill(col_live.begin(), col_live.end(), 0);
        for (const Entry& e : ents)
            if (!e.conv) col_live[e.col] = 1;
        if (pipe) ca.step_finish();
    }
    const int iter = std::min(j, it);
    // X(h) = Um(j2, 1:nn) * Xm(:, 1) * Uaux   (:163-165)
    std::vector<int64_t> need;
    std::unordered_map<int64_t, size_t> at;
    for (const Entry& e : ents)
        if (!at.count(e.j2)) {
            at.emplace(e.j2, need.size());
            need.push_back(e.j2);
        }
    std::vector<double> U;
    ca.rows(need, iter + 1, U);
    for (Entry& e : ents) {
        const size_t ri = at[e.j2];
        double x = 0.0;
        for (size_t i = 0; i < e.Xm.size(); ++i) x += U[(ri * (iter + 1) + i) * C + e.col] * e.Xm[i];
        e.Xm.assign(1, x * ca.uaux(e.col));
    }
    return iter;
}

}  // namespace

void function_multiple_entries_impl(kt_matrix_s* A, int64_t k, const int64_t* oi,
                                    const int64_t* oj, int fun, double tol, int it, double* X,
                                    int* iter_out) {
    const int64_t n = A->n;
    if (it <= 0) it = (int)std::min<int64_t>(100, n);  // :24-26
    for (int64_t h = 0; h < k; ++h)
        if (oi[h] < 0 || oi[h] >= n || oj[h] < 0 || oj[h] >= n)
            fail(KT_ERR_ARG, "omega index out of range");
    // I = unique(omega(:, 1), 'stable')   (:42)
    std::vector<int64_t> I;
    std::unordered_map<int64_t, int> pos;
    for (int64_t h = 0; h < k; ++h)
        if (!pos.count(oi[h])) {
            pos.emplace(oi[h], (int)I.size());
            I.push_back(oi[h]);
        }
    int iter = 0;
    for (size_t g0 = 0; g0 < I.size(); g0 += 128) {
        const size_t g1 = std::min(I.size(), g0 + 128);
        std::vector<int64_t> rows(I.begin() + g0, I.begin() + g1);
        std::vector<Entry> ents;
        for (int64_t h = 0; h < k; ++h) {
            const int p = pos[oi[h]];
            if (p < (int)g0 || p >= (int)g1) continue;
            Entry e;
            e.h = h;
            e.col = p - (int)g0;
            e.j2 = oj[h];
            ents.push_back(std::move(e));
        }
        iter = std::max(iter, run_group(A, rows, ents, fun, tol, it));
        for (const Entry& e : ents) X[e.h] = e.Xm[0];
    }
    if (iter_out) *iter_out = iter;
}

// Leading eigenpair of symmetric A (compute_centrality.m:15-17, eigs(A, 1)):
// full-reorthogonalisation Arnoldi (ColArnoldi) from the ones vector,
// explicitly restarted from the Ritz vector; stops when the Ritz residual
// |h(j+1, j) y(j)| <= tol |theta|.  v: unit 2-norm, sign fixed so sum(v) >= 0.
double eigs_leading_impl(kt_matrix_s* A, double tol, int maxit, double* v, int* steps_out) {
    const int64_t n = A->n;
    if (n == 0) return 0.0;
    if (tol <= 0.0) tol = 2.220446049250313e-16;
    const int m = (int)std::min<int64_t>(std::max(maxit > 0 ? maxit : 300, 2), std::max<int64_t>(n, 2));
    std::vector<double> x(n, 1.0), G, w, Q;
    double theta = 0.0;
    int total = 0;
    for (int restart = 0; restart < 20; ++restart) {
        ColArnoldi ca(A, x.data(), 1, std::min<int64_t>(m, n));
        int j = 0;
        bool conv = false;
        std::vector<double> y;
        for (j = 1; j <= ca.steps() + 1 && j <= std::min<int64_t>(m, n); ++j) {
            ca.step();
            ca.gm(0, G);
            sym_eig_small(j, G, w, Q);
            theta = w[j - 1];
            y.assign(Q.begin() + (size_t)(j - 1) * j, Q.begin() + (size_t)j * j);
            const double res = std::fabs(ca.h(0, j, j - 1) * y[j - 1]);
            if (res <= tol * std::fabs(theta) || j == n) {
                conv = true;
                break;
            }
        }
        if (j > ca.steps()) j = ca.steps();
        total += j;
        ca.combine(y, j, x.data());
        double nrm = 0.0, sum = 0.0;
        for (double t : x) {
            nrm += t * t;
            sum += t;
        }
        nrm = std::sqrt(nrm);
        const double sg = sum < 0.0 ? -1.0 : 1.0;
        for (double& t : x) t *= sg / nrm;
        if (conv) break;
    }
    if (v) std::copy(x.begin(), x.end(), v);
    if (steps_out) *steps_out = total;
    return theta;
}

}  // namespace kt

using namespace kt;

extern "C" int kt_eigs_leading(kt_matrix_t A, double tol, int maxit, double* lambda, double* v,
                               int* steps) {
    try {
        if (!A || !lambda) fail(KT_ERR_ARG, "NULL argument");
        KT_HIP(hipSetDevice(A->ctx->device));
        require_symmetric(A, "EIGS:: symmetric A required");
        *lambda = eigs_leading_impl(A, tol, maxit, v, steps);
    } catch (const Status& s) {
        set_error(s.msg);
        return s.code;
    } catch (const std::bad_alloc&) {
        set_error("host allocation failed");
        return KT_ERR_ALLOC;
    }
    return KT_OK;
}

extern "C" int kt_function_multiple_entries(kt_matrix_t A, int64_t k, const int64_t* oi,
                                            const int64_t* oj, int fun, double tol, int it,
                                            double* X, int* iter) {
    try {
        if (!A || !X || (k > 0 && (!oi || !oj))) fail(KT_ERR_ARG, "NULL argument");
        if (k < 0) fail(KT_ERR_ARG, "negative entry count");
        if (fun < KT_FUN_EXP || fun > KT_FUN_SQRT) fail(KT_ERR_UNSUPPORTED, "unsupported function");
        KT_HIP(hipSetDevice(A->ctx->device));
        function_multiple_entries_impl(A, k, oi, oj, fun, tol, it, X, iter);
    } catch (const Status& s) {
        set_error(s.msg);
        return s.code;
    } catch (const std::bad_alloc&) {
        set_error("host allocation failed");
        return KT_ERR_ALLOC;
    }
    return KT_OK;
}

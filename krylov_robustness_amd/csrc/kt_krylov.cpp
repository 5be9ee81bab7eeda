// kt_krylov.cpp -- block Lanczos / block Arnoldi and the low-rank-update
// entry points on the device:
//   lanczos_krylov.m   -> BlockLanczos   (2-block window, CGS2, thin QR)
//   arnoldi_krylov.m   -> BlockArnoldi   (full basis, CGS2 + reorthogonalise)
//   trace_fun_update.m -> kt_trace_fun_update
//   fun_update.m       -> kt_fun_update (Arnoldi branch, nargout == 4)
//   fun_and_grad_krylov_exp.m / _fun.m -> kt_fun_and_grad_krylov_exp / _fun
//   MATLAB normest     -> kt_normest
// Device work: SpMM (HIP kernel), Gram / combine (rocBLAS dgemm), CholQR.
// Host work: the small projected matrices (H, Cm, eig, f(.)) -- exactly the
// quantities the reference forms with dense MATLAB built-ins.
#include <rocsolver/rocsolver.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <exception>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>

#include "kt_krylov.h"
#include "kt_launch.h"
#include "kt_pool.h"
#include "kt_worker.h"

namespace kt {

// ---------------------------------------------------------------------------
// dense symmetric eig: host tred2/tql2 for small n, rocSOLVER dsyevd above.
// ---------------------------------------------------------------------------
struct EigStats {
    int64_t calls = 0, dev_calls = 0;
    double ms = 0.0;
    int maxn = 0;
    ~EigStats() {
        if (KT_DIAG)
            fprintf(stderr, "[kt eig] calls %lld (device %lld) max n %d total %.1f ms\n",
                    (long long)calls, (long long)dev_calls, maxn, ms);
    }
};
static EigStats g_eig;
static std::mutex g_eig_mu;  // the projection pairs are solved on two host threads

struct EigTimer {
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    ~EigTimer() {
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        std::lock_guard<std::mutex> lk(g_eig_mu);
        g_eig.ms += ms;
    }
};

// KT_DIAG builds: per-step wall-clock phases of fun_update / trace_fun_update
// on stderr (host clock; each phase ends at a stream sync of its own)
struct PhaseClock {
    bool on = false;
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    PhaseClock() { on = KT_DIAG != 0; }
    double lap() {  // ms since the previous lap
        const auto now = std::chrono::steady_clock::now();
        const double ms = std::chrono::duration<double, std::milli>(now - t).count();
        t = now;
        return ms;
    }
};

static void sym_eig_dispatch(kt_context_s* ctx, int n, const double* A, double* w, double* V);

static void sym_eig(kt_context_s* ctx, int n, const double* A, double* w, double* V) {
    constexpr bool log = KT_DIAG >= 2;
    const auto t0 = std::chrono::steady_clock::now();
    {
        EigTimer tm;
        {
            std::lock_guard<std::mutex> lk(g_eig_mu);
            g_eig.calls++;
            g_eig.maxn = std::max(g_eig.maxn, n);
            if (n > (V ? 160 : 320)) g_eig.dev_calls++;
        }
        sym_eig_dispatch(ctx, n, A, w, V);
    }
    if (log)
        fprintf(stderr, "[kt eig] n %d %s %.3f ms\n", n, V ? "vec" : "val",
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
}

static void sym_eig_dispatch(kt_context_s* ctx, int n, const double* A, double* w, double* V) {
    if (n <= 0) return;
    // host below the size where rocSOLVER dsyevd (~10 ms at n = 225, launch
    // bound) wins: eigenvalues-only host eig is 6 ms at n = 225, with
    // vectors 15 ms (tests/test_host_eig.py timings)
    if (n <= (V ? 160 : 320)) {
        sym_eig_host(n, A, w, V);
        return;
    }
    Workspace& ws = ctx->ws;
    ws.eigA.ensure(sizeof(double) * (size_t)n * n);
    ws.eigW.ensure(sizeof(double) * 2 * (size_t)n);
    ws.eigInfo.ensure(sizeof(rocblas_int));
    double* dA = ws.eigA.as<double>();
    KT_HIP(hipMemcpyAsync(dA, A, sizeof(double) * (size_t)n * n, hipMemcpyHostToDevice, ctx->stream));
    rocblas_status s = rocsolver_dsyevd(blas(ctx), V ? rocblas_evect_original : rocblas_evect_none,
                                        rocblas_fill_upper, n, dA, n, ws.eigW.as<double>(),
                                        ws.eigW.as<double>() + n, ws.eigInfo.as<rocblas_int>());
    if (s != rocblas_status_success) fail(KT_ERR_HIP, "rocsolver_dsyevd failed");
    rocblas_int info = 0;
    KT_HIP(hipMemcpyAsync(w, ws.eigW.ptr, sizeof(double) * n, hipMemcpyDeviceToHost, ctx->stream));
    if (V) KT_HIP(hipMemcpyAsync(V, dA, sizeof(double) * (size_t)n * n, hipMemcpyDeviceToHost, ctx->stream));
    KT_HIP(hipMemcpyAsync(&info, ws.eigInfo.ptr, sizeof(info), hipMemcpyDeviceToHost, ctx->stream));
    KT_HIP(hipStreamSynchronize(ctx->stream));
    if (info != 0) fail(KT_ERR_HIP, "rocsolver_dsyevd did not converge");
}

static std::vector<double> sym_eigvals(kt_context_s* ctx, int n, const std::vector<double>& A) {
    std::vector<double> w(n);
    sym_eig(ctx, n, A.data(), w.data(), nullptr);
    std::sort(w.begin(), w.end());
    return w;
}

// exp(sgn_b * M_b) for a batch of n x n matrices (host, column-major) on the
// device: truncated Taylor of degree 18 evaluated by Paterson-Stockmeyer
// (powers X^2, X^3, X^4 and four Horner steps in X^4) on X = sgn M / 2^s,
// then s squarings; s = max(0, ceil(log2(||M||_1 / theta_18))) per matrix
// with theta_18 the double-precision Taylor bound of Al-Mohy & Higham
// (expm(M) of fun_update.m:43-59 is a scaling-and-squaring method too).  The
// batch shares every launch (strided-batched dgemm, batched k_poly4); the
// squarings run on the prefix of matrices (sorted by s) that still need one.
static std::vector<std::vector<double>> expm_device_batch(kt_context_s* ctx, int n,
                                                          const std::vector<const double*>& Ms,
                                                          const std::vector<double>& sgns) {
    const double theta18 = 1.0908637192900361;
    const int nb = (int)Ms.size();
    std::vector<int> sv(nb, 0);
    for (int b = 0; b < nb; ++b) {
        double nrm1 = 0.0;
        for (int j = 0; j < n; ++j) {
            double c = 0.0;
            for (int i = 0; i < n; ++i) c += std::fabs(Ms[b][i + (size_t)j * n]);
            nrm1 = std::max(nrm1, c);
        }
        if (nrm1 > theta18) sv[b] = (int)std::ceil(std::log2(nrm1 / theta18));
    }
    std::vector<int> ord(nb);
    for (int b = 0; b < nb; ++b) ord[b] = b;
    std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) { return sv[a] > sv[b]; });
    const size_t nn = (size_t)n * n, bn = nn * nb;
    std::vector<double> Xh(bn);
    for (int k = 0; k < nb; ++k) {
        const int b = ord[k];
        const double scale = sgns[b] * std::ldexp(1.0, -sv[b]);
        for (size_t t = 0; t < nn; ++t) Xh[k * nn + t] = scale * Ms[b][t];
    }
    DevBuf& buf = ctx->ws.expm;
    buf.ensure(sizeof(double) * bn * 6);
    double* X1 = buf.as<double>();
    double* X2 = X1 + bn;
    double* X3 = X2 + bn;
    double* X4 = X3 + bn;
    double* T = X4 + bn;
    double* U = T + bn;
    hipStream_t st = ctx->stream;
    KT_HIP(hipMemcpyAsync(X1, Xh.data(), sizeof(double) * bn, hipMemcpyHostToDevice, st));
    const double one = 1.0, zero = 0.0;
    auto mm = [&](const double* A, const double* B, double* C, int cnt) {
        if (rocblas_dgemm_strided_batched(blas(ctx), rocblas_operation_none, rocblas_operation_none, n, n, n,
                                          &one, A, n, (rocblas_stride)nn, B, n, (rocblas_stride)nn, &zero, C,
                                          n, (rocblas_stride)nn, cnt) != rocblas_status_success)
            fail(KT_ERR_HIP, "rocblas_dgemm_strided_batched(expm) failed");
    };
    mm(X1, X1, X2, nb);
    mm(X2, X1, X3, nb);
    mm(X2, X2, X4, nb);
    double c[19];
    c[0] = 1.0;
    for (int k = 1; k <= 18; ++k) c[k] = c[k - 1] / k;
    // T = B_4 = c16 I + c17 X + c18 X^2;  T = T X^4 + B_k, k = 3..0
    KT_HIP(launch_poly4(n, 0.0, nullptr, c[16], c[17], X1, c[18], X2, 0.0, nullptr, T, st, nb));
    for (int k = 3; k >= 0; --k) {
        mm(T, X4, U, nb);
        KT_HIP(launch_poly4(n, 1.0, U, c[4 * k], c[4 * k + 1], X1, c[4 * k + 2], X2, c[4 * k + 3], X3, T, st,
                            nb));
    }
    // squarings of the matrices with s > q (a prefix), ping-ponging between T
    // and U: matrix k's result ends in T for even s_k, in U for odd
    double* buf2[2] = {T, U};
    for (int q = 0;; ++q) {
        int cnt = 0;
        while (cnt < nb && sv[ord[cnt]] > q) ++cnt;
        if (cnt == 0) break;
        mm(buf2[q & 1], buf2[q & 1], buf2[(q + 1) & 1], cnt);
    }
    std::vector<double> Fh(bn);
    for (int k = 0; k < nb;) {  // one read-back per run of equal parity
        const int par = sv[ord[k]] & 1;
        int e = k + 1;
        while (e < nb && (sv[ord[e]] & 1) == par) ++e;
        KT_HIP(hipMemcpyAsync(Fh.data() + k * nn, buf2[par] + k * nn, sizeof(double) * nn * (e - k),
                              hipMemcpyDeviceToHost, st));
        k = e;
    }
    KT_HIP(hipStreamSynchronize(st));
    std::vector<std::vector<double>> out(nb);
    for (int k = 0; k < nb; ++k) out[ord[k]].assign(Fh.begin() + k * nn, Fh.begin() + (k + 1) * nn);
    return out;
}

static std::vector<double> expm_device(kt_context_s* ctx, int n, const std::vector<double>& M,
                                       double sgn) {
    return std::move(expm_device_batch(ctx, n, {M.data()}, {sgn})[0]);
}

// f(M) for symmetric M (fun_update.m:43-59 maps exp/sinh/cosh/sin/cos/log/sqrt
// to expm/funm/logm/sqrtm; on a symmetric matrix all equal V f(L) V').  Above
// the host-eig size, exp/sinh/cosh take the reference's own route, expm
// (scaling and squaring on the device): (expm(M) -+ expm(-M)) / 2.
static std::vector<double> sym_matfun(kt_context_s* ctx, int n, const std::vector<double>& M,
                                      int fun) {
    if (n > 160 && (fun == KT_FUN_EXP || fun == KT_FUN_SINH || fun == KT_FUN_COSH)) {
        std::vector<double> E = expm_device(ctx, n, M, 1.0);
        if (fun == KT_FUN_EXP) return E;
        const std::vector<double> Em = expm_device(ctx, n, M, -1.0);
        const double sg = fun == KT_FUN_SINH ? -1.0 : 1.0;
        for (size_t t = 0; t < E.size(); ++t) E[t] = 0.5 * (E[t] + sg * Em[t]);
        return E;
    }
    std::vector<double> w(n), V((size_t)n * n), F((size_t)n * n);
    sym_eig(ctx, n, M.data(), w.data(), V.data());
    if (n <= 160) {
        sym_fun_from_eig(n, w.data(), V.data(), fun, F.data());
        return F;
    }
    // F = (V diag f(w)) V' as one device dgemm
    std::vector<double> VF(V);
    for (int k = 0; k < n; ++k) {
        const double fk = fscalar(fun, w[k]);
        for (int i = 0; i < n; ++i) VF[i + (size_t)k * n] *= fk;
    }
    DevBuf dV, dVF, dF;
    dV.ensure(sizeof(double) * V.size());
    dVF.ensure(sizeof(double) * V.size());
    dF.ensure(sizeof(double) * V.size());
    KT_HIP(hipMemcpyAsync(dV.ptr, V.data(), sizeof(double) * V.size(), hipMemcpyHostToDevice, ctx->stream));
    KT_HIP(hipMemcpyAsync(dVF.ptr, VF.data(), sizeof(double) * V.size(), hipMemcpyHostToDevice, ctx->stream));
    const double one = 1.0, zero = 0.0;
    if (rocblas_dgemm(blas(ctx), rocblas_operation_none, rocblas_operation_transpose, n, n, n, &one,
                      dVF.as<double>(), n, dV.as<double>(), n, &zero, dF.as<double>(), n) !=
        rocblas_status_success)
        fail(KT_ERR_HIP, "rocblas_dgemm(matfun) failed");
    KT_HIP(hipMemcpyAsync(F.data(), dF.ptr, sizeof(double) * F.size(), hipMemcpyDeviceToHost, ctx->stream));
    KT_HIP(hipStreamSynchronize(ctx->stream));
    dV.release();
    dVF.release();
    dF.release();
    return F;
}

// The elementwise handle of kt_trace_fun_update_fn, for the duration of the call.
struct ScalarFn {
    kt_scalar_fn f = nullptr;
    void* user = nullptr;
};
static thread_local ScalarFn tl_scalar_fn;

// trace_fun_update.m:43-47 / :85-89 with d1, d2 ascending
double trace_diff(const std::vector<double>& d1, const std::vector<double>& d2, int fun) {
    double x = 0.0;
    if (fun == kFunCallback) {  // sum(fun(d1) - fun(d2))
        if (!tl_scalar_fn.f) fail(KT_ERR_ARG, "no scalar function set");
        std::vector<double> f1(d1.size()), f2(d2.size());
        // a failed handle aborts the call: its zero-filled or partial output
        // must never reach the sum or the stop test
        if (tl_scalar_fn.f(d1.data(), f1.data(), (int64_t)d1.size(), tl_scalar_fn.user) != 0 ||
            tl_scalar_fn.f(d2.data(), f2.data(), (int64_t)d2.size(), tl_scalar_fn.user) != 0)
            fail(KT_ERR_CALLBACK, "trace_fun_update: fun callback failed");
        for (size_t i = 0; i < d1.size(); ++i) x += f1[i] - f2[i];
        return x;
    }
    if (fun == KT_FUN_EXP) {
        for (size_t i = 0; i < d1.size(); ++i) x += std::exp(d1[i]) * (1.0 - std::exp(d2[i] - d1[i]));
    } else {
        for (size_t i = 0; i < d1.size(); ++i) x += fscalar(fun, d1[i]) - fscalar(fun, d2[i]);
    }
    return x;
}

static bool is_symmetric_host(const kt_matrix_s* A) {
    const int64_t n = A->n;
    for (int64_t i = 0; i < n; ++i)
        for (int64_t k = A->h_rowptr[i]; k < A->h_rowptr[i + 1]; ++k) {
            const int64_t j = A->h_col[k];
            // find (j, i)
            const int32_t* b = A->h_col.data() + A->h_rowptr[j];
            const int32_t* e = A->h_col.data() + A->h_rowptr[j + 1];
            const int32_t* f = std::lower_bound(b, e, (int32_t)i);
            if (f == e || *f != (int32_t)i) return false;
            if (A->h_val[f - A->h_col.data()] != A->h_val[k]) return false;
        }
    return true;
}

void require_symmetric(kt_matrix_s* A, const char* msg) {
    if (A->symmetric < 0) A->symmetric = is_symmetric_host(A) ? 1 : 0;
    if (!A->symmetric) fail(KT_ERR_NOT_HERMITIAN, msg);
}

// dense host copy of A (original numbering), column-major
// The two projections of a Krylov step (tGm with the low-rank update, Gm
// without, trace_fun_update.m:83-84 / fun_update.m:106) are independent:
// host-size problems are solved on two host threads; exp/sinh/cosh above
// kDevExpm go through ONE batched device expm (2 matrices for exp, 4 for
// sinh/cosh = (expm(M) -+ expm(-M)) / 2).
constexpr int kDevExpm = 64;
constexpr int kPairThreads = 48;  // below this a second thread costs more than it saves

template <class F1, class F2>
static void run_pair(bool parallel, F1&& f1, F2&& f2) {
    if (!parallel) {
        f1();
        f2();
        return;
    }
    std::exception_ptr err;
    std::thread th([&] {
        try {
            f2();
        } catch (...) {
            err = std::current_exception();
        }
    });
    try {
        f1();
    } catch (...) {
        th.join();
        throw;
    }
    th.join();
    if (err) std::rethrow_exception(err);
}

// f(M1) - f(M2) for symmetric n x n M1, M2
static std::vector<double> sym_matfun_diff(kt_context_s* ctx, int n, const std::vector<double>& M1,
                                           const std::vector<double>& M2, int fun) {
    const bool expfam = fun == KT_FUN_EXP || fun == KT_FUN_SINH || fun == KT_FUN_COSH;
    if (expfam && n > kDevExpm) {
        std::vector<std::vector<double>> E;
        if (fun == KT_FUN_EXP) {
            E = expm_device_batch(ctx, n, {M1.data(), M2.data()}, {1.0, 1.0});
            for (size_t t = 0; t < E[0].size(); ++t) E[0][t] -= E[1][t];
            return std::move(E[0]);
        }
        E = expm_device_batch(ctx, n, {M1.data(), M1.data(), M2.data(), M2.data()}, {1.0, -1.0, 1.0, -1.0});
        const double sg = fun == KT_FUN_SINH ? -1.0 : 1.0;
        std::vector<double> D(E[0].size());
        for (size_t t = 0; t < D.size(); ++t)
            D[t] = 0.5 * (E[0][t] + sg * E[1][t]) - 0.5 * (E[2][t] + sg * E[3][t]);
        return D;
    }
    std::vector<double> F1, F2;
    const bool host = n <= 160;  // sym_matfun's host-eig range (no device work)
    run_pair(host && n >= kPairThreads, [&] { F1 = sym_matfun(ctx, n, M1, fun); },
             [&] { F2 = sym_matfun(ctx, n, M2, fun); });
    for (size_t t = 0; t < F1.size(); ++t) F1[t] -= F2[t];
    return F1;
}

// sorted eigenvalues of both projections
static void sym_eigvals_pair(kt_context_s* ctx, int n, const std::vector<double>& M1,
                             const std::vector<double>& M2, std::vector<double>& w1,
                             std::vector<double>& w2) {
    const bool host = n <= 320;  // sym_eig_dispatch's values-only host range
    run_pair(host && n >= kPairThreads, [&] { w1 = sym_eigvals(ctx, n, M1); },
             [&] { w2 = sym_eigvals(ctx, n, M2); });
}

// Bounds lo <= ||D||_2 <= hi for symmetric n x n D (fro2 = ||D||_F^2, c2 = the
// largest squared column norm) from k normalised squarings on the device:
// N_0 = D / ||D||_F, N_i = N_{i-1}^2 / ||N_{i-1}^2||_F, D^(2^i) = s_i N_i with
// log s_i = 2 log s_{i-1} + log ||N_{i-1}^2||_F.  false: no bounds (KT_NORM_POW=0).
constexpr int kNormPowMin = 96;
static bool sym_norm2_power_bounds(kt_context_s* ctx, int n, const std::vector<double>& D, double fro2,
                                   double c2, double& lo, double& hi) {
    const char* e = getenv("KT_NORM_POW");
    if (e && e[0] == '0') return false;
    constexpr int K = 6;
    const size_t nn = (size_t)n * n;
    DevBuf& b = ctx->ws.expm;
    b.ensure(sizeof(double) * (2 * nn + 2 * K + 2 + (size_t)n));
    double* M0 = b.as<double>();
    double* M1 = M0 + nn;
    double* out = M1 + nn;
    double* colsq = out + 2 * K + 2;
    const double s0 = std::sqrt(fro2);
    std::vector<double> N0(nn);
    for (size_t t = 0; t < nn; ++t) N0[t] = D[t] / s0;
    hipStream_t st = ctx->stream;
    KT_HIP(hipMemcpyAsync(M0, N0.data(), sizeof(double) * nn, hipMemcpyHostToDevice, st));
    const double one = 1.0, zero = 0.0;
    double* cur = M0;
    double* nxt = M1;
    for (int i = 0; i < K; ++i) {
        if (rocblas_dgemm(blas(ctx), rocblas_operation_none, rocblas_operation_none, n, n, n, &one, cur, n, cur, n,
                          &zero, nxt, n) != rocblas_status_success)
            fail(KT_ERR_HIP, "rocblas_dgemm(norm powers) failed");
        KT_HIP(launch_fro_colmax_scale(n, nxt, out + 2 * i, colsq, st));
        std::swap(cur, nxt);
    }
    double h[2 * K];
    KT_HIP(hipMemcpyAsync(h, out, sizeof(h), hipMemcpyDeviceToHost, st));
    KT_HIP(hipStreamSynchronize(st));
    lo = std::sqrt(c2);
    hi = s0;
    double logs = std::log(s0);
    double m = 1.0;
    for (int i = 0; i < K; ++i) {
        const double f2 = h[2 * i], cm2 = h[2 * i + 1];
        if (!(f2 > 0.0) || !std::isfinite(f2)) break;  // D^(2^i) vanished (nilpotent to rounding)
        logs = 2.0 * logs + 0.5 * std::log(f2);
        m *= 2.0;
        // ||N_i||_F = 1 after the scaling; its largest column norm is sqrt(cm2 / f2)
        hi = std::min(hi, std::exp(logs / m));
        lo = std::max(lo, std::exp((logs + 0.5 * std::log(cm2 / f2)) / m));
    }
    return true;
}

// ||D||_2 < tol for symmetric n x n D, decided from bounds when they settle
// it (max column 2-norm <= ||D||_2 <= ||D||_F, then the power bounds above),
// else from the spectrum
static bool sym_norm2_below(kt_context_s* ctx, int n, const std::vector<double>& D, double tol) {
    double fro2 = 0.0, col2max = 0.0;
    for (int j = 0; j < n; ++j) {
        double c2 = 0.0;
        for (int i = 0; i < n; ++i) c2 += D[i + (size_t)j * n] * D[i + (size_t)j * n];
        fro2 += c2;
        col2max = std::max(col2max, c2);
    }
    if (std::sqrt(fro2) < tol) return true;
    if (std::sqrt(col2max) >= tol) return false;
    // Tighter bounds from powers: for symmetric D and m = 2^k,
    //   maxcol(D^m)^(1/m) <= ||D||_2 <= ||D^m||_F^(1/m) <= n^(1/(2m)) ||D||_2,
    // so k normalised squarings on the device (one n^3 GEMM each, tens of us)
    // close the gap to a factor n^(1/2^(k+1)) (1.04 at n = 225, k = 6) instead
    // of a host eigensolve (1.3-1.6 ms at n = 225).  Only a bracket that
    // still straddles tol goes on to the spectrum.
    if (n >= kNormPowMin) {
        double lo = 0.0, hi = HUGE_VAL;
        if (sym_norm2_power_bounds(ctx, n, D, fro2, col2max, lo, hi)) {
            if (hi * (1.0 + 1e-10) < tol) return true;
            if (lo * (1.0 - 1e-10) >= tol) return false;
        }
    }
    const std::vector<double> ev = sym_eigvals(ctx, n, D);
    return std::max(std::fabs(ev.front()), std::fabs(ev.back())) < tol;
}

static std::vector<double> dense_A(const kt_matrix_s* A) {
    const int64_t n = A->n;
    std::vector<double> D((size_t)n * n, 0.0);
    for (int64_t i = 0; i < n; ++i)
        for (int64_t k = A->h_rowptr[i]; k < A->h_rowptr[i + 1]; ++k)
            D[(size_t)A->h_col[k] * n + i] += A->h_val[k];  // CSC==CSR for symmetric
    return D;
}

// M + U B U' (host, column-major), U n x r, B r x r
static void add_UBUt(std::vector<double>& M, int64_t n, int r, const double* U, const double* B) {
    std::vector<double> UB((size_t)n * r, 0.0);
    for (int j = 0; j < r; ++j)
        for (int l = 0; l < r; ++l) {
            const double b = B[l + (size_t)j * r];
            if (b == 0.0) continue;
            for (int64_t i = 0; i < n; ++i) UB[i + (size_t)j * n] += U[i + (size_t)l * n] * b;
        }
    for (int j = 0; j < r; ++j)
        for (int64_t c = 0; c < n; ++c) {
            const double u = U[c + (size_t)j * n];
            if (u == 0.0) continue;
            for (int64_t i = 0; i < n; ++i) M[i + (size_t)c * n] += UB[i + (size_t)j * n] * u;
        }
}

// ---------------------------------------------------------------------------
// BlockLanczos: lanczos_krylov.m (start :30-58, extend :60-67,
// add_inf_pole :73-101, CGS2 :109-115).  Window slots 0/1 of `win`.
// ---------------------------------------------------------------------------

struct BlockLanczos {
    kt_matrix_s* A;
    kt_context_s* ctx;
    int64_t n;
    int bs, PB;
    DevMat win, W;
    int cur = 0, prev = -1;
    int Hr = 0, Hc = 0;
    std::vector<double> H;  // column-major Hr x Hc
    bool lucky = false;

    BlockLanczos(kt_matrix_s* A_, int bs_) : A(A_), ctx(A_->ctx), n(A_->n), bs(bs_) {
        PB = pow2_at_least(bs);
        if (PB > 128) fail(KT_ERR_UNSUPPORTED, "block size > 128");
        win.alloc(ctx, n, 2 * PB);
        W.alloc(ctx, n, PB);
    }
    double* slot(int s) { return win.col(s * PB); }

    void grow(int add) {
        std::vector<double> Hn((size_t)(Hr + add) * (Hc + add), 0.0);
        for (int j = 0; j < Hc; ++j)
            for (int i = 0; i < Hr; ++i) Hn[i + (size_t)j * (Hr + add)] = H[i + (size_t)j * Hr];
        H.swap(Hn);
        Hr += add;
        Hc += add;
    }

    void start(const double* U) {  // U: host n x bs column-major (original numbering)
        upload_rows(A, U, bs, slot(0), 2 * PB);
        std::vector<double> R;
        block_qr(ctx, n, slot(0), 2 * PB, bs, R);  // [V, ~] = qr(b, 0)    :48
        cur = 0;
        prev = -1;
        Hr = bs;
        Hc = 0;
        H.clear();
        add_inf_pole();
    }
    void extend() { add_inf_pole(); }

    void add_inf_pole() {
        const int ld = 2 * PB;
        spmm(A, slot(cur), ld, W.col(0), PB, bs);  // w = A * w   :81
        grow(bs);                                  // :85
        // CGS2 against the window (both slots in one Gram; absent slot -> 0)
        std::vector<double> h((size_t)2 * PB * bs, 0.0);
        const size_t cnt = (size_t)2 * PB * bs;
        double* hg = nullptr;
        if (prev >= 0) {  // both slots live: Gram blocks stay on the device
            PinnedBuf& hp = ctx->ws.pin_small;
            hp.ensure(sizeof(double) * 2 * cnt);
            hg = hp.as<double>();
            for (int pass = 0; pass < 2; ++pass) {
                const double* dG = gram_device(ctx, n, win.col(0), ld, 2 * PB, W.col(0), PB, bs);
                KT_HIP(hipMemcpyAsync(hg + pass * cnt, dG, sizeof(double) * cnt, hipMemcpyDeviceToHost,
                                      ctx->stream));
                combine_device(ctx, n, win.col(0), ld, 2 * PB, dG, bs, -1.0, 1.0, W.col(0), PB);
            }
        }
        for (int pass = 0; !hg && pass < 2; ++pass) {  // :109-115
            std::vector<double> g;
            gram(ctx, n, win.col(0), ld, 2 * PB, W.col(0), PB, bs, g);
            if (prev < 0)
                for (int j = 0; j < bs; ++j)
                    for (int i = 0; i < 2 * PB; ++i)
                        if (i / PB != cur) g[i + (size_t)j * 2 * PB] = 0.0;
            std::vector<double> C(g.size());
            for (size_t t = 0; t < g.size(); ++t) {
                C[t] = -g[t];
                h[t] += g[t];
            }
            combine(ctx, n, win.col(0), ld, 2 * PB, C, bs, 1.0, W.col(0), PB);
        }
        std::vector<double> R;
        block_qr(ctx, n, W.col(0), PB, bs, R);  // [w, R] = qr(w, 0)   :90
        if (hg)  // (block_qr synchronised the stream after the read-backs were queued)
            for (size_t t = 0; t < cnt; ++t) h[t] = (0.0 + hg[t]) + hg[cnt + t];  // h += g, twice
        // H(max(1,end-3bs+1):end-bs, end-bs+1:end) = h      :88
        const int c0 = Hc - bs;
        auto put = [&](int s, int row0) {
            for (int j = 0; j < bs; ++j)
                for (int i = 0; i < bs; ++i)
                    H[(row0 + i) + (size_t)(c0 + j) * Hr] = h[(s * PB + i) + (size_t)j * 2 * PB];
        };
        if (prev >= 0) {
            put(prev, Hr - 3 * bs);
            put(cur, Hr - 2 * bs);
        } else {
            put(cur, Hr - 2 * bs);
        }
        for (int j = 0; j < bs; ++j)
            for (int i = 0; i < bs; ++i) H[(Hr - bs + i) + (size_t)(c0 + j) * Hr] = R[i + (size_t)j * bs];
        lucky = norm_fro(R) < 1e-8;  // :91-93
        // window rotation :94-99
        const int dst = (prev < 0) ? 1 - cur : prev;
        copy_cols(ctx, n, W.col(0), PB, slot(dst), ld, PB);
        prev = cur;
        cur = dst;
    }
};

// ---------------------------------------------------------------------------
// BlockArnoldi: arnoldi_krylov.m (start :32-62, extend :64-72,
// add_inf_pole :78-111).  Full basis in `V` (block b at columns b*PB).
// ---------------------------------------------------------------------------
struct BlockArnoldi {
    kt_matrix_s* A;
    kt_context_s* ctx;
    int64_t n;
    int bs, PB, maxblk;
    int nblk = 0;  // blocks in V
    DevMat V, W;
    int Hr = 0, Hc = 0;
    std::vector<double> H;
    bool lucky = false;

    BlockArnoldi(kt_matrix_s* A_, int bs_, int maxblk_) : A(A_), ctx(A_->ctx), n(A_->n), bs(bs_),
                                                           maxblk(maxblk_) {
        PB = pow2_at_least(bs);
        if (PB > 128) fail(KT_ERR_UNSUPPORTED, "block size > 128");
        // V is written block by block (start: block 0 zeroed + the selector;
        // extend: W's PB columns, zero padding included), so only what a step
        // reads is ever initialised -- no memset of all maxblk blocks
        V.alloc(ctx, n, maxblk * PB, false);
        W.alloc(ctx, n, PB);
    }
    int ld() const { return maxblk * PB; }
    double* blk(int b) { return V.col(b * PB); }

    void grow(int add) {
        std::vector<double> Hn((size_t)(Hr + add) * (Hc + add), 0.0);
        for (int j = 0; j < Hc; ++j)
            for (int i = 0; i < Hr; ++i) Hn[i + (size_t)j * (Hr + add)] = H[i + (size_t)j * Hr];
        H.swap(Hn);
        Hr += add;
        Hc += add;
    }

    void start(const double* U) {
        PhaseClock pc;
        pre_ = false;
        hpar_ = 0;
        // the Gram read-backs of two consecutive steps (the next step's first
        // passes are queued before this step's last read-back is consumed):
        // sized once for the whole run, so no reallocation under a copy
        slot_ = (size_t)3 * (size_t)maxblk * PB * bs;
        ctx->ws.pin_arn.ensure(sizeof(double) * 2 * slot_);
        KT_HIP(hipMemset2DAsync(blk(0), sizeof(double) * ld(), 0, sizeof(double) * PB, (size_t)n, ctx->stream));
        upload_rows(A, U, bs, blk(0), ld());
        const double t_up = pc.on ? pc.lap() : 0.0;
        std::vector<double> R;
        block_qr(ctx, n, blk(0), ld(), bs, R);  // [V, ~] = qr(b, 0)   :50
        if (pc.on) KT_HIP(hipStreamSynchronize(ctx->stream));
        const double t_qr = pc.on ? pc.lap() : 0.0;
        nblk = 1;
        Hr = bs;
        Hc = 0;
        H.clear();
        add_inf_pole(0);
        if (pc.on)
            fprintf(stderr, "[kt arnoldi start] n %lld bs %d ld %d: upload %.3f qr %.3f first pole %.3f ms\n",
                    (long long)n, bs, ld(), t_up, t_qr, pc.lap());
    }
    void extend() { add_inf_pole(nblk - 1); }

    // w = A * V(:, last block), then the two CGS passes against the nb blocks
    // V(:, 0:nb) (:86, :119-125) with the Gram blocks kept on the device and
    // read back (pinned, asynchronously) into step slot `par`
    void head(int last, int nb, int par) {
        const int L = ld();
        const int pv = nb * PB;
        spmm(A, blk(last), L, W.col(0), PB, bs);  // w = A * w   :86
        const size_t cnt = (size_t)pv * bs;
        double* hg = ctx->ws.pin_arn.as<double>() + (size_t)par * slot_;
        for (int pass = 0; pass < 2; ++pass) {
            const double* dG = gram_device(ctx, n, V.col(0), L, pv, W.col(0), PB, bs);
            KT_HIP(hipMemcpyAsync(hg + pass * cnt, dG, sizeof(double) * cnt, hipMemcpyDeviceToHost, ctx->stream));
            combine_device(ctx, n, V.col(0), L, pv, dG, bs, -1.0, 1.0, W.col(0), PB);
        }
    }

    void add_inf_pole(int last) {
        if (nblk >= maxblk) fail(KT_ERR_UNSUPPORTED, "Arnoldi basis capacity exceeded");
        const int L = ld();
        const int pv = nblk * PB;
        const size_t cnt = (size_t)pv * bs;
        // the spmm and the first two CGS2 passes of this step were queued at
        // the end of the previous one (pre_), while its last read-back drained
        if (!pre_) head(last, nblk, hpar_);
        pre_ = false;
        double* hg = ctx->ws.pin_arn.as<double>() + (size_t)hpar_ * slot_;
        // w = w - V (V'w), the Gram block read back into hg + off
        auto project = [&](size_t off) {
            const double* dG = gram_device(ctx, n, V.col(0), L, pv, W.col(0), PB, bs);
            KT_HIP(hipMemcpyAsync(hg + off, dG, sizeof(double) * cnt, hipMemcpyDeviceToHost, ctx->stream));
            combine_device(ctx, n, V.col(0), L, pv, dG, bs, -1.0, 1.0, W.col(0), PB);
        };
        std::vector<double> r;
        block_qr(ctx, n, W.col(0), PB, bs, r, true);  // [w, r] = qr(w, 0)   :99
        lucky = norm2_small(bs, bs, r.data()) < 1e-12;  // :100-102
        // (no sync here: every block_qr path waits for the stream up to a point
        // queued after the two Gram read-backs -- its own Gram or factor
        // read-back -- so hg is complete; the QR's trailing W R^-1 may still run)
        std::vector<double> h(cnt);
        for (size_t t = 0; t < cnt; ++t) h[t] = (0.0 + hg[t]) + hg[cnt + t];  // h += g, twice
        grow(bs);  // :93-94
        const int c0 = Hc - bs;
        auto hrow = [&](int padded_row) { return (padded_row / PB) * bs + padded_row % PB; };
        for (int j = 0; j < bs; ++j)
            for (int i = 0; i < pv; ++i)
                if (i % PB < bs) H[hrow(i) + (size_t)(c0 + j) * Hr] = h[i + (size_t)j * pv];  // :96
        // reorthogonalise :104-106
        project(2 * cnt);
        // the read-back of hh is complete at this event
        if (!hh_ev_) KT_HIP(hipEventCreateWithFlags(&hh_ev_, hipEventDisableTiming));
        KT_HIP(hipEventRecord(hh_ev_, ctx->stream));
        copy_cols(ctx, n, W.col(0), PB, blk(nblk), L, PB);  // V = [V, w]   :110
        // queue the next step's spmm and first two passes (they read the block
        // just copied; stream order) before waiting for this read-back, so the
        // device keeps working through the host's turn-around.  When the run
        // stops here they are never used (W and the other slot only).
        if (nblk + 1 < maxblk && !lucky) {
            head(nblk, nblk + 1, hpar_ ^ 1);
            pre_ = true;
        }
        if (pre_) KT_HIP(hipEventSynchronize(hh_ev_));  // (not the queued head behind it)
        else KT_HIP(hipStreamSynchronize(ctx->stream));
        std::vector<double> hh(hg + 2 * cnt, hg + 3 * cnt);
        std::vector<double> hr((size_t)pv * bs);
        matmul(pv, bs, bs, hh.data(), r.data(), hr.data());
        for (int j = 0; j < bs; ++j)
            for (int i = 0; i < pv; ++i)
                if (i % PB < bs) H[hrow(i) + (size_t)(c0 + j) * Hr] += hr[i + (size_t)j * pv];
        for (int j = 0; j < bs; ++j)  // :108
            for (int i = 0; i < bs; ++i) H[(Hr - bs + i) + (size_t)(c0 + j) * Hr] = r[i + (size_t)j * bs];
        nblk += 1;
        if (pre_) hpar_ ^= 1;
    }

    ~BlockArnoldi() {
        if (hh_ev_) (void)hipEventDestroy(hh_ev_);
    }
    BlockArnoldi(const BlockArnoldi&) = delete;
    BlockArnoldi& operator=(const BlockArnoldi&) = delete;

   private:
    hipEvent_t hh_ev_ = nullptr;
    bool pre_ = false;  // the next step's head() is queued
    int hpar_ = 0;      // pinned read-back slot of the current step
    size_t slot_ = 0;   // doubles per slot
};

// Cm = (V1' U) B (V1' U)'   (trace_fun_update.m:65-66, fun_update.m:80-81)
static std::vector<double> make_Cm(kt_context_s* ctx, kt_matrix_s* A, const double* V1, int ldv,
                                   int bs, const double* U, int rk, const double* B) {
    DevMat Ud;
    const int PU = pow2_at_least(rk);
    Ud.alloc(ctx, A->n, PU);
    upload_rows(A, U, rk, Ud.col(0), PU);
    std::vector<double> G;  // bs x rk
    gram(ctx, A->n, V1, ldv, bs, Ud.col(0), PU, rk, G);
    std::vector<double> GB((size_t)bs * rk), Cm((size_t)bs * bs);
    matmul(bs, rk, rk, G.data(), B, GB.data());
    for (int j = 0; j < bs; ++j)
        for (int i = 0; i < bs; ++i) {
            double s = 0.0;
            for (int l = 0; l < rk; ++l) s += GB[i + (size_t)l * bs] * G[j + (size_t)l * bs];
            Cm[i + (size_t)j * bs] = s;
        }
    return Cm;
}

static bool b_hermitian(int rk, const double* B) {
    for (int j = 0; j < rk; ++j)
        for (int i = 0; i < rk; ++i)
            if (B[i + (size_t)j * rk] != B[j + (size_t)i * rk]) return false;
    return true;
}

// top-left nn x nn of column-major M (Mr rows)
static std::vector<double> top_left(const std::vector<double>& M, int Mr, int nn) {
    std::vector<double> T((size_t)nn * nn);
    for (int j = 0; j < nn; ++j)
        for (int i = 0; i < nn; ++i) T[i + (size_t)j * nn] = M[i + (size_t)j * Mr];
    return T;
}

// The context a pipelined block-Krylov run hands its projected work to
// (ctx->helper, created on first use), or nullptr for the serial loop:
// env_name set to "0", or the helper cannot be created.
static kt_context_s* pipeline_helper(kt_context_s* ctx, const char* env_name) {
    const char* e = getenv(env_name);  // read per call (A/B within one process)
    if (e && e[0] == '0') return nullptr;
    if (!ctx->helper) {
        kt_context_t h = nullptr;
        if (kt_context_create(ctx->device, &h) != KT_OK) {
            (void)hipGetLastError();
            KT_HIP(hipSetDevice(ctx->device));
            return nullptr;
        }
        ctx->helper = h;
        KT_HIP(hipSetDevice(ctx->device));
    }
    return ctx->helper;
}

// ---------------------------------------------------------------------------
// trace_fun_update.m
// ---------------------------------------------------------------------------
double trace_fun_update_impl(kt_matrix_s* A, int rk, const double* U, const double* B, double tol,
                             int it, int fun, int* iter_out, int* lucky_out) {
    kt_context_s* ctx = A->ctx;
    const int64_t n = A->n;
    if (it <= 0) it = (int)std::min<int64_t>(100, n);  // :25-27
    if (n <= 130) {                                    // :37-51 dense shortcut
        std::vector<double> fA = dense_A(A), fAt = fA;
        add_UBUt(fAt, n, rk, U, B);
        for (int64_t j = 0; j < n; ++j)
            for (int64_t i = 0; i < j; ++i) {
                const double s = 0.5 * (fAt[i + j * n] + fAt[j + i * n]);
                fAt[i + j * n] = fAt[j + i * n] = s;
            }
        std::vector<double> w1, w2;
        sym_eigvals_pair(ctx, (int)n, fAt, fA, w1, w2);
        const double x = trace_diff(w1, w2, fun);
        if (iter_out) *iter_out = 0;
        if (lucky_out) *lucky_out = 0;
        return x;
    }
    const bool herm = b_hermitian(rk, B);  // :55
    if (!herm) fail(KT_ERR_UNSUPPORTED, "trace_fun_update: non-Hermitian B (needs a general eig)");
    BlockLanczos L(A, rk);
    const int d = 2;  // :58
    // As in fun_update_impl: step j's eigenvalues and Xm (:83-89) only decide
    // whether to go on, so they run on a worker thread (helper context for
    // the projections too large for the host solver) while this thread runs
    // Lanczos step j + 1; the stop test (:104-118) is applied in step order
    // on the worker, and the loop ends at the first step that says stop.
    // Identical results to the serial loop (KT_TFU_PIPE=0).
    struct Step {
        double Xm = 0.0;
        bool stop = false, lucky = false;
    };
    std::vector<Step> steps((size_t)it + 2);
    double Xstop[2] = {0.0, 0.0};
    const ScalarFn sfn = tl_scalar_fn;  // the elementwise handle travels to the worker thread
    auto project = [&](kt_context_s* c, int jj, int nn, std::vector<double>& tGm, std::vector<double>& Gm) {
        tl_scalar_fn = sfn;
        std::vector<double> w1, w2;
        sym_eigvals_pair(c, nn, tGm, Gm, w1, w2);
        Step& S = steps[jj];
        S.Xm = trace_diff(w1, w2, fun);  // :83-89
        if (jj <= d) {                   // :104-118
            Xstop[jj - 1] = S.Xm;
        } else {
            S.stop = std::fabs(S.Xm - Xstop[0]) < tol;
            if (!S.stop) {
                Xstop[0] = Xstop[1];
                Xstop[1] = S.Xm;
            }
        }
    };
    kt_context_s* hctx = pipeline_helper(ctx, "KT_TFU_PIPE");
    RunWorker W;  // finished before steps / Xstop go out of scope
    if (hctx) W.reset(ctx_worker(ctx, kWorkerPipeline));
    std::vector<double> Cm;
    int jfin = 0;
    PhaseClock pc;
    for (int j = 1; j <= it; ++j) {
        if (j == 1) {
            L.start(U);                                                        // :64
            const double* V1 = L.win.col(L.prev * L.PB);                       // Um(:, 1:end-rk)
            Cm = make_Cm(ctx, A, V1, 2 * L.PB, rk, U, rk, B);                  // :65-66
        } else {
            L.extend();                                                        // :68
        }
        steps[j].lucky = L.lucky;
        const double t_ext = pc.on ? pc.lap() : 0.0;
        if (W && j >= 2) {
            W->wait(j - 2);
            if (pc.on)
                fprintf(stderr, "[kt tfu] step %d stop %d (waited %.3f ms after extend %d: %.3f ms)\n", j - 1,
                        (int)steps[j - 1].stop, pc.lap(), j, t_ext);
            if (steps[j - 1].stop) {
                jfin = j - 1;
                break;
            }
        }
        const int nn = L.Hr - rk;                                              // :72-73
        std::vector<double> Gm = top_left(L.H, L.Hr, nn), tGm = Gm;
        for (int jj = 0; jj < rk; ++jj)
            for (int ii = 0; ii < rk; ++ii) tGm[ii + (size_t)jj * nn] += Cm[ii + (size_t)jj * rk];  // :74-77
        for (int b = 0; b < nn; ++b)                                           // :78-81
            for (int a = 0; a < b; ++a) {
                double sv = 0.5 * (Gm[a + (size_t)b * nn] + Gm[b + (size_t)a * nn]);
                Gm[a + (size_t)b * nn] = Gm[b + (size_t)a * nn] = sv;
                sv = 0.5 * (tGm[a + (size_t)b * nn] + tGm[b + (size_t)a * nn]);
                tGm[a + (size_t)b * nn] = tGm[b + (size_t)a * nn] = sv;
            }
        const bool last = steps[j].lucky || j == it;                           // :119-124 / loop end
        if (W) {
            W->submit([&, j, nn, tGm = std::move(tGm), Gm = std::move(Gm)]() mutable {
                project(hctx, j, nn, tGm, Gm);
            });
            if (last) {
                W->wait(j - 1);
                jfin = j;
                break;
            }
        } else {
            project(ctx, j, nn, tGm, Gm);
            if (pc.on) fprintf(stderr, "[kt tfu] step %d nn %d extend %.3f eig %.3f ms\n", j, nn, t_ext, pc.lap());
            if (steps[j].stop || last) {
                jfin = j;
                break;
            }
        }
    }
    W.reset();
    if (iter_out) *iter_out = jfin;
    if (lucky_out) *lucky_out = steps[jfin].lucky ? 1 : 0;
    return steps[jfin].Xm;
}

// ---------------------------------------------------------------------------
// fun_update.m (Arnoldi branch).  Returns Xm (nx x nx) and either the device
// basis (dense == false) or the dense fallback marker (Um = eye(n)).
// ---------------------------------------------------------------------------
struct FunUpdateResult {
    std::vector<double> Xm;
    int nx = 0;
    int iter = 0;
    bool lucky = false;
    bool dense = false;
    std::unique_ptr<BlockArnoldi> basis;
};

FunUpdateResult fun_update_impl(kt_matrix_s* A, int rk, const double* U, const double* B, int fun,
                                double tol, int it) {
    kt_context_s* ctx = A->ctx;
    const int64_t n = A->n;
    if (it <= 0) it = (int)std::min<int64_t>(100, n);  // :24-26
    const bool herm = b_hermitian(rk, B);              // :41
    if (!herm) fail(KT_ERR_UNSUPPORTED, "fun_update: non-Hermitian B");
    FunUpdateResult res;
    // basis never needs more than ~n/2 columns before the dense fallback (:85)
    const int maxblk = (int)std::min<int64_t>(it + 1, n / (2 * (int64_t)rk) + 2);
    res.basis.reset(new BlockArnoldi(A, rk, std::max(maxblk, 2)));
    BlockArnoldi& Ar = *res.basis;
    const int d = 2;
    // Step j's projected work -- Xm = f(tGm) - f(Gm) (:93-106) and the stop
    // test (:108-126) -- decides only WHETHER to go on; the next Arnoldi step
    // does not read it.  So it runs on a worker thread with the helper
    // context (own stream and rocBLAS handle) while this thread extends the
    // basis to step j + 1 on the device; the loop then reads step j's
    // decision and stops there if it says so (the speculative block is
    // ignored: Xm, nx, iter, lucky are step j's, and Um is the basis'
    // first nx columns).  Same arithmetic, same order: results identical to
    // the serial loop (KT_FU_PIPE=0).
    struct Step {
        std::vector<double> F1;
        int nn = 0;
        bool stop = false, lucky = false;
    };
    std::vector<Step> steps((size_t)it + 2);
    std::vector<std::vector<double>> Xstop;
    auto project = [&](kt_context_s* c, int jj, std::vector<double>& tGm, std::vector<double>& Gm) {
        Step& S = steps[jj];
        S.F1 = sym_matfun_diff(c, S.nn, tGm, Gm, fun);                      // :106
        if (jj <= d) {                                                       // :109-126
            Xstop.push_back(S.F1);
            return;
        }
        const int nn = S.nn;
        const int n0 = (int)std::lround(std::sqrt((double)Xstop[0].size()));
        std::vector<double> D = S.F1;
        for (int b = 0; b < n0; ++b)
            for (int a = 0; a < n0; ++a) D[a + (size_t)b * nn] -= Xstop[0][a + (size_t)b * n0];
        // 2-norm of the symmetric difference (= max |eig|) below tol?
        S.stop = sym_norm2_below(c, nn, D, tol);
        if (!S.stop) {
            Xstop.erase(Xstop.begin());
            Xstop.push_back(S.F1);
        }
    };
    kt_context_s* hctx = pipeline_helper(ctx, "KT_FU_PIPE");
    RunWorker W;  // finished before steps / Xstop go out of scope
    if (hctx) W.reset(ctx_worker(ctx, kWorkerPipeline));
    std::vector<double> Cm;
    int jfin = 0;
    PhaseClock pc;
    for (int j = 1; j <= it; ++j) {
        if (j == 1) {
            Ar.start(U);                                                     // :79
            if (pc.on) fprintf(stderr, "[kt fu] Ar.start %.3f ms\n", pc.lap());
            Cm = make_Cm(ctx, A, Ar.blk(0), Ar.ld(), rk, U, rk, B);         // :80-81
        } else {
            Ar.extend();                                                     // :83
        }
        steps[j].lucky = Ar.lucky;
        const double t_ext = pc.on ? pc.lap() : 0.0;
        if (pc.on && j == 1) fprintf(stderr, "[kt fu] start %.3f ms\n", t_ext);
        // the previous step's decision (its work ran during this extension)
        if (W && j >= 2) {
            W->wait(j - 2);
            if (pc.on)
                fprintf(stderr, "[kt fu] step %d nn %d stop %d (waited %.3f ms after extend %d: %.3f ms)\n", j - 1,
                        steps[j - 1].nn, (int)steps[j - 1].stop, pc.lap(), j, t_ext);
            if (steps[j - 1].stop) {
                jfin = j - 1;
                break;
            }
        }
        if (2 * (int64_t)Ar.nblk * rk >= n) {  // size(Um,2) >= size(Um,1)/2   :85-90
            std::vector<double> fA = dense_A(A), fAt = fA;
            add_UBUt(fAt, n, rk, U, B);
            std::vector<double> F1 = sym_matfun_diff(ctx, (int)n, fAt, fA, fun);
            W.reset();
            res.Xm.swap(F1);
            res.nx = (int)n;
            res.iter = j;
            res.lucky = Ar.lucky;
            res.dense = true;
            ctx->fu_dense++;
            ctx->fu_last_cols = n;
            return res;
        }
        const int nn = Ar.Hr - rk;                                           // :93
        std::vector<double> Gm = top_left(Ar.H, Ar.Hr, nn);
        for (int b = 0; b < nn; ++b)                                         // :94
            for (int a = 0; a < b; ++a) {
                const double sv = 0.5 * (Gm[a + (size_t)b * nn] + Gm[b + (size_t)a * nn]);
                Gm[a + (size_t)b * nn] = Gm[b + (size_t)a * nn] = sv;
            }
        std::vector<double> tGm = Gm;
        for (int jj = 0; jj < rk; ++jj)                                      // :97-104
            for (int ii = 0; ii < rk; ++ii)
                tGm[ii + (size_t)jj * nn] += 0.5 * (Cm[ii + (size_t)jj * rk] + Cm[jj + (size_t)ii * rk]);
        steps[j].nn = nn;
        const bool last = steps[j].lucky || j == it;                         // :127-130 / loop end
        if (W) {
            W->submit([&, j, tGm = std::move(tGm), Gm = std::move(Gm)]() mutable { project(hctx, j, tGm, Gm); });
            if (last) {
                W->wait(j - 1);
                jfin = j;
                break;
            }
        } else {
            project(ctx, j, tGm, Gm);
            if (pc.on) fprintf(stderr, "[kt fu] step %d nn %d extend %.3f project %.3f ms\n", j, nn, t_ext, pc.lap());
            if (steps[j].stop || last) {
                jfin = j;
                break;
            }
        }
    }
    if (pc.on) pc.lap();
    W.reset();
    if (pc.on) fprintf(stderr, "[kt fu] join %.3f ms\n", pc.lap());
    Step& S = steps[jfin];
    res.Xm.swap(S.F1);
    res.nx = S.nn;
    res.iter = jfin;
    res.lucky = S.lucky;
    ctx->fu_last_cols = res.nx;
    return res;
}

// ---------------------------------------------------------------------------
// fun_update.m's Lanczos branch (nargout <= 3, :69-76): the same loop as the
// Arnoldi branch over lanczos_krylov's 2-block window (BlockLanczos, as
// trace_fun_update runs it) -- Cm from the first block (:72-73), Gm the
// projected block tridiagonal (:93-94), Xm = f(tGm) - f(Gm) (:106), the
// 2-norm lag-2 stop (:108-126) -- with no dense fallback (:85-90 belongs to
// the Arnoldi branch).  Serial.  The reference then indexes Um(:, 1:size(Xm,1))
// on the n x 2rk window (:137), which fails once the run took three or more
// steps; that error is the caller's to raise (the MEX shim does), the C ABI
// returns Xm.
// ---------------------------------------------------------------------------
static FunUpdateResult fun_update_lanczos_impl(kt_matrix_s* A, int rk, const double* U, const double* B,
                                               int fun, double tol, int it) {
    kt_context_s* ctx = A->ctx;
    const int64_t n = A->n;
    if (it <= 0) it = (int)std::min<int64_t>(100, n);  // :24-26
    if (!b_hermitian(rk, B)) fail(KT_ERR_UNSUPPORTED, "fun_update: non-Hermitian B");  // :41
    FunUpdateResult res;
    BlockLanczos L(A, rk);
    const int d = 2;  // :63
    std::vector<std::vector<double>> Xstop;
    std::vector<double> Cm, F1;
    int nn = 0, j = 1;
    for (j = 1; j <= it; ++j) {
        if (j == 1) {
            L.start(U);                                                            // :71
            Cm = make_Cm(ctx, A, L.win.col(L.prev * L.PB), 2 * L.PB, rk, U, rk, B);  // :72-73
        } else {
            L.extend();                                                            // :75
        }
        nn = L.Hr - rk;                                                            // :93
        std::vector<double> Gm = top_left(L.H, L.Hr, nn);
        for (int b = 0; b < nn; ++b)                                               // :94
            for (int a = 0; a < b; ++a) {
                const double sv = 0.5 * (Gm[a + (size_t)b * nn] + Gm[b + (size_t)a * nn]);
                Gm[a + (size_t)b * nn] = Gm[b + (size_t)a * nn] = sv;
            }
        std::vector<double> tGm = Gm;
        for (int jj = 0; jj < rk; ++jj)                                            // :97-104
            for (int ii = 0; ii < rk; ++ii)
                tGm[ii + (size_t)jj * nn] += 0.5 * (Cm[ii + (size_t)jj * rk] + Cm[jj + (size_t)ii * rk]);
        F1 = sym_matfun_diff(ctx, nn, tGm, Gm, fun);                               // :106
        bool stop = false;
        if (j <= d) {                                                              // :109-110
            Xstop.push_back(F1);
        } else {                                                                   // :111-126
            const int n0 = (int)std::lround(std::sqrt((double)Xstop[0].size()));
            std::vector<double> D = F1;
            for (int b = 0; b < n0; ++b)
                for (int a = 0; a < n0; ++a) D[a + (size_t)b * nn] -= Xstop[0][a + (size_t)b * n0];
            stop = sym_norm2_below(ctx, nn, D, tol);
            if (!stop) {
                Xstop.erase(Xstop.begin());
                Xstop.push_back(F1);
            }
        }
        if (stop || L.lucky) break;                                                // :122-130
    }
    res.Xm.swap(F1);
    res.nx = nn;
    res.iter = std::min(j, it);                                                    // :132
    res.lucky = L.lucky;
    ctx->fu_last_cols = nn;
    return res;
}

// MATLAB normest (2-norm power estimate) on the device: x = sum(abs(A))',
// repeat x = A'(A x)/||.|| until |e - e0| <= tol e.
static double normest_compute(kt_matrix_s* A, double tol);

// MATLAB normest is a deterministic function of (A, tol); the fmincon loops
// call fun_and_grad_* (fun_and_grad_krylov_exp.m:26, _fun.m:27) with the same
// A and tol every iteration, so the estimate is kept with the matrix (until an
// edit bumps its version): the same value without a dozen host round trips.
double normest_impl(kt_matrix_s* A, double tol) {
    if (A->normest_ok && A->normest_version == A->version && A->normest_tol == tol) return A->normest_val;
    const double e = normest_compute(A, tol);
    A->normest_ok = true;
    A->normest_version = A->version;
    A->normest_tol = tol;
    A->normest_val = e;
    return e;
}

static double normest_compute(kt_matrix_s* A, double tol) {
    kt_context_s* ctx = A->ctx;
    const int64_t n = A->n;
    if (n == 0) return 0.0;
    std::vector<double> x(n, 0.0);
    for (int64_t i = 0; i < n; ++i)
        for (int64_t k = A->h_rowptr[i]; k < A->h_rowptr[i + 1]; ++k) x[A->h_col[k]] += std::fabs(A->h_val[k]);
    DevMat X, Y;
    X.alloc(ctx, n, 1);
    Y.alloc(ctx, n, 1);
    upload_rows(A, x.data(), 1, X.col(0), 1);
    std::vector<double> g;
    gram(ctx, n, X.col(0), 1, 1, X.col(0), 1, 1, g);
    double e = std::sqrt(g[0]);
    if (e == 0.0) return 0.0;
    combine(ctx, n, X.col(0), 1, 1, std::vector<double>{1.0 / e}, 1, 0.0, Y.col(0), 1);
    copy_cols(ctx, n, Y.col(0), 1, X.col(0), 1, 1);
    double e0 = 0.0;
    for (int cnt = 0; std::fabs(e - e0) > tol * e && cnt < 100; ++cnt) {
        e0 = e;
        spmm(A, X.col(0), 1, Y.col(0), 1, 1);  // Ax
        gram(ctx, n, Y.col(0), 1, 1, Y.col(0), 1, 1, g);
        const double nAx = std::sqrt(g[0]);
        spmm(A, Y.col(0), 1, X.col(0), 1, 1);  // A'Ax (A symmetric)
        gram(ctx, n, X.col(0), 1, 1, X.col(0), 1, 1, g);
        const double nx = std::sqrt(g[0]);
        if (nAx == 0.0 || nx == 0.0) return 0.0;
        e = nx / nAx;
        combine(ctx, n, X.col(0), 1, 1, std::vector<double>{1.0 / nx}, 1, 0.0, Y.col(0), 1);
        copy_cols(ctx, n, Y.col(0), 1, X.col(0), 1, 1);
    }
    return e;
}

// Low-rank factor from edge weights (fun_and_grad_krylov_exp.m:56-73).
static void lowrank_from_edges(int64_t n, int64_t nom, const double* X, const double* Omega,
                               std::vector<int64_t>& aux, std::vector<double>& U,
                               std::vector<double>& B) {
    aux.clear();
    for (int64_t t = 0; t < 2 * nom; ++t) aux.push_back((int64_t)std::llround(Omega[t]));
    std::sort(aux.begin(), aux.end());
    aux.erase(std::unique(aux.begin(), aux.end()), aux.end());  // :57 unique(Omega(:))
    for (int64_t a : aux)
        if (a < 1 || a > n) fail(KT_ERR_ARG, "Omega index out of range");
    const int k = (int)aux.size();
    U.assign((size_t)n * k, 0.0);
    B.assign((size_t)k * k, 0.0);
    for (int j = 0; j < k; ++j) U[(aux[j] - 1) + (size_t)j * n] = 1.0;  // :65-67
    auto idx = [&](double v) {
        return (int)(std::lower_bound(aux.begin(), aux.end(), (int64_t)std::llround(v)) - aux.begin());
    };
    for (int64_t t = 0; t < nom; ++t) {  // :68-73
        const int i1 = idx(Omega[t]), i2 = idx(Omega[t + nom]);
        B[i1 + (size_t)i2 * k] = X[t];
        B[i2 + (size_t)i1 * k] = X[t];
    }
}

// gr_k = -2 (base_k + Um(O1_k,:) Xm Um(O2_k,:)')   (fun_and_grad_krylov_exp.m:85-88)
static void gradient(kt_matrix_s* A, FunUpdateResult& fu, int64_t nom, const double* Omega,
                     const double* base, double* gr) {
    const int nx = fu.nx;
    if (fu.dense) {  // Um = eye(n)
        for (int64_t t = 0; t < nom; ++t) {
            const int64_t i = std::llround(Omega[t]) - 1, j = std::llround(Omega[t + nom]) - 1;
            gr[t] = -2.0 * (base[t] + fu.Xm[i + (size_t)j * nx]);
        }
        return;
    }
    BlockArnoldi& Ar = *fu.basis;
    std::vector<int64_t> rows;
    for (int64_t t = 0; t < 2 * nom; ++t) rows.push_back(std::llround(Omega[t]) - 1);
    std::vector<double> R;  // (2 nom) x (nblk PB), padded columns
    download_rows(A, Ar.V.col(0), Ar.ld(), Ar.nblk * Ar.PB, rows, R);
    const int nr = (int)rows.size();
    // Um's rows O1_k, O2_k as contiguous nx-vectors (unpadded columns)
    std::vector<double> Ur((size_t)nr * nx);
    for (int col = 0; col < nx; ++col) {
        const int pc = (col / Ar.bs) * Ar.PB + col % Ar.bs;
        for (int r = 0; r < nr; ++r) Ur[(size_t)r * nx + col] = R[r + (size_t)pc * nr];
    }
    // one entry per task on the host pool (nom x nx^2 FMAs: 2.5 M for |Omega|
    // = 30 at nx = 290, ~3 ms on one thread); same summation order as before
    HostPool::get().run((int)nom, [&](int t) {
        const double* u1 = Ur.data() + (size_t)t * nx;
        const double* u2 = Ur.data() + (size_t)(t + nom) * nx;
        double s = 0.0;
        for (int b = 0; b < nx; ++b) {
            const double* xc = fu.Xm.data() + (size_t)b * nx;
            double xb = 0.0;
            for (int a = 0; a < nx; ++a) xb += u1[a] * xc[a];
            s += xb * u2[b];
        }
        gr[t] = -2.0 * (base[t] + s);
    });
}

// Second device copy of A on its own context (stream + workspace), rebuilt
// when A was edited since (set_pairs keeps it current); nullptr when KT_TWIN=0
// or when the copy cannot be built (e.g. HBM too full for a second A and its
// workspace): the caller then runs the serial order, which needs no second
// copy, instead of failing.  A failed build is not retried until A changes.
kt_matrix_s* twin_of(kt_matrix_s* A) {
    const char* tw = getenv("KT_TWIN");  // read per call (A/B within one process)
    if (tw && tw[0] == '0') return nullptr;
    if (A->twin && A->twin_version == A->version) return A->twin;
    if (A->twin_failed && A->twin_failed_version == A->version) return nullptr;
    if (A->twin) {
        kt_matrix_destroy(A->twin);
        A->twin = nullptr;
    }
    auto give_up = [&] {
        if (A->twin) {
            kt_matrix_destroy(A->twin);
            A->twin = nullptr;
        }
        A->twin_failed = true;
        A->twin_failed_version = A->version;
        (void)hipGetLastError();  // a failed allocation must not leak into later checks
        KT_HIP(hipSetDevice(A->ctx->device));
        return (kt_matrix_s*)nullptr;
    };
    // KT_TWIN_FAULT=1 (tests): act as if the twin's allocation had failed
    const char* fault = getenv("KT_TWIN_FAULT");
    if (fault && fault[0] == '1') return give_up();
    if (!A->twin_ctx && kt_context_create(A->ctx->device, &A->twin_ctx) != KT_OK) {
        A->twin_ctx = nullptr;
        return give_up();
    }
    const int64_t n = A->n;
    std::vector<int64_t> ir(A->h_col.begin(), A->h_col.end());
    if (kt_matrix_create_csc(A->twin_ctx, n, A->h_rowptr.data(), ir.data(), A->h_val.data(), 0, &A->twin) !=
        KT_OK) {
        A->twin = nullptr;
        return give_up();
    }
    A->twin->symmetric = A->symmetric;
    A->twin->long_thresh = A->long_thresh;
    A->twin_version = A->version;
    A->twin_failed = false;
    KT_HIP(hipSetDevice(A->ctx->device));
    return A->twin;
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

int kt_householder_qr(kt_context_t ctx, int64_t n, int64_t bs, const double* W, double* Q,
                      double* R) {
    KT_TRY
    if (!ctx || !W || !Q || !R) fail(KT_ERR_ARG, "NULL argument");
    if (bs < 1 || bs > 128 || n < bs) fail(KT_ERR_UNSUPPORTED, "need 1 <= bs <= 128 and n >= bs");
    KT_HIP(hipSetDevice(ctx->device));
    DevBuf d;
    d.ensure(sizeof(double) * (size_t)n * bs);
    std::vector<double> rm((size_t)n * bs);
    for (int64_t c = 0; c < bs; ++c)
        for (int64_t i = 0; i < n; ++i) rm[(size_t)i * bs + c] = W[i + (size_t)c * n];
    KT_HIP(hipMemcpyAsync(d.ptr, rm.data(), sizeof(double) * rm.size(), hipMemcpyHostToDevice, ctx->stream));
    std::vector<double> Rv;
    householder_qr(ctx, n, d.as<double>(), (int)bs, (int)bs, Rv);
    KT_HIP(hipMemcpyAsync(rm.data(), d.ptr, sizeof(double) * rm.size(), hipMemcpyDeviceToHost, ctx->stream));
    KT_HIP(hipStreamSynchronize(ctx->stream));
    for (int64_t c = 0; c < bs; ++c)
        for (int64_t i = 0; i < n; ++i) Q[i + (size_t)c * n] = rm[(size_t)i * bs + c];
    std::copy(Rv.begin(), Rv.end(), R);
    KT_CATCH
}

int kt_normest(kt_matrix_t A, double tol, double* nrm) {
    KT_TRY
    if (!A || !nrm) fail(KT_ERR_ARG, "NULL argument");
    KT_HIP(hipSetDevice(A->ctx->device));
    *nrm = normest_impl(A, tol);
    KT_CATCH
}

int kt_trace_fun_update(kt_matrix_t A, int64_t rk, const double* U, const double* B, double tol,
                        int it, int fun, double* Xm, int* iter, int* lucky) {
    KT_TRY
    if (!A || !U || !B || !Xm || rk < 1) fail(KT_ERR_ARG, "NULL argument or empty U");
    if (rk > 128) fail(KT_ERR_UNSUPPORTED, "rank > 128");
    if (fun < KT_FUN_EXP || fun > KT_FUN_SQRT) fail(KT_ERR_ARG, "unknown fun code");
    KT_HIP(hipSetDevice(A->ctx->device));
    *Xm = trace_fun_update_impl(A, (int)rk, U, B, tol, it, fun, iter, lucky);
    KT_CATCH
}

int kt_trace_fun_update_fn(kt_matrix_t A, int64_t rk, const double* U, const double* B, double tol,
                           int it, kt_scalar_fn f, void* user, double* Xm, int* iter, int* lucky) {
    KT_TRY
    if (!A || !U || !B || !Xm || !f || rk < 1) fail(KT_ERR_ARG, "NULL argument or empty U");
    if (rk > 128) fail(KT_ERR_UNSUPPORTED, "rank > 128");
    KT_HIP(hipSetDevice(A->ctx->device));
    struct Scope {  // the handle is visible to trace_diff for this call only
        explicit Scope(ScalarFn s) { tl_scalar_fn = s; }
        ~Scope() { tl_scalar_fn = ScalarFn{}; }
    } scope(ScalarFn{f, user});
    *Xm = trace_fun_update_impl(A, (int)rk, U, B, tol, it, kFunCallback, iter, lucky);
    KT_CATCH
}

int kt_fun_update(kt_matrix_t A, int64_t rk, const double* U, const double* B, int fun, double tol,
                  int it, int64_t max_cols, double* Xm, int64_t* ncols, int* iter, int* lucky,
                  double* Um) {
    KT_TRY
    if (!A || !U || !B || !ncols || rk < 1) fail(KT_ERR_ARG, "NULL argument or empty U");
    if (fun < KT_FUN_EXP || fun > KT_FUN_SQRT) fail(KT_ERR_ARG, "unknown fun code");
    KT_HIP(hipSetDevice(A->ctx->device));
    FunUpdateResult fu = fun_update_impl(A, (int)rk, U, B, fun, tol, it);
    *ncols = fu.nx;
    if (iter) *iter = fu.iter;
    if (lucky) *lucky = fu.lucky ? 1 : 0;
    if (fu.nx > max_cols) fail(KT_ERR_ARG, "max_cols smaller than the result (query *ncols)");
    if (Xm)
        for (int j = 0; j < fu.nx; ++j)
            for (int i = 0; i < fu.nx; ++i) Xm[i + (size_t)j * fu.nx] = fu.Xm[i + (size_t)j * fu.nx];
    if (Um) {  // n x nx column-major, original numbering (fun_update.m:137)
        const int64_t n = A->n;
        if (fu.dense) {
            std::memset(Um, 0, sizeof(double) * (size_t)n * fu.nx);
            for (int64_t i = 0; i < n; ++i) Um[i + (size_t)i * n] = 1.0;
        } else {
            BlockArnoldi& Ar = *fu.basis;
            const int ldv = Ar.ld();
            std::vector<double> host((size_t)n * ldv);
            KT_HIP(hipMemcpyAsync(host.data(), Ar.V.col(0), sizeof(double) * host.size(),
                                  hipMemcpyDeviceToHost, A->ctx->stream));
            KT_HIP(hipStreamSynchronize(A->ctx->stream));
            for (int c = 0; c < fu.nx; ++c) {
                const int pc = (c / Ar.bs) * Ar.PB + c % Ar.bs;
                for (int64_t i = 0; i < n; ++i) Um[i + (size_t)c * n] = host[(size_t)i * ldv + pc];
            }
        }
    }
    KT_CATCH
}

int kt_fun_update_lanczos(kt_matrix_t A, int64_t rk, const double* U, const double* B, int fun, double tol,
                          int it, int64_t max_cols, double* Xm, int64_t* ncols, int* iter, int* lucky) {
    KT_TRY
    if (!A || !U || !B || !Xm || !ncols) fail(KT_ERR_ARG, "NULL argument");
    if (rk < 1 || rk > 128) fail(KT_ERR_ARG, "rk must be in [1, 128]");
    if (fun < KT_FUN_EXP || fun > KT_FUN_SQRT) fail(KT_ERR_ARG, "unknown fun code");
    KT_HIP(hipSetDevice(A->ctx->device));
    FunUpdateResult r = fun_update_lanczos_impl(A, (int)rk, U, B, fun, tol, it);
    if (r.nx > max_cols) fail(KT_ERR_ARG, "max_cols too small for the projected size");
    std::copy(r.Xm.begin(), r.Xm.end(), Xm);
    *ncols = r.nx;
    if (iter) *iter = r.iter;
    if (lucky) *lucky = r.lucky ? 1 : 0;
    KT_CATCH
}

int kt_fun_and_grad_krylov_exp(kt_matrix_t A, int64_t nom, const double* X, const double* Omega,
                               const double* eA, double tol, int it, double* f, double* gr) {
    KT_TRY
    if (!A || !f || !gr || (nom > 0 && (!X || !Omega || !eA))) fail(KT_ERR_ARG, "NULL argument");
    KT_HIP(hipSetDevice(A->ctx->device));
    require_symmetric(A, "FUN_AND_GRAD_KRYLOV:: matrix A is not Hermitian");  // :21-23
    const double nrmA = normest_impl(A, 1e-2);                                // :26
    double sabs = 0.0;
    for (int64_t t = 0; t < nom; ++t) sabs += std::fabs(X[t]);
    if (sabs == 0.0) {                                                        // :30-54
        *f = 0.0;
        for (int64_t t = 0; t < nom; ++t) gr[t] = -2.0 * eA[t];
        return KT_OK;
    }
    std::vector<int64_t> aux;
    std::vector<double> U, B;
    lowrank_from_edges(A->n, nom, X, Omega, aux, U, B);
    const int k = (int)aux.size();
    PhaseClock pc;
    FunUpdateResult fu = fun_update_impl(A, k, U.data(), B.data(), KT_FUN_EXP, tol * std::exp(nrmA), it);  // :83
    const double t_fu = pc.on ? pc.lap() : 0.0;
    double tr = 0.0;
    for (int i = 0; i < fu.nx; ++i) tr += fu.Xm[i + (size_t)i * fu.nx];
    *f = -tr;                                                                 // :84
    gradient(A, fu, nom, Omega, eA, gr);                                      // :85-88
    if (pc.on) fprintf(stderr, "[kt fg_exp] fun_update %.3f ms, gradient %.3f ms\n", t_fu, pc.lap());
    KT_CATCH
}

int kt_fun_and_grad_krylov_fun(kt_matrix_t A, int64_t nom, const double* X, const double* Omega,
                               int fun, int dfun, const double* dfA, double tol, int it, double* f,
                               double* gr) {
    KT_TRY
    if (!A || !f || !gr || (nom > 0 && (!X || !Omega || !dfA))) fail(KT_ERR_ARG, "NULL argument");
    if (fun < KT_FUN_EXP || fun > KT_FUN_SQRT || dfun < KT_FUN_EXP || dfun > KT_FUN_SQRT)
        fail(KT_ERR_ARG, "unknown fun code");
    KT_HIP(hipSetDevice(A->ctx->device));
    require_symmetric(A, "FUN_AND_GRAD_KRYLOV_FCONNECTIVITY:: matrix A is not Hermitian");  // :22-24
    const double nrmA = normest_impl(A, 1e-2);                                             // :27
    double sabs = 0.0;
    for (int64_t t = 0; t < nom; ++t) sabs += std::fabs(X[t]);
    if (sabs == 0.0) {                                                                     // :31-35
        *f = 0.0;
        for (int64_t t = 0; t < nom; ++t) gr[t] = -2.0 * dfA[t];
        return KT_OK;
    }
    std::vector<int64_t> aux;
    std::vector<double> U, B;
    lowrank_from_edges(A->n, nom, X, Omega, aux, U, B);
    const int k = (int)aux.size();
    // :64 and :65 are independent Krylov runs on the same A: trace_fun_update
    // runs on the twin context (own stream) on a second host thread while
    // fun_update runs here, so their kernels and host eigensolves overlap.
    const double tol_f = tol * fscalar(fun, nrmA), tol_df = tol * fscalar(dfun, nrmA);
    kt_matrix_s* A2 = twin_of(A);
    double fval = 0.0;
    Status terr{KT_OK, ""};
    RunWorker T;  // the twin's call on a persistent thread of A's context (finished on every exit)
    if (A2) {
        T.reset(ctx_worker(A->ctx, kWorkerTwin));
        T->submit([&] {
            try {
                KT_HIP(hipSetDevice(A2->ctx->device));
                fval = trace_fun_update_impl(A2, k, U.data(), B.data(), tol_f, it, fun, nullptr, nullptr);
            } catch (const Status& s) {
                terr = s;
            } catch (...) {
                terr = Status{KT_ERR_HIP, "trace_fun_update (twin) failed"};
            }
        });
    }
    PhaseClock pc;
    FunUpdateResult fu = fun_update_impl(A, k, U.data(), B.data(), dfun, tol_df, it);          // :64
    const double t_fu = pc.on ? pc.lap() : 0.0;
    bool serial = !A2;
    if (A2) {
        T->wait(0);
        if (pc.on) fprintf(stderr, "[kt fg_fun] fun_update %.3f ms, then waited %.3f ms for the twin's trace_fun_update\n",
                           t_fu, pc.lap());
        if (terr.code == KT_ERR_ALLOC) {  // the twin's workspace did not fit: serial order
            (void)hipGetLastError();
            A2->ctx->pool.clear();  // its idle scratch blocks back to the device
            KT_HIP(hipSetDevice(A->ctx->device));
            serial = true;
        } else if (terr.code != KT_OK) {
            throw terr;
        }
    }
    if (serial) {
        fval = trace_fun_update_impl(A, k, U.data(), B.data(), tol_f, it, fun, nullptr, nullptr);  // :65
    }
    *f = -fval;
    gradient(A, fu, nom, Omega, dfA, gr);                                                   // :67-70
    KT_CATCH
}

}  // extern "C"

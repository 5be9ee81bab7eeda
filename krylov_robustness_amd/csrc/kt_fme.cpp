// kt_fme.cpp -- function_multiple_entries.m on the device.
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
#include <cstring>
#include <unordered_map>

#include "kt_krylov.h"
#include "kt_launch.h"

namespace kt {

namespace {

struct Entry {
    int64_t h;    // position in omega
    int col;      // column (distinct row index) within the group
    int64_t j2;   // omega(h, 2), 0-based
    std::vector<double> Xm;  // f(Gm) e1 at convergence / last step
    std::vector<double> stop[3];
    int nstop = 0;
    bool conv = false;
};

// f(G) e1 for the j x j Arnoldi projection G (column-major); G is symmetric
// up to rounding for symmetric A and is symmetrised first (the reference's
// expm/funm of the Hessenberg G agree to that rounding).
std::vector<double> fun_e1(int j, const std::vector<double>& G, int fun) {
    std::vector<double> S((size_t)j * j), w(j), V((size_t)j * j);
    for (int b = 0; b < j; ++b)
        for (int a = 0; a < j; ++a)
            S[a + (size_t)b * j] = 0.5 * (G[a + (size_t)b * j] + G[b + (size_t)a * j]);
    sym_eig_host(j, S.data(), w.data(), V.data());
    std::vector<double> out(j, 0.0);
    for (int k = 0; k < j; ++k) {
        const double coef = fscalar(fun, w[k]) * V[0 + (size_t)k * j];
        for (int i = 0; i < j; ++i) out[i] += V[i + (size_t)k * j] * coef;
    }
    return out;
}

int run_group(kt_matrix_s* A, const std::vector<int64_t>& rows, std::vector<Entry>& ents, int fun,
              double tol, int it) {
    kt_context_s* ctx = A->ctx;
    const int64_t n = A->n;
    const int C = (int)rows.size();
    const int P = pow2_at_least(C);
    const int64_t vs = n * (int64_t)P;  // step-block stride
    DevBuf basis, Wb, part, red, idx;
    basis.ensure(sizeof(double) * (size_t)vs * (it + 1));
    Wb.ensure(sizeof(double) * (size_t)vs);
    const int nrb = col_nrb((int)n, ctx->num_cu);
    part.ensure(sizeof(double) * (size_t)nrb * P * (it + 1));
    // red: h1 | h2 | hh (it x P each) | s (P) | r (P)
    red.ensure(sizeof(double) * ((size_t)3 * it * P + 2 * P));
    double* V = basis.as<double>();
    double* W = Wb.as<double>();
    double* h1 = red.as<double>();
    double* h2 = h1 + (size_t)it * P;
    double* hh = h2 + (size_t)it * P;
    double* sq = hh + (size_t)it * P;
    double* rr = sq + P;
    std::vector<int> ridx(rows.begin(), rows.end());
    idx.ensure(sizeof(int) * ridx.size());
    KT_HIP(hipMemcpyAsync(idx.ptr, ridx.data(), sizeof(int) * ridx.size(), hipMemcpyHostToDevice,
                          ctx->stream));
    KT_HIP(hipMemsetAsync(V, 0, sizeof(double) * (size_t)vs, ctx->stream));
    KT_HIP(launch_col_select(C, P, idx.as<int>(), V, ctx->stream));
    // [V, ~] = qr(e_i, 0)   (arnoldi_krylov.m:50)
    KT_HIP(launch_col_dots((int)n, P, 1, 0, V, V, 1, ctx->num_cu, part.as<double>(), sq, ctx->stream));
    KT_HIP(launch_col_householder((int)n, P, sq, V, V, rr, ctx->stream));
    // Uaux(c) = (V' e_i)(1) = V(i, c)   (function_multiple_entries.m:94-95)
    std::vector<double> uaux(C);
    for (int c = 0; c < C; ++c)
        KT_HIP(hipMemcpyAsync(&uaux[c], V + (int64_t)rows[c] * P + c, sizeof(double),
                              hipMemcpyDeviceToHost, ctx->stream));
    KT_HIP(hipStreamSynchronize(ctx->stream));

    std::vector<std::vector<double>> H(C);  // column-major (it+1) x it per column
    const int Hld = it + 1;
    for (auto& x : H) x.assign((size_t)Hld * it, 0.0);
    std::vector<double> hb1((size_t)it * P), hb2((size_t)it * P), hbh((size_t)it * P), rb(P);
    std::vector<char> col_live(C, 1);
    const int d = 3;  // lag (function_multiple_entries.m:63)
    int j = 0;
    for (j = 1; j <= it; ++j) {
        double* Vj1 = V + (size_t)(j - 1) * vs;
        double* Vj = V + (size_t)j * vs;
        spmm(A, Vj1, P, W, P, C);  // w = A * V(:, end)   (arnoldi_krylov.m:86)
        // CGS2 against the whole basis (arnoldi_krylov.m:119-125)
        KT_HIP(launch_col_dots((int)n, P, j, vs, V, W, 0, ctx->num_cu, part.as<double>(), h1, ctx->stream));
        KT_HIP(launch_col_update((int)n, P, j, vs, V, h1, W, ctx->stream));
        KT_HIP(launch_col_dots((int)n, P, j, vs, V, W, 0, ctx->num_cu, part.as<double>(), h2, ctx->stream));
        KT_HIP(launch_col_update((int)n, P, j, vs, V, h2, W, ctx->stream));
        // [w, r] = qr(w, 0)   (:99)
        KT_HIP(launch_col_dots((int)n, P, 1, 0, W, W, 1, ctx->num_cu, part.as<double>(), sq, ctx->stream));
        KT_HIP(launch_col_householder((int)n, P, sq, W, Vj, rr, ctx->stream));
        // reorthogonalise: hh = V' w; w = w - V hh   (:104-106)
        KT_HIP(launch_col_dots((int)n, P, j, vs, V, Vj, 0, ctx->num_cu, part.as<double>(), hh, ctx->stream));
        KT_HIP(launch_col_update((int)n, P, j, vs, V, hh, Vj, ctx->stream));
        KT_HIP(hipMemcpyAsync(hb1.data(), h1, sizeof(double) * (size_t)j * P, hipMemcpyDeviceToHost, ctx->stream));
        KT_HIP(hipMemcpyAsync(hb2.data(), h2, sizeof(double) * (size_t)j * P, hipMemcpyDeviceToHost, ctx->stream));
        KT_HIP(hipMemcpyAsync(hbh.data(), hh, sizeof(double) * (size_t)j * P, hipMemcpyDeviceToHost, ctx->stream));
        KT_HIP(hipMemcpyAsync(rb.data(), rr, sizeof(double) * P, hipMemcpyDeviceToHost, ctx->stream));
        KT_HIP(hipStreamSynchronize(ctx->stream));
        for (int c = 0; c < C; ++c) {
            std::vector<double>& Hc = H[c];
            const double r = rb[c];
            for (int k = 0; k < j; ++k)  // H(1:end-1, end) = h + hh * r   (:96, :106)
                Hc[k + (size_t)(j - 1) * Hld] =
                    (hb1[(size_t)k * P + c] + hb2[(size_t)k * P + c]) + hbh[(size_t)k * P + c] * r;
            Hc[j + (size_t)(j - 1) * Hld] = r;  // H(end, end) = r   (:108)
        }
        // f(Gm) e1 for the columns that still have unconverged entries
        std::vector<std::vector<double>> F(C);
        for (int c = 0; c < C; ++c) {
            if (!col_live[c]) continue;
            std::vector<double> G((size_t)j * j);
            for (int b = 0; b < j; ++b)
                for (int a = 0; a < j; ++a) G[a + (size_t)b * j] = H[c][a + (size_t)b * Hld];
            F[c] = fun_e1(j, G, fun);
        }
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
    }
    const int iter = std::min(j, it);
    // X(h) = Um(j2, 1:nn) * Xm(:, 1) * Uaux   (:163-165)
    std::unordered_map<int64_t, std::vector<double>> urow;  // j2 -> (iter+1) x P
    for (const Entry& e : ents) {
        if (urow.count(e.j2)) continue;
        std::vector<double> buf((size_t)(iter + 1) * P);
        KT_HIP(hipMemcpy2DAsync(buf.data(), sizeof(double) * P, V + e.j2 * P, sizeof(double) * vs,
                                sizeof(double) * P, (size_t)(iter + 1), hipMemcpyDeviceToHost,
                                ctx->stream));
        urow.emplace(e.j2, std::move(buf));
    }
    KT_HIP(hipStreamSynchronize(ctx->stream));
    for (Entry& e : ents) {
        const std::vector<double>& u = urow[e.j2];
        double x = 0.0;
        for (size_t i = 0; i < e.Xm.size(); ++i) x += u[i * P + e.col] * e.Xm[i];
        e.Xm.assign(1, x * uaux[e.col]);
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

}  // namespace kt

using namespace kt;

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

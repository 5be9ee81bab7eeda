// kt_frechet.cpp -- multiple_frechet_eval.m and hessianfcn_exp.m /
// hessianfcn_fun.m on the device.
//
// multiple_frechet_eval builds, per omega entry (i, j), the row space
// K(A, e_i) and the column space K(A', e_j) by single-vector Arnoldi and
// takes the (1,2) block of f([Gm_i, Cm; 0, Hm_j']) with Cm = c e1 e1'
// (multiple_frechet_eval.m:99-163).  For the symmetric matrices the
// Hessians use (A + XX + XX'), K(A', e_t) = K(A, e_t), so one Arnoldi run per
// distinct index serves both families (ColArnoldi, kt_fme.cpp), and with
// Gm_i = Q1 L1 Q1', Hm_j' = Q2 L2 Q2' (symmetric up to rounding) the block is
// the Daleckii-Krein form
//   X = c Q1 (D o (q1 q2')) Q2',   D_ab = f[l1_a, l2_b] (divided differences),
// q = first rows of Q1, Q2 -- equal to the reference's expm/funm of the
// 2j x 2j block matrix up to rounding.  Stopping: the lag-3 spectral-norm
// test of :172-195.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <unordered_map>

#include "kt_colarnoldi.h"
#include "kt_pool.h"

namespace kt {

namespace {

double fprime(int fun, double x) {
    switch (fun) {
    case KT_FUN_EXP: return std::exp(x);
    case KT_FUN_SINH: return std::cosh(x);
    case KT_FUN_COSH: return std::sinh(x);
    case KT_FUN_SIN: return std::cos(x);
    case KT_FUN_COS: return -std::sin(x);
    case KT_FUN_LOG: return 1.0 / x;
    case KT_FUN_SQRT: return 0.5 / std::sqrt(x);
    }
    return NAN;
}

double sinhc(double x) { return std::fabs(x) < 1e-8 ? 1.0 + x * x / 6.0 : std::sinh(x) / x; }
double sinc(double x) { return std::fabs(x) < 1e-8 ? 1.0 - x * x / 6.0 : std::sin(x) / x; }

// f[a, b] = (f(a) - f(b)) / (a - b), evaluated without cancellation
double divdiff(int fun, double a, double b) {
    const double d = a - b;
    if (d == 0.0) return fprime(fun, a);
    const double m = 0.5 * (a + b), h = 0.5 * d;
    switch (fun) {
    case KT_FUN_EXP: return std::exp(b) * (std::fabs(d) < 1e-300 ? 1.0 : std::expm1(d) / d);
    case KT_FUN_SINH: return std::cosh(m) * sinhc(h);
    case KT_FUN_COSH: return std::sinh(m) * sinhc(h);
    case KT_FUN_SIN: return std::cos(m) * sinc(h);
    case KT_FUN_COS: return -std::sin(m) * sinc(h);
    case KT_FUN_LOG: return std::log1p(d / b) / d;
    case KT_FUN_SQRT: return 1.0 / (std::sqrt(a) + std::sqrt(b));
    }
    return NAN;
}

struct FEntry {
    int ti, tj;                 // index slots of omega(h,1), omega(h,2)
    int nn = 0;                 // size of Xm
    std::vector<double> Xm;     // nn x nn column-major
    std::vector<double> stop[3];
    int nstop = 0;
    bool conv = false;
};

double spectral_norm(int m, const std::vector<double>& M) {
    std::vector<double> G((size_t)m * m, 0.0), w(m);
    for (int j = 0; j < m; ++j)
        for (int i = 0; i < m; ++i) {
            double s = 0.0;
            for (int l = 0; l < m; ++l) s += M[l + (size_t)i * m] * M[l + (size_t)j * m];
            G[i + (size_t)j * m] = s;
        }
    sym_eig_host(m, G.data(), w.data(), nullptr);
    double mx = 0.0;
    for (double v : w) mx = std::max(mx, v);
    return std::sqrt(mx);
}

struct Slot {
    int group, col;
};

}  // namespace

// out[h + t * k] = Df(A)(e_oi[h] e_oj[h]')(ri[t], rj[t]); returns iterations
int frechet_entries_impl(kt_matrix_s* A, int64_t k, const int64_t* oi, const int64_t* oj, int fun,
                         double tol, int it, int64_t nt, const int64_t* ri, const int64_t* rj,
                         double* out) {
    const int64_t n = A->n;
    if (it <= 0) it = (int)std::min<int64_t>(100, n);  // :35-37
    for (int64_t h = 0; h < k; ++h)
        if (oi[h] < 0 || oi[h] >= n || oj[h] < 0 || oj[h] >= n)
            fail(KT_ERR_ARG, "omega index out of range");
    for (int64_t t = 0; t < nt; ++t)
        if (ri[t] < 0 || ri[t] >= n || rj[t] < 0 || rj[t] >= n)
            fail(KT_ERR_ARG, "target index out of range");
    // distinct indices of both families (unique(.., 'stable'), :57-58)
    std::vector<int64_t> T;
    std::unordered_map<int64_t, int> slot_of;
    auto add = [&](int64_t x) {
        if (!slot_of.count(x)) {
            slot_of.emplace(x, (int)T.size());
            T.push_back(x);
        }
    };
    for (int64_t h = 0; h < k; ++h) add(oi[h]);
    for (int64_t h = 0; h < k; ++h) add(oj[h]);
    std::vector<std::unique_ptr<ColArnoldi>> groups;
    std::vector<Slot> slot(T.size());
    for (size_t g0 = 0; g0 < T.size(); g0 += 128) {
        const size_t g1 = std::min(T.size(), g0 + 128);
        std::vector<int64_t> st(T.begin() + g0, T.begin() + g1);
        groups.emplace_back(new ColArnoldi(A, st, it));
        for (size_t s = g0; s < g1; ++s) slot[s] = {(int)groups.size() - 1, (int)(s - g0)};
    }
    std::vector<FEntry> ents(k);
    for (int64_t h = 0; h < k; ++h) {
        ents[h].ti = slot_of[oi[h]];
        ents[h].tj = slot_of[oj[h]];
    }
    const int d = 3;  // :80
    int j = 0;
    // one group (<= 128 distinct indices): the host work of step j below runs
    // while the device runs step j + 1 (as function_multiple_entries; the
    // speculative step's block is never read when step j stops).  Same
    // arithmetic, same results; KT_FRECHET_PIPE=0 steps first, then works.
    const char* pe = getenv("KT_FRECHET_PIPE");
    const bool pipe = groups.size() == 1 && !(pe && pe[0] == '0');
    if (pipe) groups[0]->step();
    for (j = 1; j <= it; ++j) {
        if (!pipe) {
            for (auto& g : groups) g->step();
        } else if (j < it) {
            groups[0]->step_launch();
        }
        // eigendecompositions of the live projections
        std::vector<char> live(T.size(), 0);
        for (const FEntry& e : ents)
            if (!e.conv) live[e.ti] = live[e.tj] = 1;
        // the per-index eigensolves and the per-entry blocks are independent:
        // spread over the host pool (they are the step's critical path on a
        // small graph; the device step takes a fraction of it)
        std::vector<std::vector<double>> W(T.size()), Q(T.size());
        std::vector<int> ls;
        for (size_t s = 0; s < T.size(); ++s)
            if (live[s]) ls.push_back((int)s);
        HostPool& pool = HostPool::get();
        pool.run((int)ls.size(), [&](int i) {
            const int s = ls[i];
            std::vector<double> Gs;
            groups[slot[s].group]->gm(slot[s].col, Gs);
            sym_eig_small(j, Gs, W[s], Q[s]);
        }, 4);
        std::vector<int> act;
        for (size_t h = 0; h < ents.size(); ++h)
            if (!ents[h].conv) act.push_back((int)h);
        std::vector<char> open_(act.size(), 0);  // entry not stopped at this step
        pool.run((int)act.size(), [&](int i) {
            FEntry& e = ents[act[i]];
            const double c = groups[slot[e.ti].group]->uaux(slot[e.ti].col) *
                             groups[slot[e.tj].group]->uaux(slot[e.tj].col);  // Cm(1,1)  :152
            const std::vector<double>& Q1 = Q[e.ti];
            const std::vector<double>& Q2 = Q[e.tj];
            std::vector<double> M((size_t)j * j), Tm((size_t)j * j, 0.0), X((size_t)j * j, 0.0);
            for (int b = 0; b < j; ++b)
                for (int a = 0; a < j; ++a)
                    M[a + (size_t)b * j] = c * divdiff(fun, W[e.ti][a], W[e.tj][b]) *
                                           Q1[(size_t)a * j] * Q2[(size_t)b * j];
            // X = Q1 M Q2'
            for (int b = 0; b < j; ++b)
                for (int l = 0; l < j; ++l) {
                    const double m = M[l + (size_t)b * j];
                    if (m == 0.0) continue;
                    for (int a = 0; a < j; ++a) Tm[a + (size_t)b * j] += Q1[a + (size_t)l * j] * m;
                }
            for (int b = 0; b < j; ++b)
                for (int l = 0; l < j; ++l) {
                    const double q = Q2[b + (size_t)l * j];
                    for (int a = 0; a < j; ++a) X[a + (size_t)b * j] += Tm[a + (size_t)l * j] * q;
                }
            e.Xm.swap(X);
            e.nn = j;
            if (j <= d) {
                e.stop[j - 1] = e.Xm;
                open_[i] = 1;
            } else {
                const std::vector<double>& old = e.stop[0];
                const int no = (int)std::lround(std::sqrt((double)old.size()));
                std::vector<double> D = e.Xm;
                for (int b = 0; b < no; ++b)
                    for (int a = 0; a < no; ++a) D[a + (size_t)b * j] -= old[a + (size_t)b * no];
                const double err = spectral_norm(j, D);  // norm(Xm - Xstop{1})   :172
                if (err > tol) open_[i] = 1;
                else e.conv = true;
                e.stop[0] = std::move(e.stop[1]);
                e.stop[1] = std::move(e.stop[2]);
                e.stop[2] = e.Xm;
            }
        }, 4);
        bool stop = true;
        for (char o : open_) stop = stop && !o;
        if (stop) break;
        if (pipe) groups[0]->step_finish();
    }
    const int iter = std::min(j, it);
    // basis rows at every target row, for every index slot
    std::vector<int64_t> R;
    std::unordered_map<int64_t, size_t> rpos;
    for (int64_t t = 0; t < nt; ++t)
        for (int64_t r : {ri[t], rj[t]})
            if (!rpos.count(r)) {
                rpos.emplace(r, R.size());
                R.push_back(r);
            }
    const int nk = iter;  // Um = Um(:, 1:end-rk)   (:207-212)
    std::vector<std::vector<double>> rowsv(groups.size());
    for (size_t g = 0; g < groups.size(); ++g) groups[g]->rows(R, nk, rowsv[g]);
    auto U = [&](int s, int64_t r, int a) {
        const Slot& sl = slot[s];
        const int C = groups[sl.group]->cols();
        return rowsv[sl.group][(rpos[r] * nk + a) * C + sl.col];
    };
    for (int64_t h = 0; h < k; ++h) {
        const FEntry& e = ents[h];
        for (int64_t t = 0; t < nt; ++t) {
            double s = 0.0;
            for (int b = 0; b < e.nn; ++b) {
                const double vb = U(e.tj, rj[t], b);
                if (vb == 0.0) continue;
                double col = 0.0;
                for (int a = 0; a < e.nn; ++a) col += U(e.ti, ri[t], a) * e.Xm[a + (size_t)b * e.nn];
                s += col * vb;
            }
            out[h + t * k] = s;
        }
    }
    return iter;
}

// A + XX + XX' for XX = sparse(Omega(:,1), Omega(:,2), X)  (hessianfcn_exp.m:5-7)
static kt_matrix_s* matrix_plus_edges(kt_matrix_s* A, int64_t k, const int64_t* oi,
                                      const int64_t* oj, const double* x) {
    const int64_t n = A->n;
    std::vector<std::vector<std::pair<int32_t, double>>> add(n);
    for (int64_t h = 0; h < k; ++h) {
        add[oi[h]].push_back({(int32_t)oj[h], x[h]});
        add[oj[h]].push_back({(int32_t)oi[h], x[h]});
    }
    auto* B = new kt_matrix_s();
    B->ctx = A->ctx;
    B->n = n;
    B->h_rowptr.assign(n + 1, 0);
    for (int64_t i = 0; i < n; ++i) {
        std::vector<std::pair<int32_t, double>> row;
        for (int64_t t = A->h_rowptr[i]; t < A->h_rowptr[i + 1]; ++t) row.push_back({A->h_col[t], A->h_val[t]});
        row.insert(row.end(), add[i].begin(), add[i].end());
        std::stable_sort(row.begin(), row.end(), [](const auto& p, const auto& q) { return p.first < q.first; });
        for (size_t t = 0; t < row.size(); ++t) {
            if (!B->h_col.empty() && (int64_t)B->h_col.size() > B->h_rowptr[i] && B->h_col.back() == row[t].first)
                B->h_val.back() += row[t].second;  // sparse() sums duplicates
            else {
                B->h_col.push_back(row[t].first);
                B->h_val.push_back(row[t].second);
            }
        }
        B->h_rowptr[i + 1] = (int64_t)B->h_col.size();
    }
    B->nnz = (int64_t)B->h_col.size();
    B->symmetric = 1;
    refresh_device(B);
    return B;
}

}  // namespace kt

using namespace kt;

extern "C" {

int kt_frechet_entries(kt_matrix_t A, int64_t k, const int64_t* oi, const int64_t* oj, int fun,
                       double tol, int it, int64_t ntarget, const int64_t* ti, const int64_t* tj,
                       double* out, int* iter) {
    try {
        if (!A || (k > 0 && (!oi || !oj)) || (ntarget > 0 && (!ti || !tj || !out)))
            fail(KT_ERR_ARG, "NULL argument");
        if (k < 0 || ntarget < 0) fail(KT_ERR_ARG, "negative count");
        if (fun < KT_FUN_EXP || fun > KT_FUN_SQRT) fail(KT_ERR_UNSUPPORTED, "unsupported function");
        KT_HIP(hipSetDevice(A->ctx->device));
        require_symmetric(A, "MULTIPLE_FRECHET_EVAL:: symmetric A required by this implementation");
        const int r = frechet_entries_impl(A, k, oi, oj, fun, tol, it, ntarget, ti, tj, out);
        if (iter) *iter = r;
    } catch (const Status& s) {
        set_error(s.msg);
        return s.code;
    } catch (const std::bad_alloc&) {
        set_error("host allocation failed");
        return KT_ERR_ALLOC;
    }
    return KT_OK;
}

int kt_hessianfcn(kt_matrix_t A, int64_t nomega, const double* X, const double* Omega, int fun,
                  double tol, int it, double* Hes) {
    kt_matrix_s* B = nullptr;
    try {
        if (!A || !X || !Omega || !Hes) fail(KT_ERR_ARG, "NULL argument");
        if (nomega < 1) fail(KT_ERR_ARG, "empty Omega");
        if (fun < KT_FUN_EXP || fun > KT_FUN_SQRT) fail(KT_ERR_UNSUPPORTED, "unsupported function");
        KT_HIP(hipSetDevice(A->ctx->device));
        require_symmetric(A, "HESSIANFCN:: symmetric A required by this implementation");
        const int64_t n = A->n;
        std::vector<int64_t> oi(nomega), oj(nomega);
        for (int64_t h = 0; h < nomega; ++h) {
            oi[h] = (int64_t)Omega[h] - 1;
            oj[h] = (int64_t)Omega[h + nomega] - 1;
            if (oi[h] < 0 || oi[h] >= n || oj[h] < 0 || oj[h] >= n) fail(KT_ERR_ARG, "Omega index out of range");
        }
        B = matrix_plus_edges(A, nomega, oi.data(), oj.data(), X);  // Atilde   :5-7
        std::vector<double> F((size_t)nomega * nomega);
        frechet_entries_impl(B, nomega, oi.data(), oj.data(), fun, tol, it, nomega, oi.data(), oj.data(),
                             F.data());  // :8
        for (int64_t j = 0; j < nomega; ++j) {  // :9-15 (upper triangle, mirrored)
            for (int64_t l = j; l < nomega; ++l) Hes[j + l * nomega] = -2.0 * F[j + l * nomega];
            for (int64_t l = j + 1; l < nomega; ++l) Hes[l + j * nomega] = Hes[j + l * nomega];
        }
    } catch (const Status& s) {
        if (B) { B->hub.release(); B->nat.release(); delete B; }
        set_error(s.msg);
        return s.code;
    } catch (const std::bad_alloc&) {
        if (B) { B->hub.release(); B->nat.release(); delete B; }
        set_error("host allocation failed");
        return KT_ERR_ALLOC;
    }
    if (B) {
        (void)hipStreamSynchronize(B->ctx->stream);
        B->hub.release();
        B->nat.release();
        delete B;
    }
    return KT_OK;
}

}  // extern "C"

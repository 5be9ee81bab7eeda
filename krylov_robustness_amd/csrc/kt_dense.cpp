// kt_dense.cpp -- small dense host linear algebra for the projected problems.
//
// The m x m tridiagonal eigenproblem of each probe is solved on the host, as
// the north star prescribes (BASELINE.json north_star):
// implicit-shift QL that rotates only the first row of the eigenvector matrix
// (Golub-Welsch), giving theta_k and tau_k = (Q e1)_k for the quadrature
//   e1' f(T) e1 = sum_k tau_k^2 f(theta_k).
#include <cfloat>
#include <cmath>

#include "kt_internal.h"

namespace kt {

double fscalar(int fun, double x) {
    switch (fun) {
    case KT_FUN_EXP: return std::exp(x);
    case KT_FUN_SINH: return std::sinh(x);
    case KT_FUN_COSH: return std::cosh(x);
    case KT_FUN_SIN: return std::sin(x);
    case KT_FUN_COS: return std::cos(x);
    case KT_FUN_LOG: return std::log(x);
    case KT_FUN_SQRT: return std::sqrt(x);
    default: return NAN;
    }
}

// Symmetric tridiagonal (d[0..m-1], e[0..m-2]) -> eigenvalues in d and the
// first eigenvector components in z.
static void ql_first_row(int m, double* d, double* e, double* z) {
    e[m - 1] = 0.0;
    for (int i = 0; i < m; ++i) z[i] = (i == 0) ? 1.0 : 0.0;
    for (int l = 0; l < m; ++l) {
        int iter = 0;
        for (;;) {
            int mm = l;
            for (; mm < m - 1; ++mm) {
                const double dd = std::fabs(d[mm]) + std::fabs(d[mm + 1]);
                if (std::fabs(e[mm]) <= DBL_EPSILON * dd) break;
            }
            if (mm == l || iter++ == 100) break;
            double g = (d[l + 1] - d[l]) / (2.0 * e[l]);
            double r = std::hypot(g, 1.0);
            g = d[mm] - d[l] + e[l] / (g + std::copysign(r, g));
            double s = 1.0, c = 1.0, p = 0.0;
            bool deflated = false;
            for (int i = mm - 1; i >= l; --i) {
                const double f = s * e[i], b = c * e[i];
                r = std::hypot(f, g);
                e[i + 1] = r;
                if (r == 0.0) {
                    d[i + 1] -= p;
                    e[mm] = 0.0;
                    deflated = true;
                    break;
                }
                s = f / r;
                c = g / r;
                g = d[i + 1] - p;
                r = (d[i] - g) * s + 2.0 * c * b;
                p = s * r;
                d[i + 1] = g + p;
                g = c * r - b;
                const double zf = z[i + 1];
                z[i + 1] = s * z[i] + c * zf;
                z[i] = c * z[i] - s * zf;
            }
            if (deflated) continue;
            d[l] -= p;
            e[l] = g;
            e[mm] = 0.0;
        }
    }
}

double tridiag_quadrature(int m, const double* alpha, const double* off, int fun) {
    if (m <= 0) return 0.0;
    std::vector<double> d(alpha, alpha + m), e(m, 0.0), z(m);
    for (int i = 0; i + 1 < m; ++i) e[i] = off[i];
    ql_first_row(m, d.data(), e.data(), z.data());
    double q = 0.0;
    for (int i = 0; i < m; ++i) q += z[i] * z[i] * fscalar(fun, d[i]);
    return q;
}

}  // namespace kt

// ---------------------------------------------------------------------------
// Small dense symmetric/triangular kernels on the host (column-major).
// Used for the projected problems of the block-Krylov paths:
//   CholQR factors (lanczos_krylov.m:48,90 qr), eig of Gm / tGm
//   (trace_fun_update.m:83-84), f(tGm) - f(Gm) (fun_update.m:106).
// ---------------------------------------------------------------------------
namespace kt {

// G = R'R, R upper (in place over the upper triangle; lower zeroed).
bool chol_upper(double* G, int n) {
    for (int j = 0; j < n; ++j) {
        double d = G[j + j * n];
        for (int k = 0; k < j; ++k) d -= G[k + j * n] * G[k + j * n];
        if (!(d > 0.0)) return false;
        d = std::sqrt(d);
        G[j + j * n] = d;
        for (int i = j + 1; i < n; ++i) {
            double s = G[j + i * n];
            for (int k = 0; k < j; ++k) s -= G[k + j * n] * G[k + i * n];
            G[j + i * n] = s / d;
        }
    }
    for (int j = 0; j < n; ++j)
        for (int i = j + 1; i < n; ++i) G[i + j * n] = 0.0;
    return true;
}

// Rinv = R^{-1} for upper triangular R (column-major).
void tri_upper_inv(const double* R, int n, double* X) {
    for (int i = 0; i < n * n; ++i) X[i] = 0.0;
    for (int j = 0; j < n; ++j) {
        X[j + j * n] = 1.0 / R[j + j * n];
        for (int i = j - 1; i >= 0; --i) {
            double s = 0.0;
            for (int k = i + 1; k <= j; ++k) s += R[i + k * n] * X[k + j * n];
            X[i + j * n] = -s / R[i + i * n];
        }
    }
}

// Householder reduction of a symmetric matrix to tridiagonal form (d, e) with
// the accumulated orthogonal transform in Z (if want_vectors), followed by
// implicit-shift QL.  On exit: w ascending eigenvalues, Z (col-major) the
// eigenvectors.  Classic tred2/tql2 structure, written for column-major.
static void tred2(int n, double* a /* in: sym, out: Q */, double* d, double* e, bool vecs) {
    for (int i = n - 1; i > 0; --i) {
        const int l = i - 1;
        double h = 0.0, scale = 0.0;
        if (l > 0) {
            for (int k = 0; k <= l; ++k) scale += std::fabs(a[i + k * n]);
            if (scale == 0.0) {
                e[i] = a[i + l * n];
            } else {
                for (int k = 0; k <= l; ++k) {
                    a[i + k * n] /= scale;
                    h += a[i + k * n] * a[i + k * n];
                }
                double f = a[i + l * n];
                double g = (f >= 0.0 ? -std::sqrt(h) : std::sqrt(h));
                e[i] = scale * g;
                h -= f * g;
                a[i + l * n] = f - g;
                f = 0.0;
                for (int j = 0; j <= l; ++j) {
                    a[j + i * n] = a[i + j * n] / h;
                    g = 0.0;
                    for (int k = 0; k <= j; ++k) g += a[j + k * n] * a[i + k * n];
                    for (int k = j + 1; k <= l; ++k) g += a[k + j * n] * a[i + k * n];
                    e[j] = g / h;
                    f += e[j] * a[i + j * n];
                }
                const double hh = f / (h + h);
                for (int j = 0; j <= l; ++j) {
                    f = a[i + j * n];
                    e[j] = g = e[j] - hh * f;
                    for (int k = 0; k <= j; ++k) a[j + k * n] -= (f * e[k] + g * a[i + k * n]);
                }
            }
        } else {
            e[i] = a[i + l * n];
        }
        d[i] = h;
    }
    d[0] = 0.0;
    e[0] = 0.0;
    if (!vecs) {  // eigenvalues only: no accumulation of the transformations
        for (int i = 0; i < n; ++i) d[i] = a[i + i * n];
        return;
    }
    for (int i = 0; i < n; ++i) {
        const int l = i - 1;
        if (d[i] != 0.0) {
            for (int j = 0; j <= l; ++j) {
                double g = 0.0;
                for (int k = 0; k <= l; ++k) g += a[i + k * n] * a[k + j * n];
                for (int k = 0; k <= l; ++k) a[k + j * n] -= g * a[k + i * n];
            }
        }
        d[i] = a[i + i * n];
        a[i + i * n] = 1.0;
        for (int j = 0; j <= l; ++j) a[j + i * n] = a[i + j * n] = 0.0;
    }
}

static void tql2(int n, double* d, double* e, double* z /* nullable */) {
    for (int i = 1; i < n; ++i) e[i - 1] = e[i];
    e[n - 1] = 0.0;
    for (int l = 0; l < n; ++l) {
        int iter = 0;
        for (;;) {
            int m = l;
            for (; m < n - 1; ++m) {
                const double dd = std::fabs(d[m]) + std::fabs(d[m + 1]);
                if (std::fabs(e[m]) <= DBL_EPSILON * dd) break;
            }
            if (m == l || iter++ == 200) break;
            double g = (d[l + 1] - d[l]) / (2.0 * e[l]);
            double r = std::hypot(g, 1.0);
            g = d[m] - d[l] + e[l] / (g + std::copysign(r, g));
            double s = 1.0, c = 1.0, p = 0.0;
            bool deflated = false;
            for (int i = m - 1; i >= l; --i) {
                double f = s * e[i];
                const double b = c * e[i];
                r = std::hypot(f, g);
                e[i + 1] = r;
                if (r == 0.0) {
                    d[i + 1] -= p;
                    e[m] = 0.0;
                    deflated = true;
                    break;
                }
                s = f / r;
                c = g / r;
                g = d[i + 1] - p;
                r = (d[i] - g) * s + 2.0 * c * b;
                p = s * r;
                d[i + 1] = g + p;
                g = c * r - b;
                if (z) {
                    for (int k = 0; k < n; ++k) {
                        f = z[k + (i + 1) * n];
                        z[k + (i + 1) * n] = s * z[k + i * n] + c * f;
                        z[k + i * n] = c * z[k + i * n] - s * f;
                    }
                }
            }
            if (deflated) continue;
            d[l] -= p;
            e[l] = g;
            e[m] = 0.0;
        }
    }
    // sort ascending (selection sort; n is small)
    for (int i = 0; i < n - 1; ++i) {
        int k = i;
        for (int j = i + 1; j < n; ++j)
            if (d[j] < d[k]) k = j;
        if (k != i) {
            std::swap(d[i], d[k]);
            if (z)
                for (int r = 0; r < n; ++r) std::swap(z[r + i * n], z[r + k * n]);
        }
    }
}

void sym_eig_host(int n, const double* A, double* w, double* V /* nullable */) {
    if (n <= 0) return;
    std::vector<double> a(A, A + (size_t)n * n), e(n);
    tred2(n, a.data(), w, e.data(), V != nullptr);
    tql2(n, w, e.data(), V ? a.data() : nullptr);
    if (V) std::copy(a.begin(), a.end(), V);
}

// F = V f(diag(w)) V'
void sym_fun_from_eig(int n, const double* w, const double* V, int fun, double* F) {
    std::vector<double> fw(n);
    for (int k = 0; k < n; ++k) fw[k] = fscalar(fun, w[k]);
    for (int j = 0; j < n; ++j)
        for (int i = 0; i < n; ++i) F[i + j * n] = 0.0;
    for (int k = 0; k < n; ++k) {
        const double* v = V + (size_t)k * n;
        for (int j = 0; j < n; ++j) {
            const double s = fw[k] * v[j];
            double* Fj = F + (size_t)j * n;
            for (int i = 0; i < n; ++i) Fj[i] += v[i] * s;
        }
    }
}

}  // namespace kt

extern "C" int kt_host_sym_eig(int n, const double* A, double* w, double* V) {
    if (n < 0 || (n > 0 && (!A || !w))) {
        kt::set_error("kt_host_sym_eig: bad argument");
        return KT_ERR_ARG;
    }
    kt::sym_eig_host(n, A, w, V);
    return KT_OK;
}

// kt_dense.cpp -- small dense host linear algebra for the projected problems.
//
// The m x m tridiagonal eigenproblem of each probe is solved on the host, as
// the north star prescribes (BASELINE.json north_star):
// implicit-shift QL that rotates only the first row of the eigenvector matrix
// (Golub-Welsch), giving theta_k and tau_k = (Q e1)_k for the quadrature
//   e1' f(T) e1 = sum_k tau_k^2 f(theta_k).
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdlib>

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

// Radius of a plane rotation: sqrt(f^2 + g^2), rescaled through hypot only
// when the squares could leave the double range.  (glibc's hypot is a libm
// call of ~20 ns; the QL sweep below is a serial chain of ~m^2 rotations, so
// at m = 30 hypot alone was 40% of a column's quadrature.)
static inline double rot_radius(double f, double g) {
    const double af = std::fabs(f), ag = std::fabs(g);
    const double mx = af > ag ? af : ag;
    if (mx > 1e150 || (mx < 1e-150 && mx > 0.0)) return std::hypot(f, g);
    return std::sqrt(f * f + g * g);
}

struct Rot {
    int i;
    double s, c;
};

// Symmetric tridiagonal (d[0..m-1], e[0..m-2]) -> eigenvalues in d and the
// first eigenvector components in z (implicit-shift QL rotating only the first
// row of the eigenvector matrix Z).  With `log`, every rotation applied to z
// is recorded in order: Z = R_1 R_2 ... R_k, R_j acting on columns (i, i+1).
// (The QL iteration is EISPACK IMTQL2's, public domain: Bowdler, Martin,
// Reinsch & Wilkinson, Numer. Math. 11 (1968); first-row form after Golub &
// Welsch, Math. Comp. 23 (1969).)
static void ql_first_row(int m, double* d, double* e, double* z, std::vector<Rot>* log = nullptr) {
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
            double r = rot_radius(g, 1.0);
            g = d[mm] - d[l] + e[l] / (g + std::copysign(r, g));
            double s = 1.0, c = 1.0, p = 0.0;
            bool deflated = false;
            for (int i = mm - 1; i >= l; --i) {
                const double f = s * e[i], b = c * e[i];
                r = rot_radius(f, g);
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
                if (log) log->push_back({i, s, c});
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

// The quadrature and f(T) e1 = Z f(Theta) Z' e1 from one QL pass: Z' e1 = z
// (the rotated first row), and Z v = R_1 (R_2 (... R_k v)) replays the logged
// rotations backwards on the one vector v = f(theta) .* z -- O(rotations),
// where forming Z (tred2 + tql2 with vectors) costs m times that.
double tridiag_fun_e1(int m, const double* alpha, const double* off, int fun, double* fe1) {
    if (m <= 0) return 0.0;
    std::vector<double> d(alpha, alpha + m), e(m, 0.0), z(m);
    for (int i = 0; i + 1 < m; ++i) e[i] = off[i];
    std::vector<Rot> log;
    log.reserve((size_t)4 * m * m);
    ql_first_row(m, d.data(), e.data(), z.data(), &log);
    double q = 0.0;
    for (int k = 0; k < m; ++k) {
        const double fk = fscalar(fun, d[k]);
        q += z[k] * z[k] * fk;
        fe1[k] = fk * z[k];
    }
    for (size_t j = log.size(); j-- > 0;) {
        const Rot& R = log[j];
        const double a = fe1[R.i], b = fe1[R.i + 1];
        fe1[R.i] = R.c * a + R.s * b;
        fe1[R.i + 1] = R.c * b - R.s * a;
    }
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
// eigenvectors, written for column-major.
// Source: the EISPACK routines TRED2 (Householder tridiagonalisation, with
// the transform accumulated) and IMTQL2 / TQL2 (implicit-shift QL), public
// domain -- Martin, Reinsch & Wilkinson, "Householder's tridiagonalization of a
// symmetric matrix" and Bowdler, Martin, Reinsch & Wilkinson, "The QR and QL
// algorithms for symmetric matrices", Numer. Math. 11 (1968), Handbook for
// Automatic Computation vol. II (Wilkinson & Reinsch 1971), contributions II/2
// and II/3; Smith et al., EISPACK Guide (1976).
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
            double r = rot_radius(g, 1.0);
            g = d[m] - d[l] + e[l] / (g + std::copysign(r, g));
            double s = 1.0, c = 1.0, p = 0.0;
            bool deflated = false;
            for (int i = m - 1; i >= l; --i) {
                double f = s * e[i];
                const double b = c * e[i];
                r = rot_radius(f, g);
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

// Eigenvalues only, larger n: Householder tridiagonalisation from the left
// on the lower triangle of the column-major copy -- every inner loop runs
// down a contiguous column (symmetric matrix-vector product and rank-2
// update), where tred2's walk along rows strides by n.  Golub & Van Loan's
// house(): P x = mu e1, so the subdiagonal is mu.  Output in tql2's layout
// (e[i] couples i-1 and i, e[0] unused).
template <int>
static inline __attribute__((always_inline)) void tridiag_lower_cols(int n, double* __restrict__ a, double* __restrict__ d,
                                                                     double* __restrict__ e, double* __restrict__ v,
                                                                     double* __restrict__ p) {
    for (int k = 0; k + 2 < n; ++k) {
        const int m = n - k - 1;
        double* x = a + (k + 1) + (size_t)k * n;  // A(k+1:n, k)
        double sigma = 0.0;
        for (int i = 1; i < m; ++i) sigma += x[i] * x[i];
        d[k] = a[k + (size_t)k * n];
        const double alpha = x[0];
        if (sigma == 0.0) {  // already reduced in this column
            e[k + 1] = alpha;
            continue;
        }
        const double mu = std::sqrt(alpha * alpha + sigma);
        const double v0 = alpha <= 0.0 ? alpha - mu : -sigma / (alpha + mu);
        const double tau = 2.0 * v0 * v0 / (sigma + v0 * v0);
        const double iv0 = 1.0 / v0;
        v[0] = 1.0;
        for (int i = 1; i < m; ++i) v[i] = x[i] * iv0;
        e[k + 1] = mu;
        double* __restrict__ B = a + (k + 1) + (size_t)(k + 1) * n;  // trailing block, lower triangle valid
        // p = tau B v (B symmetric, lower triangle stored)
        for (int i = 0; i < m; ++i) p[i] = 0.0;
        for (int j = 0; j < m; ++j) {
            const double* __restrict__ col = B + (size_t)j * n;
            const double vj = v[j];
            double s0 = col[j] * vj, s1 = 0.0, s2 = 0.0, s3 = 0.0;  // 4 partial sums: vectorisable
            int i = j + 1;
            for (; i + 3 < m; i += 4) {
                p[i] += col[i] * vj;
                p[i + 1] += col[i + 1] * vj;
                p[i + 2] += col[i + 2] * vj;
                p[i + 3] += col[i + 3] * vj;
                s0 += col[i] * v[i];
                s1 += col[i + 1] * v[i + 1];
                s2 += col[i + 2] * v[i + 2];
                s3 += col[i + 3] * v[i + 3];
            }
            for (; i < m; ++i) {
                p[i] += col[i] * vj;
                s0 += col[i] * v[i];
            }
            p[j] += (s0 + s1) + (s2 + s3);
        }
        double pv = 0.0;
        for (int i = 0; i < m; ++i) {
            p[i] *= tau;
            pv += p[i] * v[i];
        }
        const double K = 0.5 * tau * pv;
        for (int i = 0; i < m; ++i) p[i] -= K * v[i];  // w
        // B -= v w' + w v' (lower triangle)
        for (int j = 0; j < m; ++j) {
            double* __restrict__ col = B + (size_t)j * n;
            const double vj = v[j], wj = p[j];
            for (int i = j; i < m; ++i) col[i] -= v[i] * wj + p[i] * vj;
        }
    }
    if (n >= 2) {
        d[n - 2] = a[(n - 2) + (size_t)(n - 2) * n];
        e[n - 1] = a[(n - 1) + (size_t)(n - 2) * n];
    }
    d[n - 1] = a[(n - 1) + (size_t)(n - 1) * n];
    e[0] = 0.0;
}

__attribute__((target("avx2,fma"))) static void tridiag_lower_cols_avx2(int n, double* a, double* d, double* e,
                                                                        double* v, double* p) {
    tridiag_lower_cols<1>(n, a, d, e, v, p);
}
static void tridiag_lower_cols_base(int n, double* a, double* d, double* e, double* v, double* p) {
    tridiag_lower_cols<0>(n, a, d, e, v, p);
}

// tql2 without eigenvectors for the column path (EISPACK TQL1 / IMTQL1 form)
static void tql_values(int n, double* d, double* e) {
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
            double r = rot_radius(g, 1.0);
            g = d[m] - d[l] + e[l] / (g + std::copysign(r, g));
            double s = 1.0, c = 1.0, p = 0.0;
            bool deflated = false;
            for (int i = m - 1; i >= l; --i) {
                const double f = s * e[i];
                const double b = c * e[i];
                r = rot_radius(f, g);
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
            }
            if (deflated) continue;
            d[l] -= p;
            e[l] = g;
            e[m] = 0.0;
        }
    }
    std::sort(d, d + n);
}

// values-only problems from this size take tridiag_lower_cols (smaller ones,
// e.g. the greedy candidates' 2j x 2j projections, keep tred2 bit for bit)
constexpr int kColTridiagMinN = 96;

void sym_eig_host(int n, const double* A, double* w, double* V /* nullable */) {
    if (n <= 0) return;
    if (!V && n >= kColTridiagMinN) {
        std::vector<double> a(A, A + (size_t)n * n), e(n), v(n), p(n);
        static const bool avx2 = __builtin_cpu_supports("avx2") && __builtin_cpu_supports("fma");
        if (avx2) tridiag_lower_cols_avx2(n, a.data(), w, e.data(), v.data(), p.data());
        else tridiag_lower_cols_base(n, a.data(), w, e.data(), v.data(), p.data());
        tql_values(n, w, e.data());
        return;
    }
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

extern "C" int kt_host_tridiag_quad(int m, const double* alpha, const double* off, int fun, double* q,
                                    double* fe1) {
    if (m < 1 || !alpha || (m > 1 && !off) || !q || fun < KT_FUN_EXP || fun > KT_FUN_SQRT) {
        kt::set_error("kt_host_tridiag_quad: bad argument");
        return KT_ERR_ARG;
    }
    *q = fe1 ? kt::tridiag_fun_e1(m, alpha, off, fun, fe1) : kt::tridiag_quadrature(m, alpha, off, fun);
    return KT_OK;
}

extern "C" int kt_host_sym_eig(int n, const double* A, double* w, double* V) {
    if (n < 0 || (n > 0 && (!A || !w))) {
        kt::set_error("kt_host_sym_eig: bad argument");
        return KT_ERR_ARG;
    }
    kt::sym_eig_host(n, A, w, V);
    return KT_OK;
}

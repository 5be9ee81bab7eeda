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

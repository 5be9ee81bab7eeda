// kt_pairs.hip -- kernels of the batched greedy candidate evaluation
// (krylov_miobi.m:76-99: one block-2 Lanczos run per candidate edge, all
// candidates of a greedy step advanced together).
//
// Layout: a "pair block" is a row-major n x ld device array; candidate c owns
// columns 2c and 2c+1 (16 bytes per row).  The SpMM that advances every
// candidate is the shared k_spmm_block kernel over all 2C columns.  The
// per-candidate work -- CGS2 against the 2-block window
// (lanczos_krylov.m:109-115) and the thin Householder QR (:90) -- is done as
// five row SWEEPS over all candidates at once, with coalesced access: the 64
// lanes of a wave take 64 consecutive candidates (1 KB of one row), the waves
// and workgroups split the rows.  Between sweeps a small kernel reduces the
// per-workgroup partial sums (one wave per candidate, fixed order: results
// are bit-reproducible) and derives that candidate's coefficients.
//
//   sweep A : g1 = [p c]' w                         (CGS pass 1 dots)
//   sweep B : w -= [p c] g1 ;  g2 = [p c]' w         (pass 1 update, pass 2 dots)
//   sweep C : w -= [p c] g2 ;  s1 = |w0(2:n)|^2, ab = w0(2:n)' w1(2:n)
//   coef C  : dlarfg on column 1 (beta1, tau1), H1 applied to column 2
//   sweep D : z = w1 - kappa w0 ;  s2 = |z(3:n)|^2, dz = w0(3:n)' z(3:n)
//   coef D  : dlarfg on z(2:n) (beta2, tau2), R, d = v1' v2
//   sweep E : w <- [q1 q2] = dorg2r(H1, H2)
// Exactly rank-deficient blocks take LAPACK's tau = 0 branch, so their
// completions match MATLAB's qr(w, 0).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "kt_launch.h"

namespace kt {

constexpr int kSweepBlock = 256;
constexpr int kSweepWaves = kSweepBlock / 64;

// per-candidate coefficient record (doubles)
enum : int {
    CF_G1 = 0,      // 8: pass-1 h, column-major 4x2 (rows p0 p1 c0 c1)
    CF_G2 = 8,      // 8: pass-2 h
    CF_SCAL1 = 16,  // 1/(alpha1 - beta1)
    CF_TAU1 = 17,
    CF_KAPPA = 18,  // tau1 * t * scal1: z = w1 - kappa * w0 (rows >= 1)
    CF_SCAL2 = 19,
    CF_TAU2 = 20,
    CF_K2 = 21,     // tau1 * (v1(2) - tau2 * d)
    CF_V11 = 22,    // v1(2)
    CF_BETA1 = 23,
    CF_R12 = 24,
    CF_NCOEF = 25
};

enum { PH_A = 0, PH_B = 1, PH_C = 2, PH_C0 = 3, PH_D = 4, PH_E = 5 };

template <int PH> struct PhaseNV { static constexpr int v = 8; };
template <> struct PhaseNV<PH_C> { static constexpr int v = 2; };
template <> struct PhaseNV<PH_C0> { static constexpr int v = 2; };
template <> struct PhaseNV<PH_D> { static constexpr int v = 2; };
template <> struct PhaseNV<PH_E> { static constexpr int v = 0; };

__device__ __forceinline__ double2 ld2(const double* B, int64_t r, int ld, int64_t off) {
    return *reinterpret_cast<const double2*>(B + r * ld + off);
}

// One sweep over rows [r0, r1) of this workgroup for the 64 candidates of
// group blockIdx.x; partial sums (NV per candidate) to
// part[(k * C + c) * nrb + blockIdx.y].
template <int PH>
__global__ __launch_bounds__(kSweepBlock) void k_pairs_sweep(
    int n, int C, int rows_per_blk, const double* __restrict__ prev,
    const double* __restrict__ cur, double* __restrict__ W, int ld,
    const double* __restrict__ coef, double* __restrict__ part, const int* __restrict__ skip) {
    constexpr int NV = PhaseNV<PH>::v;
    __shared__ double lds[NV > 0 ? NV * kSweepWaves * 64 : 1];
    if (skip && *skip == 0) return;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int c = blockIdx.x * 64 + lane;
    const bool valid = c < C;
    const int cc = valid ? c : C - 1;  // clamp: loads stay in the candidate columns
    const int64_t off = 2 * (int64_t)cc;
    const int r0 = blockIdx.y * rows_per_blk;
    const int r1 = min(n, r0 + rows_per_blk);
    const double* cf = coef + (int64_t)cc * CF_NCOEF;
    double g[8];
    if (PH == PH_B || PH == PH_C) {
        const int base = PH == PH_B ? CF_G1 : CF_G2;
#pragma unroll
        for (int k = 0; k < 8; ++k) g[k] = cf[base + k];
    }
    double acc[NV > 0 ? NV : 1];
#pragma unroll
    for (int k = 0; k < (NV > 0 ? NV : 1); ++k) acc[k] = 0.0;
    const double scal1 = (PH == PH_D || PH == PH_E) ? cf[CF_SCAL1] : 0.0;
    const double kappa = (PH == PH_D || PH == PH_E) ? cf[CF_KAPPA] : 0.0;
    for (int r = r0 + wave; r < r1; r += kSweepWaves) {
        double2 w = ld2(W, r, ld, off);
        if (PH == PH_A || PH == PH_B || PH == PH_C) {
            const double2 u = ld2(cur, r, ld, off);
            const double2 p = prev ? ld2(prev, r, ld, off) : make_double2(0.0, 0.0);
            if (PH != PH_A) {
                w.x -= p.x * g[0] + p.y * g[1] + u.x * g[2] + u.y * g[3];
                w.y -= p.x * g[4] + p.y * g[5] + u.x * g[6] + u.y * g[7];
                if (valid) *reinterpret_cast<double2*>(W + (int64_t)r * ld + off) = w;
            }
            if (PH != PH_C) {
                acc[0] += p.x * w.x; acc[1] += p.y * w.x; acc[2] += u.x * w.x; acc[3] += u.y * w.x;
                acc[4] += p.x * w.y; acc[5] += p.y * w.y; acc[6] += u.x * w.y; acc[7] += u.y * w.y;
            }
        }
        if (PH == PH_C || PH == PH_C0) {
            if (r >= 1) {
                acc[0] += w.x * w.x;
                acc[1] += w.x * w.y;
            }
        }
        if (PH == PH_D) {
            if (r >= 2) {
                const double z = w.y - kappa * w.x;
                acc[0] += z * z;
                acc[1] += w.x * z;
            }
        }
        if (PH == PH_E && valid) {
            const double tau1 = cf[CF_TAU1], tau2 = cf[CF_TAU2], scal2 = cf[CF_SCAL2];
            const double k2 = cf[CF_K2];
            double v1, v2;
            if (r == 0) {
                v1 = 1.0;
                v2 = 0.0;
            } else if (r == 1) {
                v1 = cf[CF_V11];
                v2 = 1.0;
            } else {
                v1 = w.x * scal1;
                v2 = (w.y - kappa * w.x) * scal2;
            }
            double2 q;
            q.x = (r == 0 ? 1.0 : 0.0) - tau1 * v1;
            q.y = (r == 1 ? 1.0 : 0.0) - tau2 * v2 - k2 * v1;
            *reinterpret_cast<double2*>(W + (int64_t)r * ld + off) = q;
        }
    }
    if (NV > 0) {
#pragma unroll
        for (int k = 0; k < NV; ++k) lds[(k * kSweepWaves + wave) * 64 + lane] = acc[k];
        __syncthreads();
        if (wave == 0 && valid) {
            const int nrb = gridDim.y;
#pragma unroll
            for (int k = 0; k < NV; ++k) {
                double s = 0.0;
#pragma unroll
                for (int w = 0; w < kSweepWaves; ++w) s += lds[(k * kSweepWaves + w) * 64 + lane];
                part[((int64_t)k * C + c) * nrb + blockIdx.y] = s;
            }
        }
    }
}

// NV partial sums of candidate c at once (k = k0 .. k0+NV-1): the loads of
// every k are issued together each round, same per-lane order as
// wave_sum_part, so the results are bit-identical
template <int NV>
__device__ __forceinline__ void wave_sum_parts(const double* __restrict__ part, int C, int nrb,
                                               int k0, int c, double* out) {
    const int lane = threadIdx.x & 63;
    double s[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) s[k] = 0.0;
    for (int i = lane; i < nrb; i += 64) {
        double x[NV];
#pragma unroll
        for (int k = 0; k < NV; ++k) x[k] = part[((int64_t)(k0 + k) * C + c) * nrb + i];
#pragma unroll
        for (int k = 0; k < NV; ++k) s[k] += x[k];
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1)
#pragma unroll
        for (int k = 0; k < NV; ++k) s[k] += __shfl_xor(s[k], o, 64);
#pragma unroll
    for (int k = 0; k < NV; ++k) out[k] = s[k];
}

// LAPACK dlarfg on (alpha, ||x||^2 = xx): beta, tau and 1/(alpha - beta)
__device__ __forceinline__ void larfg(double alpha, double xx, double& beta, double& tau,
                                      double& scal) {
    if (xx == 0.0) {  // H = I
        beta = alpha;
        tau = 0.0;
        scal = 1.0;
        return;
    }
    beta = -copysign(hypot(alpha, sqrt(xx)), alpha);
    tau = (beta - alpha) / beta;
    scal = 1.0 / (alpha - beta);
}

// Coefficients after a sweep; one wave per candidate (4 per workgroup).
//   PH_A -> g1;  PH_B -> g2;  PH_C/PH_C0 -> column-1 reflector and kappa;
//   PH_D -> column-2 reflector, d, k2, and the host record hr[c*11 + 0..10]
//          = (h = g1 + g2 [8], R11, R12, R22)
template <int PH>
__global__ __launch_bounds__(256) void k_pairs_coef(int C, int nrb, const double* __restrict__ part,
                                                    const double* __restrict__ W, int ld,
                                                    double* __restrict__ coef,
                                                    double* __restrict__ hr,
                                                    const int* __restrict__ skip) {
    const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (c >= C || (skip && *skip == 0)) return;
    double* cf = coef + (int64_t)c * CF_NCOEF;
    const int64_t off = 2 * (int64_t)c;
    if (PH == PH_A || PH == PH_B) {
        double v[8];
        wave_sum_parts<8>(part, C, nrb, 0, c, v);
        if (lane == 0) {
            const int base = PH == PH_A ? CF_G1 : CF_G2;
#pragma unroll
            for (int k = 0; k < 8; ++k) cf[base + k] = v[k];
        }
    } else if (PH == PH_C || PH == PH_C0) {
        double v2[2];
        wave_sum_parts<2>(part, C, nrb, 0, c, v2);
        const double s1 = v2[0], ab = v2[1];
        if (lane == 0) {
            const double2 w0 = ld2(W, 0, ld, off), w1 = ld2(W, 1, ld, off);
            double beta1, tau1, scal1;
            larfg(w0.x, s1, beta1, tau1, scal1);
            const double t = w0.y + scal1 * ab;  // v1' w(:,2)
            cf[CF_SCAL1] = scal1;
            cf[CF_TAU1] = tau1;
            cf[CF_KAPPA] = tau1 * t * scal1;
            cf[CF_BETA1] = beta1;
            cf[CF_R12] = w0.y - tau1 * t;
            cf[CF_V11] = w1.x * scal1;
            if (PH == PH_C0) {
#pragma unroll
                for (int k = 0; k < 16; ++k) cf[CF_G1 + k] = 0.0;
            }
        }
    } else {  // PH_D
        double v2[2];
        wave_sum_parts<2>(part, C, nrb, 0, c, v2);
        const double s2 = v2[0], dz = v2[1];
        if (lane == 0) {
            const double2 w1 = ld2(W, 1, ld, off);
            const double z1 = w1.y - cf[CF_KAPPA] * w1.x;
            double beta2, tau2, scal2;
            larfg(z1, s2, beta2, tau2, scal2);
            const double v11 = cf[CF_V11];
            const double d = v11 + cf[CF_SCAL1] * scal2 * dz;  // v1' v2
            cf[CF_SCAL2] = scal2;
            cf[CF_TAU2] = tau2;
            cf[CF_K2] = cf[CF_TAU1] * (v11 - tau2 * d);
            double* o = hr + (int64_t)c * 11;
#pragma unroll
            for (int k = 0; k < 8; ++k) o[k] = cf[CF_G1 + k] + cf[CF_G2 + k];
            o[8] = cf[CF_BETA1];
            o[9] = cf[CF_R12];
            o[10] = beta2;
        }
    }
}

// ---------------------------------------------------------------------------
// Per-candidate projected eigenproblems on the device (trace_fun_update.m:
// 71-118 for every candidate of a batch, one thread per candidate): build
// the 2j x 2j block-tridiagonal Gm from the step history, tGm = Gm + Cm,
// symmetrise, eigenvalues by Householder tridiagonalisation + implicit QL
// (the host kt_dense.cpp routine), Xm = sum f(d1) - f(d2), lag-2 stop and
// lucky breakdown.  Done candidates are frozen, so the Lanczos loop can run
// ahead of the host.
// ---------------------------------------------------------------------------
__device__ double dev_fscalar(int fun, double x) {
    switch (fun) {
    case 0: return exp(x);
    case 1: return sinh(x);
    case 2: return cosh(x);
    case 3: return sin(x);
    case 4: return cos(x);
    case 5: return log(x);
    case 6: return sqrt(x);
    }
    return 0.0;
}

// eigenvalues (ascending, in d) of the symmetric n x n column-major `a`
// (destroyed); e: n scratch.  The device copy of kt_dense.cpp's host routine:
// Source: the EISPACK routines TRED2 (Householder tridiagonalisation, with
// the transform accumulated) and IMTQL2 / TQL2 (implicit-shift QL), public
// domain -- Martin, Reinsch & Wilkinson, "Householder's tridiagonalization of a
// symmetric matrix" and Bowdler, Martin, Reinsch & Wilkinson, "The QR and QL
// algorithms for symmetric matrices", Numer. Math. 11 (1968), Handbook for
// Automatic Computation vol. II (Wilkinson & Reinsch 1971), contributions II/2
// and II/3; Smith et al., EISPACK Guide (1976).
__device__ void dev_sym_eigvals(int n, double* a, double* d, double* e) {
    for (int i = n - 1; i > 0; --i) {  // tred2, values only
        const int l = i - 1;
        double h = 0.0, scale = 0.0;
        if (l > 0) {
            for (int k = 0; k <= l; ++k) scale += fabs(a[i + k * n]);
            if (scale == 0.0) {
                e[i] = a[i + l * n];
            } else {
                for (int k = 0; k <= l; ++k) {
                    a[i + k * n] /= scale;
                    h += a[i + k * n] * a[i + k * n];
                }
                double f = a[i + l * n];
                double g = (f >= 0.0 ? -sqrt(h) : sqrt(h));
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
    for (int i = 0; i < n; ++i) d[i] = a[i + i * n];
    // implicit QL, values only (tql2 without vectors)
    for (int i = 1; i < n; ++i) e[i - 1] = e[i];
    e[n - 1] = 0.0;
    const double eps = 2.220446049250313e-16;
    for (int l = 0; l < n; ++l) {
        int iter = 0;
        for (;;) {
            int m = l;
            for (; m < n - 1; ++m) {
                const double dd = fabs(d[m]) + fabs(d[m + 1]);
                if (fabs(e[m]) <= eps * dd) break;
            }
            if (m == l || iter++ == 200) break;
            double g = (d[l + 1] - d[l]) / (2.0 * e[l]);
            double r = hypot(g, 1.0);
            g = d[m] - d[l] + e[l] / (g + copysign(r, g));
            double sn = 1.0, cs = 1.0, p = 0.0;
            bool deflated = false;
            for (int i = m - 1; i >= l; --i) {
                const double f = sn * e[i];
                const double b = cs * e[i];
                r = hypot(f, g);
                e[i + 1] = r;
                if (r == 0.0) {
                    d[i + 1] -= p;
                    e[m] = 0.0;
                    deflated = true;
                    break;
                }
                sn = f / r;
                cs = g / r;
                g = d[i + 1] - p;
                r = (d[i] - g) * sn + 2.0 * cs * b;
                p = sn * r;
                d[i + 1] = g + p;
                g = cs * r - b;
            }
            if (deflated) continue;
            d[l] -= p;
            e[l] = g;
            e[m] = 0.0;
        }
    }
    for (int i = 1; i < n; ++i) {  // insertion sort
        const double v = d[i];
        int k = i - 1;
        while (k >= 0 && d[k] > v) {
            d[k + 1] = d[k];
            --k;
        }
        d[k + 1] = v;
    }
}

// state per candidate (doubles): [0] Xstop(1) [1] Xstop(2) [2] Xm [3] iter
// [4] lucky [5] done
enum : int { PS_X0 = 0, PS_X1 = 1, PS_XM = 2, PS_ITER = 3, PS_LUCKY = 4, PS_DONE = 5, PS_N = 8 };

__global__ void k_pair_eig(int C, int j, int it, int fun, double tol,
                           const double* __restrict__ hist, const double* __restrict__ Cm,
                           double* __restrict__ scratch, int64_t sstride,
                           double* __restrict__ state) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    double* st = state + (int64_t)c * PS_N;
    if (st[PS_DONE] != 0.0) return;
    const int nn = 2 * j;
    double* G = scratch + (int64_t)c * sstride;
    double* T = G + (size_t)nn * nn;
    double* d1 = T + (size_t)nn * nn;
    double* d2 = d1 + nn;
    double* e = d2 + nn;
    for (int t = 0; t < nn * nn; ++t) G[t] = 0.0;
    for (int b = 0; b < j; ++b) {  // lanczos_krylov.m:85-90 block placement
        const double* h = hist + ((int64_t)b * C + c) * 11;
        // D = h(cur) at (2b, 2b);  P = h(prev) at (2b-2, 2b);  R at (2b+2, 2b)
        G[(2 * b) + (2 * b) * nn] = h[2];
        G[(2 * b + 1) + (2 * b) * nn] = h[3];
        G[(2 * b) + (2 * b + 1) * nn] = h[6];
        G[(2 * b + 1) + (2 * b + 1) * nn] = h[7];
        if (b >= 1) {
            G[(2 * b - 2) + (2 * b) * nn] = h[0];
            G[(2 * b - 1) + (2 * b) * nn] = h[1];
            G[(2 * b - 2) + (2 * b + 1) * nn] = h[4];
            G[(2 * b - 1) + (2 * b + 1) * nn] = h[5];
        }
        if (b + 1 < j) {
            G[(2 * b + 2) + (2 * b) * nn] = h[8];
            G[(2 * b + 2) + (2 * b + 1) * nn] = h[9];
            G[(2 * b + 3) + (2 * b + 1) * nn] = h[10];
        }
    }
    for (int t = 0; t < nn * nn; ++t) T[t] = G[t];
    const double* cm = Cm + (int64_t)c * 4;
    T[0] += cm[0];
    T[1] += cm[1];
    T[nn] += cm[2];
    T[nn + 1] += cm[3];
    for (int b = 0; b < nn; ++b)  // (X + X') / 2   trace_fun_update.m:78-81
        for (int a = 0; a < b; ++a) {
            double x = 0.5 * (G[a + b * nn] + G[b + a * nn]);
            G[a + b * nn] = G[b + a * nn] = x;
            x = 0.5 * (T[a + b * nn] + T[b + a * nn]);
            T[a + b * nn] = T[b + a * nn] = x;
        }
    dev_sym_eigvals(nn, T, d1, e);
    dev_sym_eigvals(nn, G, d2, e);
    double xm = 0.0;  // :85-89
    if (fun == 0) {
        for (int i = 0; i < nn; ++i) xm += exp(d1[i]) * (1.0 - exp(d2[i] - d1[i]));
    } else {
        for (int i = 0; i < nn; ++i) xm += dev_fscalar(fun, d1[i]) - dev_fscalar(fun, d2[i]);
    }
    const double* hj = hist + ((int64_t)(j - 1) * C + c) * 11;
    const bool lucky = sqrt(hj[8] * hj[8] + hj[9] * hj[9] + hj[10] * hj[10]) < 1e-8;  // :91-93
    st[PS_XM] = xm;
    st[PS_LUCKY] = lucky ? 1.0 : 0.0;
    bool stop = false;
    if (j <= 2) {  // :104-118, lag d = 2
        st[PS_X0 + j - 1] = xm;
    } else if (fabs(xm - st[PS_X0]) < tol) {
        stop = true;
    } else {
        st[PS_X0] = st[PS_X1];
        st[PS_X1] = xm;
    }
    if (stop || lucky || j == it) {
        st[PS_DONE] = 1.0;
        st[PS_ITER] = j;
    }
}

// ---- one workgroup per candidate (2j <= 56): wave 0 solves the updated
// projection T, wave 1 the plain one G, concurrently; both live in LDS ----
// The xor butterfly v += v[lane ^ o], o = 32, 16, ..., 1, in every lane.
// KT_WAVE_DPP=1 (default) moves the partners without the LDS crossbar
// (__shfl_xor compiles to two ds_bpermute_b32 per double and step, ~400 of
// them in k_pair_reg, each an LDS round trip): o = 32, 16 by gfx950's
// v_permlane32/16_swap (the swap hands every lane its partner half: the sum
// lo + hi is own + partner up to the order of the operands, which fp64
// addition ignores), o = 8 by DPP row_ror:8 (= lane ^ 8 within a row of 16),
// o = 4 by row_ror:4 (lane (i - 4) mod 16 holds the same value as lane i ^ 4
// once the o = 8 step made lanes i and i ^ 8 equal), o = 2, 1 by quad_perm.
// Every lane adds the same pairs as the shuffle form: bit-identical sums.
// Wave-uniform control flow only (every call site: the DPP moves read the
// other lanes' registers).
#ifndef KT_WAVE_DPP
#define KT_WAVE_DPP 1
#endif
template <int CTRL>
__device__ __forceinline__ double mov_dpp_d(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xF, 0xF, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
template <bool B32>
__device__ __forceinline__ double swap_sum_d(double v) {
    const long long b = __double_as_longlong(v);
    const unsigned lo = (unsigned)b, hi = (unsigned)(b >> 32);
    const auto rl = B32 ? __builtin_amdgcn_permlane32_swap(lo, lo, false, false)
                        : __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto rh = B32 ? __builtin_amdgcn_permlane32_swap(hi, hi, false, false)
                        : __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    const double x0 = __longlong_as_double(((long long)rh[0] << 32) | (unsigned int)rl[0]);
    const double x1 = __longlong_as_double(((long long)rh[1] << 32) | (unsigned int)rl[1]);
    return x0 + x1;
}
// min / max over the wave (exact and commutative: any pairing gives the
// shuffle butterfly's value), same moves as wave_sum64
template <bool MAX, bool B32>
__device__ __forceinline__ double swap_mm_d(double v) {
    const long long b = __double_as_longlong(v);
    const unsigned lo = (unsigned)b, hi = (unsigned)(b >> 32);
    const auto rl = B32 ? __builtin_amdgcn_permlane32_swap(lo, lo, false, false)
                        : __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto rh = B32 ? __builtin_amdgcn_permlane32_swap(hi, hi, false, false)
                        : __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    const double x0 = __longlong_as_double(((long long)rh[0] << 32) | (unsigned int)rl[0]);
    const double x1 = __longlong_as_double(((long long)rh[1] << 32) | (unsigned int)rl[1]);
    return MAX ? fmax(x0, x1) : fmin(x0, x1);
}
template <bool MAX>
__device__ __forceinline__ double wave_minmax64(double v) {
#if KT_WAVE_DPP
    v = swap_mm_d<MAX, true>(v);
    v = swap_mm_d<MAX, false>(v);
    v = MAX ? fmax(v, mov_dpp_d<0x128>(v)) : fmin(v, mov_dpp_d<0x128>(v));
    v = MAX ? fmax(v, mov_dpp_d<0x124>(v)) : fmin(v, mov_dpp_d<0x124>(v));
    v = MAX ? fmax(v, mov_dpp_d<0x4E>(v)) : fmin(v, mov_dpp_d<0x4E>(v));
    v = MAX ? fmax(v, mov_dpp_d<0xB1>(v)) : fmin(v, mov_dpp_d<0xB1>(v));
#else
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = MAX ? fmax(v, __shfl_xor(v, o, 64)) : fmin(v, __shfl_xor(v, o, 64));
#endif
    return v;
}
// min over the aligned group of g lanes (g a power of two <= 64, wave-uniform)
__device__ __forceinline__ int group_min_i(int v, int g) {
#if KT_WAVE_DPP
    if (g > 1) v = min(v, __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, false));  // lane ^ 1
    if (g > 2) v = min(v, __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, false));  // lane ^ 2
    if (g > 4) v = min(v, __builtin_amdgcn_update_dpp(0, v, 0x141, 0xF, 0xF, false)); // 7 - i: the other quad
    if (g > 8) v = min(v, __builtin_amdgcn_update_dpp(0, v, 0x140, 0xF, 0xF, false)); // 15 - i: the other 8
    if (g > 16) {
        const auto r = __builtin_amdgcn_permlane16_swap((unsigned)v, (unsigned)v, false, false);
        v = min((int)r[0], (int)r[1]);
    }
    if (g > 32) {
        const auto r = __builtin_amdgcn_permlane32_swap((unsigned)v, (unsigned)v, false, false);
        v = min((int)r[0], (int)r[1]);
    }
#else
    for (int o = 1; o < g; o <<= 1) v = min(v, __shfl_xor(v, o, 64));
#endif
    return v;
}
__device__ __forceinline__ double wave_sum64(double v) {
#if KT_WAVE_DPP
    v = swap_sum_d<true>(v);
    v = swap_sum_d<false>(v);
    v += mov_dpp_d<0x128>(v);  // row_ror:8
    v += mov_dpp_d<0x124>(v);  // row_ror:4
    v += mov_dpp_d<0x4E>(v);   // quad_perm [2,3,0,1]
    v += mov_dpp_d<0xB1>(v);   // quad_perm [1,0,3,2]
#else
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
#endif
    return v;
}

// LDS hand-off between the lanes of ONE wave (the two waves of the block run
// data-dependent control flow, so no workgroup barrier inside the solvers)
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// lane l's double, broadcast to the wave (l uniform): two v_readlane, no LDS
__device__ __forceinline__ double readlane_d(double v, int l) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)b, l);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// Householder tridiagonalisation (dsytd2, lower) of the symmetric n x n LDS
// matrix A (row stride n, n <= 64, destroyed) by one wave: lane i owns
// COLUMN i of the trailing block (symmetry: reading A(k+1+j, k+1+lane) for a
// fixed j is a contiguous, conflict-free LDS row); the reflector v and the
// rank-2 update vector w stay in registers (lane i holds element i) and are
// broadcast with v_readlane.  Returns this lane's (d_lane, e_lane) in the
// references: the diagonal and off-diagonal of the tridiagonal.
__device__ void wave_tridiag(int n, double* A, double& d_out, double& e_out) {
    const int lane = threadIdx.x & 63;
    d_out = 0.0;
    e_out = 0.0;
    for (int k = 0; k + 2 < n; ++k) {  // reflector on A(k+1:n, k) = A(k, k+1:n)'
        const int m = n - k - 1;
        const double xi = (lane < m) ? A[k * n + (k + 1 + lane)] : 0.0;
        const double akk = A[k * n + k];
        const double alpha = readlane_d(xi, 0);
        const double xn2 = wave_sum64(lane >= 1 ? xi * xi : 0.0);
        double tau = 0.0, beta = alpha, scal = 1.0;
        if (xn2 != 0.0) {
            beta = -copysign(sqrt(alpha * alpha + xn2), alpha);
            tau = (beta - alpha) / beta;
            scal = 1.0 / (alpha - beta);
        }
        if (lane == k) {
            d_out = akk;
            e_out = beta;
        }
        const double vi = (lane == 0) ? 1.0 : (lane < m ? xi * scal : 0.0);
        if (tau != 0.0) {
            // p = tau A22 v ; w = p - (tau/2)(p'v) v ; A22 -= v w' + w v'
            double* col = A + (k + 1) * n + (k + 1) + lane;  // A(k+1+j, k+1+lane) = col[j n]
            double p = 0.0;
            if (lane < m) {  // by 4: the LDS loads issue together, fma order unchanged
                int j = 0;
                for (; j + 4 <= m; j += 4) {
                    const double a0 = col[j * n], a1 = col[(j + 1) * n];
                    const double a2 = col[(j + 2) * n], a3 = col[(j + 3) * n];
                    p = fma(a0, readlane_d(vi, j), p);
                    p = fma(a1, readlane_d(vi, j + 1), p);
                    p = fma(a2, readlane_d(vi, j + 2), p);
                    p = fma(a3, readlane_d(vi, j + 3), p);
                }
                for (; j < m; ++j) p = fma(col[j * n], readlane_d(vi, j), p);
            }
            p *= tau;
            const double pv = wave_sum64(lane < m ? p * vi : 0.0);
            const double wi = p - 0.5 * tau * pv * vi;
            if (lane < m) {
                int j = 0;
                for (; j + 4 <= m; j += 4) {
                    double a[4];
#pragma unroll
                    for (int t = 0; t < 4; ++t) a[t] = col[(j + t) * n];
#pragma unroll
                    for (int t = 0; t < 4; ++t)
                        col[(j + t) * n] = a[t] - (readlane_d(vi, j + t) * wi + readlane_d(wi, j + t) * vi);
                }
                for (; j < m; ++j) col[j * n] -= readlane_d(vi, j) * wi + readlane_d(wi, j) * vi;
            }
            wave_sync();
        }
    }
    // last 2 x 2 block
    if (n >= 2 && lane == n - 2) {
        d_out = A[(n - 2) * n + (n - 2)];
        e_out = A[(n - 2) * n + (n - 1)];
    }
    if (lane == n - 1) d_out = A[(n - 1) * n + (n - 1)];
}

// Eigenvalues of the symmetric tridiagonal held in registers (lane i: d_i,
// e_i) by Sturm multisection: g = 64 / n lanes per eigenvalue, each
// counting at kMs interleaved shifts, so one round splits the bracket into
// g*kMs + 1 parts.  Rounds stop once the bracket is 2 ulp of the spectral
// radius wide (the absolute accuracy tql2 / dstebz deliver), or stops
// shrinking.  The Sturm pivots use rcp + one Newton step (only their signs
// count).  The wave solves eigenvalues k0 .. k0+ne-1 (g = 64 / ne lanes
// each); returns lambda_{k0 + lane / g} in lanes with lane % g == 0
// (others: unspecified).
template <int kMs>
__device__ double wave_multisect(int n, double di_reg, double ei_reg, int k0, int ne) {
    const int lane = threadIdx.x & 63;
    const double e2_reg = (lane + 1 < n) ? ei_reg * ei_reg : 0.0;
    double lo = 0.0, hi = 0.0, emax2 = 0.0;
    {  // Gershgorin interval (lane-parallel, then wave min/max)
        const double eprev = __shfl(ei_reg, lane > 0 ? lane - 1 : 0, 64);
        const double ep = (lane >= 1 && lane < n) ? fabs(eprev) : 0.0;
        const double en = (lane + 1 < n) ? fabs(ei_reg) : 0.0;
        double l = (lane < n) ? di_reg - ep - en : INFINITY;
        double h = (lane < n) ? di_reg + ep + en : -INFINITY;
        double m2 = e2_reg;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            l = fmin(l, __shfl_xor(l, o, 64));
            h = fmax(h, __shfl_xor(h, o, 64));
            m2 = fmax(m2, __shfl_xor(m2, o, 64));
        }
        lo = l;
        hi = h;
        emax2 = m2;
    }
    const double span = fmax(hi - lo, 1e-300);
    lo -= 2.2e-16 * span + 1e-300;
    hi += 2.2e-16 * span + 1e-300;
    const double pivmin = fmax(2.2250738585072014e-308 * fmax(1.0, emax2), 1e-300);
    const double atol = 4.4e-16 * fmax(fabs(lo), fabs(hi)) + 1e-300;
    const int g = 64 / ne;  // lanes per eigenvalue; this wave owns k0 .. k0+ne-1
    const int kl = lane / g, sub = lane % g;
    const int k = k0 + kl;
    const int M = g * kMs;  // points per round
    double a = lo, b = hi;
    const bool live = kl < ne;
    bool done = !live;  // identical across a group: it shares (a, b)
    const double d0 = readlane_d(di_reg, 0);
    for (int round = 0; round < 64; ++round) {
        if (!done && !(b - a > atol)) done = true;
        if (__ballot(!done) == 0ull) break;  // wave-uniform exit
        double x[kMs], q[kMs];
        int cnt[kMs];
        const double h = (b - a) / (double)(M + 1);
#pragma unroll
        for (int s = 0; s < kMs; ++s) {
            x[s] = a + h * (double)(sub * kMs + s + 1);
            q[s] = d0 - x[s];
            if (fabs(q[s]) < pivmin) q[s] = -pivmin;
            cnt[s] = q[s] < 0.0;
        }
        for (int i = 1; i < n; ++i) {
            const double di = readlane_d(di_reg, i), ei = readlane_d(e2_reg, i - 1);
#pragma unroll
            for (int s = 0; s < kMs; ++s) {
                double r = __builtin_amdgcn_rcp(q[s]);
                r = fma(fma(-q[s], r, 1.0), r, r);
                q[s] = (di - x[s]) - ei * r;
                if (fabs(q[s]) < pivmin) q[s] = -pivmin;
                cnt[s] += q[s] < 0.0;
            }
        }
        // first point (group-wide index) whose count exceeds k: lambda_k < x_p
        int mine = M;
#pragma unroll
        for (int s = kMs - 1; s >= 0; --s)
            if (cnt[s] > k) mine = sub * kMs + s;
        int first = mine;
        for (int o = 1; o < g; ++o) first = min(first, __shfl(mine, kl * g + (sub + o) % g, 64));
        if (!done) {
            const double na = first == 0 ? a : a + h * (double)first;
            const double nb = first == M ? b : fmin(b, a + h * (double)(first + 1));
            if (!(na > a || nb < b)) {
                done = true;  // bracket at machine resolution
            } else {
                a = na;
                b = nb;
            }
        }
    }
    return 0.5 * (a + b);
}

// W waves per projection (block 128 W): wave 0 of each tridiagonalises, then
// all W multisect disjoint eigenvalue ranges with MS counts per lane.
template <int W, int MS>
__global__ __launch_bounds__(128 * W) void k_pair_eig_wave(int C, int j, int it, int fun, double tol,
                                                       const double* __restrict__ hist,
                                                       const double* __restrict__ Cm,
                                                       double* __restrict__ state) {
    extern __shared__ double sm[];
    const int c = blockIdx.x;
    const int tid = threadIdx.x;
    constexpr int NT = 128 * W;
    const int wave = tid >> 6, lane = tid & 63;
    double* st = state + (int64_t)c * PS_N;
    if (st[PS_DONE] != 0.0) return;
    const int nn = 2 * j;
    double* G = sm;
    double* T = G + nn * nn;
    double* de = T + nn * nn;  // per projection: d (nn), e (nn)
    double* vec = de + 4 * nn;  // eigenvalues: eig(T) (nn), then eig(G) (nn)
    for (int t = tid; t < nn * nn; t += NT) G[t] = 0.0;
    __syncthreads();
    for (int b = tid; b < j; b += NT) {  // row-major G[r * nn + col]
        const double* h = hist + ((int64_t)b * C + c) * 11;
        G[(2 * b) * nn + 2 * b] = h[2];
        G[(2 * b + 1) * nn + 2 * b] = h[3];
        G[(2 * b) * nn + 2 * b + 1] = h[6];
        G[(2 * b + 1) * nn + 2 * b + 1] = h[7];
        if (b >= 1) {
            G[(2 * b - 2) * nn + 2 * b] = h[0];
            G[(2 * b - 1) * nn + 2 * b] = h[1];
            G[(2 * b - 2) * nn + 2 * b + 1] = h[4];
            G[(2 * b - 1) * nn + 2 * b + 1] = h[5];
        }
        if (b + 1 < j) {
            G[(2 * b + 2) * nn + 2 * b] = h[8];
            G[(2 * b + 2) * nn + 2 * b + 1] = h[9];
            G[(2 * b + 3) * nn + 2 * b + 1] = h[10];
        }
    }
    __syncthreads();
    for (int t = tid; t < nn * nn; t += NT) T[t] = G[t];
    __syncthreads();
    if (tid == 0) {
        const double* cm = Cm + (int64_t)c * 4;  // column-major 2x2
        T[0] += cm[0];
        T[nn] += cm[1];
        T[1] += cm[2];
        T[nn + 1] += cm[3];
    }
    __syncthreads();
    for (int t = tid; t < nn * nn; t += NT) {  // (X + X') / 2   :78-81
        const int r = t / nn, q = t % nn;
        if (q < r) {
            const double g = 0.5 * (G[r * nn + q] + G[q * nn + r]);
            const double x = 0.5 * (T[r * nn + q] + T[q * nn + r]);
            G[r * nn + q] = G[q * nn + r] = g;
            T[r * nn + q] = T[q * nn + r] = x;
        }
    }
    __syncthreads();
    const int mat = wave / W, wv = wave % W;  // mat 0: T (updated), 1: G
    if (wv == 0) {
        double dl, el;
        wave_tridiag(nn, mat == 0 ? T : G, dl, el);
        if (lane < nn) {
            de[mat * 2 * nn + lane] = dl;
            de[mat * 2 * nn + nn + lane] = el;
        }
    }
    __syncthreads();
    {
        const double dreg = lane < nn ? de[mat * 2 * nn + lane] : 0.0;
        const double ereg = lane < nn ? de[mat * 2 * nn + nn + lane] : 0.0;
        const int per = (nn + W - 1) / W;
        const int k0 = wv * per;
        const int ne = min(per, nn - k0);
        if (ne > 0) {  // wave-uniform
            const double lam = wave_multisect<MS>(nn, dreg, ereg, k0, ne);
            const int g = 64 / ne;
            if (lane % g == 0 && lane / g < ne) vec[mat * nn + k0 + lane / g] = lam;
        }
    }
    __syncthreads();
    if (wave != 0) return;
    const double* l1 = vec;       // wave 0: eig(T), ascending
    const double* l2 = vec + nn;  // wave 1: eig(G)
    double term = 0.0;  // :85-89 (k-th smallest of each)
    if (lane < nn)
        term = (fun == 0) ? exp(l1[lane]) * (1.0 - exp(l2[lane] - l1[lane]))
                          : dev_fscalar(fun, l1[lane]) - dev_fscalar(fun, l2[lane]);
    const double xm = wave_sum64(term);
    if (lane == 0) {
        const double* hj = hist + ((int64_t)(j - 1) * C + c) * 11;
        const bool lucky = sqrt(hj[8] * hj[8] + hj[9] * hj[9] + hj[10] * hj[10]) < 1e-8;
        st[PS_XM] = xm;
        st[PS_LUCKY] = lucky ? 1.0 : 0.0;
        bool stop = false;
        if (j <= 2) {
            st[PS_X0 + j - 1] = xm;
        } else if (fabs(xm - st[PS_X0]) < tol) {
            stop = true;
        } else {
            st[PS_X0] = st[PS_X1];
            st[PS_X1] = xm;
        }
        if (stop || lucky || j == it) {
            st[PS_DONE] = 1.0;
            st[PS_ITER] = j;
        }
    }
}

// ---------------------------------------------------------------------------
// Fused candidate runs (default for small n): ONE workgroup per candidate runs
// its whole trace_fun_update (krylov_miobi.m:99 -> trace_fun_update.m:53-125)
// in one launch -- the qr(U) start, then per Lanczos step the SpMM
// (lanczos_krylov.m:81), the five CGS2 / Householder sweeps of
// launch_pairs_orth (:109-115, :90) with workgroup reductions in a fixed
// order, the step's record, both projected eigenproblems in LDS (wave
// Householder + Sturm multisection, as k_pair_eig_wave) and the lag-2 stop.
// No grid-wide hand-off per step: the batched path needed ~10 dependent
// launches per step over all candidates.  The candidate's vectors live in
// its own slice of `vec` ([C][3][n][2], L2-resident for small n).
// ---------------------------------------------------------------------------
#ifndef KT_FUSED_THREADS
#define KT_FUSED_THREADS 512
#endif
constexpr int kFusedThreads = KT_FUSED_THREADS;
constexpr int kFusedWaves = kFusedThreads / 64;
constexpr int kFusedMaxNN = 56;  // 2j at which the eigenproblems leave LDS

// KT_FUSED_PROF builds (diagnostic, tools/fused_phases.sh): thread 0 of
// candidate 0 accumulates the 100 MHz wall clock per phase of the fused run
// and prints the totals at its end.  Slots: 0 start, 1 SpMM, 2-6 sweeps A-E,
// 7 eigenvalues, 8 stop test; slot 15 holds the last timestamp.
#ifdef KT_FUSED_PROF
__shared__ unsigned long long g_fprof[16];  // LDS: the marks add no global-memory stalls
#define FPROF(k)                                                          \
    do {                                                                  \
        if (blockIdx.x == 0 && threadIdx.x == 0) {                        \
            const unsigned long long t_ = wall_clock64();                 \
            g_fprof[k] += t_ - g_fprof[15];                               \
            g_fprof[15] = t_;                                             \
        }                                                                 \
    } while (0)
#else
#define FPROF(k) \
    do {         \
    } while (0)
#endif

// fixed-order workgroup sum of NV per-thread values; every thread gets them
template <int NV>
__device__ __forceinline__ void block_sum(double (&acc)[NV], double* red /* [kFusedWaves][NV] */) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < NV; ++k) acc[k] = wave_sum64(acc[k]);
    if (lane == 0)
#pragma unroll
        for (int k = 0; k < NV; ++k) red[wave * NV + k] = acc[k];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        double s = 0.0;
#pragma unroll
        for (int w = 0; w < kFusedWaves; ++w) s += red[w * NV + k];
        acc[k] = s;
    }
    __syncthreads();  // red is reused by the next reduction
}

struct FusedCSR {
    const int* rp;
    const int* ci;
    const double* va;
    const int* long_rows;
    int n_long, long_thresh, unit;
};

// W = A V (n x 2): short rows one thread each, long rows one wave each
__device__ void fused_spmm(int n, const FusedCSR& M, const double* __restrict__ V, double* __restrict__ W) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int r = tid; r < n; r += kFusedThreads) {
        const int b = M.rp[r], e = M.rp[r + 1];
        if (e - b > M.long_thresh) continue;
        double s0 = 0.0, s1 = 0.0;
        for (int k0 = b; k0 < e; k0 += 4) {  // 4 gathers in flight, added in order
            int c[4];
            double a[4];
            double2 v[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const bool ok = k0 + q < e;
                c[q] = ok ? M.ci[k0 + q] : 0;
                a[q] = ok ? (M.unit ? 1.0 : M.va[k0 + q]) : 0.0;
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] = *reinterpret_cast<const double2*>(V + 2 * (int64_t)c[q]);
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (k0 + q < e) {
                    s0 = fma(a[q], v[q].x, s0);
                    s1 = fma(a[q], v[q].y, s1);
                }
        }
        *reinterpret_cast<double2*>(W + 2 * (int64_t)r) = make_double2(s0, s1);
    }
    for (int li = wave; li < M.n_long; li += kFusedWaves) {
        const int r = M.long_rows[li];
        const int b = M.rp[r], e = M.rp[r + 1];
        double s0 = 0.0, s1 = 0.0;
        for (int k = b + lane; k < e; k += 64) {
            const int c = M.ci[k];
            const double a = M.unit ? 1.0 : M.va[k];
            const double2 v = *reinterpret_cast<const double2*>(V + 2 * (int64_t)c);
            s0 = fma(a, v.x, s0);
            s1 = fma(a, v.y, s1);
        }
        s0 = wave_sum64(s0);
        s1 = wave_sum64(s1);
        if (lane == 0) *reinterpret_cast<double2*>(W + 2 * (int64_t)r) = make_double2(s0, s1);
    }
}

// The CGS2 + thin Householder QR of W against the window [P C]
// (launch_pairs_orth's sweeps A-E on one candidate).  P == nullptr: the
// first step (window of one block, p = 0); C == nullptr: qr(U) of the start
// (sweep C0, no projection).  W is overwritten by Q; rec[0..10] = (g1 + g2
// [8], beta1, R12, beta2).  Ends with a workgroup barrier.
__device__ void fused_orth(int n, const double* __restrict__ P, const double* __restrict__ Cv,
                           double* __restrict__ W, double* cf, double* red, double* rec) {
    const int tid = threadIdx.x;
    if (Cv) {
        for (int ph = 0; ph < 2; ++ph) {  // sweep A (dots) then B (update + dots)
            double acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
            double g[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) g[k] = ph ? cf[CF_G1 + k] : 0.0;
            constexpr int U = 4;  // rows per round: their loads issue together (row order kept)
            for (int r0 = tid; r0 < n; r0 += U * kFusedThreads) {
                double2 w[U], u[U], p[U];
#pragma unroll
                for (int q = 0; q < U; ++q) {
                    const int r = r0 + q * kFusedThreads;
                    const bool ok = r < n;
                    w[q] = ok ? *reinterpret_cast<const double2*>(W + 2 * (int64_t)r) : make_double2(0.0, 0.0);
                    u[q] = ok ? *reinterpret_cast<const double2*>(Cv + 2 * (int64_t)r) : make_double2(0.0, 0.0);
                    p[q] = (ok && P) ? *reinterpret_cast<const double2*>(P + 2 * (int64_t)r) : make_double2(0.0, 0.0);
                }
#pragma unroll
                for (int q = 0; q < U; ++q) {
                    const int r = r0 + q * kFusedThreads;
                    if (ph) {
                        w[q].x -= p[q].x * g[0] + p[q].y * g[1] + u[q].x * g[2] + u[q].y * g[3];
                        w[q].y -= p[q].x * g[4] + p[q].y * g[5] + u[q].x * g[6] + u[q].y * g[7];
                        if (r < n) *reinterpret_cast<double2*>(W + 2 * (int64_t)r) = w[q];
                    }
                    acc[0] += p[q].x * w[q].x; acc[1] += p[q].y * w[q].x; acc[2] += u[q].x * w[q].x; acc[3] += u[q].y * w[q].x;
                    acc[4] += p[q].x * w[q].y; acc[5] += p[q].y * w[q].y; acc[6] += u[q].x * w[q].y; acc[7] += u[q].y * w[q].y;
                }
            }
            block_sum<8>(acc, red);
            if (tid == 0)
#pragma unroll
                for (int k = 0; k < 8; ++k) cf[(ph ? CF_G2 : CF_G1) + k] = acc[k];
            __syncthreads();
            FPROF(2 + ph);
        }
    } else if (tid == 0) {
#pragma unroll
        for (int k = 0; k < 16; ++k) cf[CF_G1 + k] = 0.0;
    }
    {  // sweep C (C0 without the projection): s1 = |w0(2:n)|^2, ab = w0(2:n)' w1(2:n)
        double acc[2] = {0.0, 0.0};
        double g[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) g[k] = Cv ? cf[CF_G2 + k] : 0.0;
        constexpr int U = 4;
        for (int r0 = tid; r0 < n; r0 += U * kFusedThreads) {
            double2 w[U], u[U], p[U];
#pragma unroll
            for (int q = 0; q < U; ++q) {
                const int r = r0 + q * kFusedThreads;
                const bool ok = r < n;
                w[q] = ok ? *reinterpret_cast<const double2*>(W + 2 * (int64_t)r) : make_double2(0.0, 0.0);
                u[q] = (ok && Cv) ? *reinterpret_cast<const double2*>(Cv + 2 * (int64_t)r) : make_double2(0.0, 0.0);
                p[q] = (ok && Cv && P) ? *reinterpret_cast<const double2*>(P + 2 * (int64_t)r) : make_double2(0.0, 0.0);
            }
#pragma unroll
            for (int q = 0; q < U; ++q) {
                const int r = r0 + q * kFusedThreads;
                if (Cv) {
                    w[q].x -= p[q].x * g[0] + p[q].y * g[1] + u[q].x * g[2] + u[q].y * g[3];
                    w[q].y -= p[q].x * g[4] + p[q].y * g[5] + u[q].x * g[6] + u[q].y * g[7];
                    if (r < n) *reinterpret_cast<double2*>(W + 2 * (int64_t)r) = w[q];
                }
                if (r >= 1 && r < n) {
                    acc[0] += w[q].x * w[q].x;
                    acc[1] += w[q].x * w[q].y;
                }
            }
        }
        block_sum<2>(acc, red);  // its barrier also publishes W's updated rows 0, 1
        if (tid == 0) {
            const double2 w0 = *reinterpret_cast<const double2*>(W), w1 = *reinterpret_cast<const double2*>(W + 2);
            double beta1, tau1, scal1;
            larfg(w0.x, acc[0], beta1, tau1, scal1);
            const double t = w0.y + scal1 * acc[1];  // v1' w(:,2)
            cf[CF_SCAL1] = scal1;
            cf[CF_TAU1] = tau1;
            cf[CF_KAPPA] = tau1 * t * scal1;
            cf[CF_BETA1] = beta1;
            cf[CF_R12] = w0.y - tau1 * t;
            cf[CF_V11] = w1.x * scal1;
        }
        __syncthreads();
        FPROF(4);
    }
    {  // sweep D: z = w1 - kappa w0;  s2 = |z(3:n)|^2, dz = w0(3:n)' z(3:n)
        double acc[2] = {0.0, 0.0};
        const double kappa = cf[CF_KAPPA];
        for (int r = tid; r < n; r += kFusedThreads) {
            if (r < 2) continue;
            const double2 w = *reinterpret_cast<const double2*>(W + 2 * (int64_t)r);
            const double z = w.y - kappa * w.x;
            acc[0] += z * z;
            acc[1] += w.x * z;
        }
        block_sum<2>(acc, red);
        if (tid == 0) {
            const double2 w1 = *reinterpret_cast<const double2*>(W + 2);
            const double z1 = w1.y - cf[CF_KAPPA] * w1.x;
            double beta2, tau2, scal2;
            larfg(z1, acc[0], beta2, tau2, scal2);
            const double v11 = cf[CF_V11];
            const double d = v11 + cf[CF_SCAL1] * scal2 * acc[1];  // v1' v2
            cf[CF_SCAL2] = scal2;
            cf[CF_TAU2] = tau2;
            cf[CF_K2] = cf[CF_TAU1] * (v11 - tau2 * d);
#pragma unroll
            for (int k = 0; k < 8; ++k) rec[k] = cf[CF_G1 + k] + cf[CF_G2 + k];
            rec[8] = cf[CF_BETA1];
            rec[9] = cf[CF_R12];
            rec[10] = beta2;
        }
        __syncthreads();
        FPROF(5);
    }
    {  // sweep E: W <- [q1 q2] = dorg2r(H1, H2)
        const double tau1 = cf[CF_TAU1], tau2 = cf[CF_TAU2], scal1 = cf[CF_SCAL1], scal2 = cf[CF_SCAL2];
        const double k2 = cf[CF_K2], kappa = cf[CF_KAPPA], v11 = cf[CF_V11];
        for (int r = tid; r < n; r += kFusedThreads) {
            const double2 w = *reinterpret_cast<const double2*>(W + 2 * (int64_t)r);
            double v1, v2;
            if (r == 0) {
                v1 = 1.0;
                v2 = 0.0;
            } else if (r == 1) {
                v1 = v11;
                v2 = 1.0;
            } else {
                v1 = w.x * scal1;
                v2 = (w.y - kappa * w.x) * scal2;
            }
            double2 q;
            q.x = (r == 0 ? 1.0 : 0.0) - tau1 * v1;
            q.y = (r == 1 ? 1.0 : 0.0) - tau2 * v2 - k2 * v1;
            *reinterpret_cast<double2*>(W + 2 * (int64_t)r) = q;
        }
        __syncthreads();
        FPROF(6);
    }
}

// Both projections of step j (trace_fun_update.m:71-89) from the records in
// LDS; returns Xm to every thread.  nn = 2j <= kFusedMaxNN: in LDS, wave 0-3
// on the updated projection T, waves 4-7 on G (wave 0 / 4 tridiagonalise,
// then 4 waves multisect each); larger nn: one thread per projection on the
// global scratch `big` (dev_sym_eigvals).
__device__ double fused_xm(int j, int fun, const double* rec /* [j][11] LDS */, const double* cm,
                           double* sm, double* big) {
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int nn = 2 * j;
    const bool lds = nn <= kFusedMaxNN;
    double* G = lds ? sm : big;
    double* T = G + nn * nn;
    double* de = T + nn * nn;   // per projection: d (nn), e (nn)
    double* ev = de + 4 * nn;   // eigenvalues: eig(T) (nn), eig(G) (nn)
    for (int t = tid; t < nn * nn; t += kFusedThreads) G[t] = 0.0;
    __syncthreads();
    for (int b = tid; b < j; b += kFusedThreads) {  // row-major G[r * nn + col]
        const double* h = rec + 11 * b;
        G[(2 * b) * nn + 2 * b] = h[2];
        G[(2 * b + 1) * nn + 2 * b] = h[3];
        G[(2 * b) * nn + 2 * b + 1] = h[6];
        G[(2 * b + 1) * nn + 2 * b + 1] = h[7];
        if (b >= 1) {
            G[(2 * b - 2) * nn + 2 * b] = h[0];
            G[(2 * b - 1) * nn + 2 * b] = h[1];
            G[(2 * b - 2) * nn + 2 * b + 1] = h[4];
            G[(2 * b - 1) * nn + 2 * b + 1] = h[5];
        }
        if (b + 1 < j) {
            G[(2 * b + 2) * nn + 2 * b] = h[8];
            G[(2 * b + 2) * nn + 2 * b + 1] = h[9];
            G[(2 * b + 3) * nn + 2 * b + 1] = h[10];
        }
    }
    __syncthreads();
    for (int t = tid; t < nn * nn; t += kFusedThreads) T[t] = G[t];
    __syncthreads();
    if (tid == 0) {  // Cm column-major 2x2
        T[0] += cm[0];
        T[nn] += cm[1];
        T[1] += cm[2];
        T[nn + 1] += cm[3];
    }
    __syncthreads();
    for (int t = tid; t < nn * nn; t += kFusedThreads) {  // (X + X') / 2   :78-81
        const int r = t / nn, q = t % nn;
        if (q < r) {
            const double g = 0.5 * (G[r * nn + q] + G[q * nn + r]);
            const double x = 0.5 * (T[r * nn + q] + T[q * nn + r]);
            G[r * nn + q] = G[q * nn + r] = g;
            T[r * nn + q] = T[q * nn + r] = x;
        }
    }
    __syncthreads();
    if (lds) {
        constexpr int W = kFusedWaves / 2;
        const int mat = wave / W, wv = wave % W;  // mat 0: T, 1: G
        if (wv == 0) {
            double dl, el;
            wave_tridiag(nn, mat == 0 ? T : G, dl, el);
            if (lane < nn) {
                de[mat * 2 * nn + lane] = dl;
                de[mat * 2 * nn + nn + lane] = el;
            }
        }
        __syncthreads();
        const double dreg = lane < nn ? de[mat * 2 * nn + lane] : 0.0;
        const double ereg = lane < nn ? de[mat * 2 * nn + nn + lane] : 0.0;
        const int per = (nn + W - 1) / W;
        const int k0 = wv * per;
        const int ne = min(per, nn - k0);
        if (ne > 0) {  // wave-uniform
            const double lam = wave_multisect<4>(nn, dreg, ereg, k0, ne);
            const int g = 64 / ne;
            if (lane % g == 0 && lane / g < ne) ev[mat * nn + k0 + lane / g] = lam;
        }
    } else if (lane == 0 && wave < 2) {  // row-major storage is its own transpose (symmetric)
        dev_sym_eigvals(nn, wave == 0 ? T : G, ev + wave * nn, de + wave * 2 * nn);
    }
    __syncthreads();
    double term = 0.0;  // :85-89 (k-th smallest of each)
    if (wave == 0)
        for (int i = lane; i < nn; i += 64)
            term += (fun == 0) ? exp(ev[i]) * (1.0 - exp(ev[nn + i] - ev[i]))
                               : dev_fscalar(fun, ev[i]) - dev_fscalar(fun, ev[nn + i]);
    term = wave_sum64(term);
    __shared__ double s_xm;
    if (tid == 0) s_xm = term;
    __syncthreads();
    const double xm = s_xm;
    __syncthreads();
    return xm;
}

// ---- eigenvalues of the symmetrised block-tridiagonal projection by block
// Sturm counts.  Gm (trace_fun_update.m:71-81) is block tridiagonal with 2x2
// blocks: diagonal blocks M_k (symmetric) and couplings U_k = M(blk k, blk
// k+1).  For a shift x the block LDL' of M - xI,
//   D_0 = M_0 - xI,   D_{k+1} = M_{k+1} - xI - U_k' D_k^{-1} U_k,
// has the inertia of M - xI (Sylvester), so #eig(M) < x = sum over k of the
// negative eigenvalues of the 2x2 D_k: an O(j) count, no tridiagonalisation.
// A near-singular D_k is evaluated at x + eps (see block_count_ms).  Checked
// on the CPU against eigvalsh on every India candidate's projections
// (tools/blk_sturm_check.py): eigenvalues within 4e-15 of the spectral radius.  The blocks are the exact (X + X')/2 entries the dense path
// forms, so both solve the same matrix.
struct Blk2 {
    double a, b, c;        // M_k = [a b; b c]
    double u0, u1, u2, u3;  // U_k = [u0 u1; u2 u3] (row-major), k < j-1
};

// MS shifts at once: MS independent LDL' chains share each block's loads
// (latency hiding); 1/det by rcp + one Newton step (full precision)
// HAS_M0: (a, b, c) of the first diagonal block come from m0 instead of B[0]
// (a compile-time switch, so the callers without an override keep their code)
template <int MS, bool HAS_M0 = false>
__device__ __forceinline__ void block_count_ms(int j, const Blk2* __restrict__ B, const double (&x)[MS],
                                               double pivmin, double eps, int (&cnt)[MS],
                                               const double* m0 = nullptr) {
    double a[MS], b[MS], c[MS];
    Blk2 cur = B[0];
    {
        const double ma = HAS_M0 ? m0[0] : cur.a, mb = HAS_M0 ? m0[1] : cur.b, mc = HAS_M0 ? m0[2] : cur.c;
#pragma unroll
        for (int s = 0; s < MS; ++s) {
            a[s] = ma - x[s];
            b[s] = mb;
            c[s] = mc - x[s];
            cnt[s] = 0;
        }
    }
    for (int k = 0;; ++k) {
        // the next block's load issued ahead of this block's dependent chain
        // (after the loop's exit test it would wait a whole LDS round trip)
        const Blk2 nx = B[min(k + 1, j - 1)];
        double det[MS];
#pragma unroll
        for (int s = 0; s < MS; ++s) {
            det[s] = fma(a[s], c[s], -b[s] * b[s]);
            if (fabs(det[s]) < pivmin) {
                // near-singular D_k: evaluate this block at x + eps -- the 2x2
                // analogue of dstebz's q = -pivmin.  Perturbing det alone fails
                // for D_k = 0 (zero adjugate: e.g. a zero leading block with the
                // shift at exactly 0).  eps^2 = 100 pivmin keeps det above
                // pivmin; |U|^2 / eps stays below 1e153 (no overflow next block).
                a[s] -= eps;
                c[s] -= eps;
                det[s] = fma(a[s], c[s], -b[s] * b[s]);
                if (fabs(det[s]) < pivmin) det[s] = -pivmin;
            }
            cnt[s] += det[s] < 0.0 ? 1 : (a[s] < 0.0 ? 2 : 0);
        }
        if (k + 1 >= j) break;
        const Blk2& q = cur;  // U_k
#pragma unroll
        for (int s = 0; s < MS; ++s) {
            double r = __builtin_amdgcn_rcp(det[s]);
            r = fma(fma(-det[s], r, 1.0), r, r);
            const double i00 = c[s] * r, i01 = -b[s] * r, i11 = a[s] * r;
            // t = D^{-1} U, S = U' t
            const double t00 = i00 * q.u0 + i01 * q.u2, t01 = i00 * q.u1 + i01 * q.u3;
            const double t10 = i01 * q.u0 + i11 * q.u2, t11 = i01 * q.u1 + i11 * q.u3;
            const double s00 = q.u0 * t00 + q.u2 * t10;
            const double s01 = q.u0 * t01 + q.u2 * t11;
            const double s11 = q.u1 * t01 + q.u3 * t11;
            a[s] = nx.a - x[s] - s00;
            b[s] = nx.b - s01;
            c[s] = nx.c - x[s] - s11;
        }
        cur = nx;
    }
}

// One shift with the derivative, for Newton on det(M - xI): cnt = #eig < x
// (as block_count_ms) and S = d/dx log|det(M - xI)| = sum_k tr(D_k^{-1} D_k'),
// with D_0' = -I, D_{k+1}' = -I + T_k' D_k' T_k, T_k = D_k^{-1} U_k.  The
// Newton step on the characteristic polynomial is x - 1/S.
template <bool HAS_M0 = false>
__device__ __forceinline__ void block_count_newton(int j, const Blk2* __restrict__ B, double x,
                                                   double pivmin, double eps, int& cnt, double& S,
                                                   const double* m0 = nullptr) {
    Blk2 cur = B[0];
    double a = (HAS_M0 ? m0[0] : cur.a) - x, b = HAS_M0 ? m0[1] : cur.b, c = (HAS_M0 ? m0[2] : cur.c) - x;
    double p = -1.0, q = 0.0, r = -1.0;  // D_k'
    cnt = 0;
    S = 0.0;
    for (int k = 0;; ++k) {
        const Blk2 nx = B[min(k + 1, j - 1)];  // ahead of the chain (block_count_ms)
        double det = fma(a, c, -b * b);
        if (fabs(det) < pivmin) {  // as block_count_ms
            a -= eps;
            c -= eps;
            det = fma(a, c, -b * b);
            if (fabs(det) < pivmin) det = -pivmin;
        }
        cnt += det < 0.0 ? 1 : (a < 0.0 ? 2 : 0);
        double rr = __builtin_amdgcn_rcp(det);
        rr = fma(fma(-det, rr, 1.0), rr, rr);
        const double i00 = c * rr, i01 = -b * rr, i11 = a * rr;
        S = fma(i00, p, fma(2.0 * i01, q, fma(i11, r, S)));
        if (k + 1 >= j) break;
        const Blk2& u = cur;
        const double t00 = i00 * u.u0 + i01 * u.u2, t01 = i00 * u.u1 + i01 * u.u3;
        const double t10 = i01 * u.u0 + i11 * u.u2, t11 = i01 * u.u1 + i11 * u.u3;
        const double s00 = u.u0 * t00 + u.u2 * t10;
        const double s01 = u.u0 * t01 + u.u2 * t11;
        const double s11 = u.u1 * t01 + u.u3 * t11;
        const double e00 = p * t00 + q * t10, e01 = p * t01 + q * t11;
        const double e10 = q * t00 + r * t10, e11 = q * t01 + r * t11;
        p = -1.0 + t00 * e00 + t10 * e10;
        q = t00 * e01 + t10 * e11;
        r = -1.0 + t01 * e01 + t11 * e11;
        a = nx.a - x - s00;
        b = nx.b - s01;
        c = nx.c - x - s11;
        cur = nx;
    }
}

// lanes per eigenvalue when one wave solves ne of them: a power of two, so a
// group's lanes are an aligned xor-butterfly range
__device__ __forceinline__ int group_lanes(int ne) {
    int g = 64;
    while (g > 1 && g * ne > 64) g >>= 1;
    return g;
}

#ifndef KT_BLK_NEWTON
#define KT_BLK_NEWTON 1
#endif
// Newton's last step is taken and the run ends once the step is below
// KT_BLK_NEWTON_ACCEPT atol (2^20 atol ~ 5e-10 of the spectral radius: the
// step's quadratic error is far below atol), then certified by the counts
// at x -+ 8 atol as before -- a lane that fails goes on bisecting.  One
// Newton count fewer per eigenvalue than at 64 atol: config 5 -1 %
// (profiles/r02_greedy_newton_accept.txt)
#ifndef KT_BLK_NEWTON_ACCEPT
#define KT_BLK_NEWTON_ACCEPT 1048576
#endif
// shifts per lane per multisection round.  The eigenvalue phase is bound by
// FP64 issue (a wave64 FMA takes 4 cycles; 2 waves per SIMD), not latency, so
// fewer shifts with more rounds does less work: 1 beats 4 by 4 % end to end
// on config 5 (profiles/r02_greedy_blk_ms.txt)
#ifndef KT_BLK_MS
#define KT_BLK_MS 1
#endif
// Waves per projection for the per-step eigenvalues (both the fused and the
// register kernel, so they solve identically): KT_XM_WAVES_SMALL while each
// wave still holds <= 16 eigenvalues (g >= 4 lanes each: the Newton path),
// else half the workgroup.  Fewer waves issue fewer FP64 operations in total;
// the others wait at the barrier (2 waves: config 5 -2-3 %,
// profiles/r02_greedy_xm_waves.txt)
#ifndef KT_XM_WAVES_SMALL
#define KT_XM_WAVES_SMALL 2
#endif
__device__ __forceinline__ int xm_waves(int nn) {
    constexpr int half = kFusedWaves / 2;
    constexpr int small = KT_XM_WAVES_SMALL < half ? KT_XM_WAVES_SMALL : half;
    return nn <= 16 * small ? small : half;
}

// Eigenvalues k0 .. k0+ne-1 (ascending) of the block matrix by one wave:
// g = group_lanes(ne) lanes per eigenvalue.  Multisection (MS interleaved
// shifts per lane, g*MS + 1 parts per round) brackets each eigenvalue; once
// every bracket is span/4096 wide a safeguarded Newton iteration
// on det(M - xI) (block_count_newton; a step leaving the count bracket is a
// bisection) converges in ~4 steps, and is accepted once its step is below
// KT_BLK_NEWTON_ACCEPT atol AND the counts at x -+ 8 atol bracket lambda_k (certified to
// 8 atol = 3.5e-15 of the spectral radius).  Lanes whose Newton run is not
// certified (~1 % on the greedy projections, tests/test_block_sturm.py)
// continue the multisection to 2 ulp of the spectral radius (as before:
// KT_BLK_NEWTON=0 builds that alone).  Returns lambda_{k0 + lane / g} in
// every lane of group lane / g < ne.
// m0 (optional): (a, b, c) of the first diagonal block in place of B[0]'s --
// the updated projection T differs from G only there (T = G + Cm)
template <int MS, bool HAS_M0 = false>
__device__ __forceinline__ double wave_multisect_blk(int j, const Blk2* B, int k0, int ne, const double* m0 = nullptr) {
    const int lane = threadIdx.x & 63;
    const int nn = 2 * j;
    double lo = INFINITY, hi = -INFINITY, smax = 0.0;
    for (int r = lane; r < nn; r += 64) {  // Gershgorin over the rows
        const int k = r >> 1, s = r & 1;
        const Blk2& m = B[k];
        const double d = (HAS_M0 && k == 0) ? m0[s ? 2 : 0] : (s ? m.c : m.a);
        double off = fabs((HAS_M0 && k == 0) ? m0[1] : m.b);
        if (k + 1 < j) off += s ? fabs(m.u2) + fabs(m.u3) : fabs(m.u0) + fabs(m.u1);  // U_k row s
        if (k >= 1) {  // U_{k-1}' row s = column s of U_{k-1}
            const Blk2& p = B[k - 1];
            off += s ? fabs(p.u1) + fabs(p.u3) : fabs(p.u0) + fabs(p.u2);
        }
        lo = fmin(lo, d - off);
        hi = fmax(hi, d + off);
        smax = fmax(smax, fmax(fabs(d), off));
    }
    lo = wave_minmax64<false>(lo);
    hi = wave_minmax64<true>(hi);
    smax = wave_minmax64<true>(smax);
    const double span = fmax(hi - lo, 1e-300);
    lo -= 2.2e-16 * span + 1e-300;
    hi += 2.2e-16 * span + 1e-300;
    const double sc = fmax(1.0, smax);
    const double pivmin = 2.2250738585072014e-308 * sc * sc * sc * sc;
    const double eps = 10.0 * sqrt(pivmin);
    const double atol = 4.4e-16 * fmax(fabs(lo), fabs(hi)) + 1e-300;
    const int g = group_lanes(ne);
    const int kl = lane / g, sub = lane % g;
    const int k = k0 + kl;
    const int M = g * MS;
    double a = lo, b = hi;
    const bool live = kl < ne;
    bool done = !live;
    auto ms_round = [&]() {
        const double h = (b - a) / (double)(M + 1);
        int mine = M;
        if (!done) {
            double xs[MS];
            int cnt[MS];
#pragma unroll
            for (int s2 = 0; s2 < MS; ++s2) xs[s2] = a + h * (double)(sub * MS + s2 + 1);
            block_count_ms<MS, HAS_M0>(j, B, xs, pivmin, eps, cnt, m0);
#pragma unroll
            for (int s2 = MS - 1; s2 >= 0; --s2)
                if (cnt[s2] > k) mine = sub * MS + s2;
        }
        const int first = group_min_i(mine, g);  // group minimum
        if (!done) {
            const double na = first == 0 ? a : a + h * (double)first;
            const double nb = first == M ? b : fmin(b, a + h * (double)(first + 1));
            if (!(na > a || nb < b)) {
                done = true;
            } else {
                a = na;
                b = nb;
            }
        }
    };
    int round = 0;
#if KT_BLK_NEWTON
    // Newton pays where a wave holds <= 16 eigenvalues (g >= 4): with more, one
    // uncertified lane in the wave sends all of them back to the multisection
    // (measured: 2j = 80 at 4 waves per projection is 10 % slower with it)
    if (g >= 4) {
    // multisection until every bracket is within span / 4096 (ceil(12 /
    // log2(g MS + 1)) rounds: 3 at g = 16, MS = 1), where Newton converges in
    // ~4 steps
    const double narrow = (hi - lo) * (1.0 / 4096.0);
    for (; round < 64; ++round) {
        if (!done && !(b - a > atol)) done = true;
        if (__ballot(!done && b - a > narrow) == 0ull) break;
        ms_round();
    }
    bool newton = !done, conv = false;
    double x = 0.5 * (a + b);
    for (int it = 0; it < 8; ++it) {
        if (__ballot(newton && !conv) == 0ull) break;
        if (newton && !conv) {
            int cnt;
            double S;
            block_count_newton<HAS_M0>(j, B, x, pivmin, eps, cnt, S, m0);
            if (cnt > k) b = x;
            else a = x;
            const double xn = x - 1.0 / S;  // S = 0 or inf: xn is not finite / = x
            const bool inb = xn >= a && xn <= b;
            if (fabs(xn - x) <= (double)KT_BLK_NEWTON_ACCEPT * atol || !(b - a > atol)) {
                conv = true;
                if (inb) x = xn;
            } else {
                x = inb ? xn : 0.5 * (a + b);
            }
        }
    }
    if (__ballot(newton && conv) != 0ull) {  // certify: #eig < x - 8 atol <= k < #eig < x + 8 atol
        int cnt[2] = {0, 0};
        if (newton && conv) {
            const double xs[2] = {x - 8.0 * atol, x + 8.0 * atol};
            block_count_ms<2, HAS_M0>(j, B, xs, pivmin, eps, cnt, m0);
            if (cnt[0] <= k && cnt[1] > k) {
                done = true;
                a = b = x;
            } else {  // keep the tighter count bracket for the multisection
                if (cnt[0] <= k) a = fmax(a, xs[0]);
                if (cnt[1] > k) b = fmin(b, xs[1]);
            }
        }
    }
    }
#endif
    for (; round < 64; ++round) {
        if (!done && !(b - a > atol)) done = true;
        if (__ballot(!done) == 0ull) break;
        ms_round();
    }
    return 0.5 * (a + b);
}

// Xm of step j from the records by block Sturm multisection (any j: the
// blocks take 7 doubles each).  Waves 0..W-1 solve the updated projection
// T, waves W..2W-1 the plain one G.
__device__ double fused_xm_blk(int j, int fun, const double* rec /* [j][11] */, const double* cm,
                               Blk2* blk /* [2][j] LDS */, double* ev /* [2][2j] LDS */) {
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int nn = 2 * j;
    for (int t = tid; t < 2 * j; t += kFusedThreads) {
        const int mat = t / j, k = t % j;  // mat 0: T = G + Cm, 1: G
        const double* h = rec + 11 * k;
        Blk2 m;
        double d00 = h[2], d10 = h[3], d01 = h[6], d11 = h[7];
        if (mat == 0 && k == 0) {  // T(0:1, 0:1) += Cm (column-major)
            d00 += cm[0];
            d10 += cm[1];
            d01 += cm[2];
            d11 += cm[3];
        }
        m.a = d00;
        m.b = 0.5 * (d10 + d01);  // (X + X')/2, lower + upper as the dense path adds them
        m.c = d11;
        if (k + 1 < j) {  // coupling to block k+1: lower block from record k, upper from record k+1
            const double* h1 = rec + 11 * (k + 1);
            m.u0 = 0.5 * (h[8] + h1[0]);
            m.u1 = 0.5 * (0.0 + h1[4]);
            m.u2 = 0.5 * (h[9] + h1[1]);
            m.u3 = 0.5 * (h[10] + h1[5]);
        } else {
            m.u0 = m.u1 = m.u2 = m.u3 = 0.0;
        }
        blk[mat * j + k] = m;
    }
    __syncthreads();
    const int W = xm_waves(nn);  // waves per projection; the rest wait at the barrier
    const int mat = wave / W, wv = wave % W;
    const int per = (nn + W - 1) / W;
    const int k0 = wv * per;
    const int ne = mat < 2 ? min(per, nn - k0) : 0;
    for (int e0 = 0; e0 < ne; e0 += 64) {  // more than 64 eigenvalues per wave: 64 at a time
        const int cnt = min(64, ne - e0);
        const double lam = wave_multisect_blk<KT_BLK_MS>(j, blk + mat * j, k0 + e0, cnt);
        const int g = group_lanes(cnt);
        if (lane % g == 0 && lane / g < cnt) ev[mat * nn + k0 + e0 + lane / g] = lam;
    }
    __syncthreads();
    double term = 0.0;  // :85-89 (k-th smallest of each)
    if (wave == 0)
        for (int i = lane; i < nn; i += 64)
            term += (fun == 0) ? exp(ev[i]) * (1.0 - exp(ev[nn + i] - ev[i]))
                               : dev_fscalar(fun, ev[i]) - dev_fscalar(fun, ev[nn + i]);
    term = wave_sum64(term);
    __shared__ double s_xm2;
    if (tid == 0) s_xm2 = term;
    __syncthreads();
    const double xm = s_xm2;
    __syncthreads();
    return xm;
}

__global__ __launch_bounds__(kFusedThreads) void k_pair_fused(
    int C, int n, FusedCSR M, const int* __restrict__ ii, const int* __restrict__ jj, double b00,
    double b10, double b01, double b11, int it, int fun, double tol, double* __restrict__ vec,
    double* __restrict__ big, int64_t big_stride, double* __restrict__ state, int blk_eig) {
    extern __shared__ double sm[];  // eig workspace (2 nn^2 + 6 nn) | records [it][11]
    __shared__ double red[kFusedWaves * 8];  // block_sum scratch
    __shared__ double cf[CF_NCOEF];
    __shared__ double rec0[11];
    __shared__ double cm[4];
    const int c = blockIdx.x, tid = threadIdx.x;
    const int64_t vn = 2 * (int64_t)n;
    double* V[3] = {vec + 3 * vn * c, vec + 3 * vn * c + vn, vec + 3 * vn * c + 2 * vn};
    double* eigsm = sm;
    const size_t eigw = blk_eig ? (size_t)18 * it
                                : (size_t)2 * kFusedMaxNN * kFusedMaxNN + 6 * kFusedMaxNN;
    double* rec = sm + eigw;  // [it][11]
#ifdef KT_FUSED_PROF
    if (c == 0 && tid == 0) {
        for (int k = 0; k < 15; ++k) g_fprof[k] = 0;
        g_fprof[15] = wall_clock64();
    }
#endif
    // [V, ~] = qr(U, 0), U = [e_i e_j]   (lanczos_krylov.m:48; krylov_miobi.m:82-84)
    for (int64_t t = tid; t < vn; t += kFusedThreads) V[0][t] = 0.0;
    __syncthreads();
    if (tid == 0) {
        V[0][2 * (int64_t)ii[c]] = 1.0;
        V[0][2 * (int64_t)jj[c] + 1] = 1.0;
    }
    __syncthreads();
    fused_orth(n, nullptr, nullptr, V[0], cf, red, rec0);
    if (tid == 0) {  // Cm = R B R'  (trace_fun_update.m:65-66; V1' U = R for unit selectors)
        const double R00 = rec0[8], R01 = rec0[9], R11 = rec0[10];  // R = [R00 R01; 0 R11]
        const double RB00 = R00 * b00 + R01 * b10, RB01 = R00 * b01 + R01 * b11;
        const double RB10 = R11 * b10, RB11 = R11 * b11;
        cm[0] = RB00 * R00 + RB01 * R01;  // column-major (0,0)
        cm[1] = RB10 * R00 + RB11 * R01;  // (1,0)
        cm[2] = RB01 * R11;               // (0,1)
        cm[3] = RB11 * R11;               // (1,1)
    }
    __syncthreads();
#ifdef KT_FUSED_PROF
    if (c == 0 && tid == 0) {  // the start's sweeps count as slot 0
        for (int k = 1; k < 15; ++k) g_fprof[0] += g_fprof[k], g_fprof[k] = 0;
    }
#endif
    FPROF(0);
    int prev = -1, cur = 0, w = 1;
    double x0 = 0.0, x1 = 0.0, xm = 0.0;
    int iter = it, lucky = 0;
    double* mybig = big ? big + big_stride * c : nullptr;
    for (int j = 1; j <= it; ++j) {
        fused_spmm(n, M, V[cur], V[w]);  // w = A * w   (lanczos_krylov.m:81)
        __syncthreads();
        FPROF(1);
        fused_orth(n, prev >= 0 ? V[prev] : nullptr, V[cur], V[w], cf, red, rec + 11 * (j - 1));
        if (!blk_eig && 2 * j > kFusedMaxNN && !mybig) {  // no global scratch: cannot continue (host checks)
            iter = -j;
            break;
        }
#ifdef KT_FUSED_NOEIG  // diagnostic build: vector work only (never stops early)
        xm = (double)j;
        (void)eigsm;
#else
        if (blk_eig)
            xm = fused_xm_blk(j, fun, rec, cm, reinterpret_cast<Blk2*>(eigsm), eigsm + 14 * (size_t)it);
        else
            xm = fused_xm(j, fun, rec, cm, eigsm, mybig);
#endif
        FPROF(7);
        const double* hj = rec + 11 * (j - 1);
        lucky = sqrt(hj[8] * hj[8] + hj[9] * hj[9] + hj[10] * hj[10]) < 1e-8;  // :91-93
        bool stop = false;
        if (j <= 2) {  // :104-118, lag d = 2
            if (j == 1) x0 = xm;
            else x1 = xm;
        } else if (fabs(xm - x0) < tol) {
            stop = true;
        } else {
            x0 = x1;
            x1 = xm;
        }
        if (stop || lucky || j == it) {
            iter = j;
            break;
        }
        const int freed = prev >= 0 ? prev : 3 - cur - w;
        prev = cur;
        cur = w;
        w = freed;
        FPROF(8);
    }
#ifdef KT_FUSED_PROF
    if (c == 0 && tid == 0)
        printf("fused_prof n=%d it=%d iter=%d start=%llu spmm=%llu A=%llu B=%llu C=%llu D=%llu E=%llu eig=%llu stop=%llu (x10ns)\n",
               n, it, iter, g_fprof[0], g_fprof[1], g_fprof[2], g_fprof[3], g_fprof[4], g_fprof[5], g_fprof[6],
               g_fprof[7], g_fprof[8]);
#endif
    if (tid == 0) {
        double* st = state + (int64_t)c * PS_N;
        st[PS_XM] = xm;
        st[PS_ITER] = iter;
        st[PS_LUCKY] = lucky ? 1.0 : 0.0;
        st[PS_DONE] = 1.0;
    }
}

// dynamic LDS: the eigen workspace (dense: 2 nn^2 + 6 nn at nn <= 56; block
// Sturm: 2 j Blk2 + 4 j eigenvalues) followed by the records [it][11]
// Batched path's per-step eigenproblems by block Sturm counts (any 2j; one
// workgroup per candidate): the records of candidate c come from hist
// [step][C][11]; same Xm, lag-2 stop and lucky test as k_pair_eig_wave.
__global__ __launch_bounds__(kFusedThreads) void k_pair_eig_blk(int C, int j, int it, int fun, double tol,
                                                               const double* __restrict__ hist,
                                                               const double* __restrict__ Cm,
                                                               double* __restrict__ state) {
    extern __shared__ double sm[];  // records [j][11] | blocks [2][j] Blk2 | eigenvalues [2][2j]
    const int c = blockIdx.x, tid = threadIdx.x;
    double* st = state + (int64_t)c * PS_N;
    if (st[PS_DONE] != 0.0) return;  // uniform over the workgroup
    double* rec = sm;
    Blk2* blk = reinterpret_cast<Blk2*>(sm + 11 * (size_t)j);
    double* ev = sm + 11 * (size_t)j + 14 * (size_t)j;
    __shared__ double cm[4];
    for (int t = tid; t < 11 * j; t += kFusedThreads) rec[t] = hist[((int64_t)(t / 11) * C + c) * 11 + t % 11];
    if (tid < 4) cm[tid] = Cm[(int64_t)c * 4 + tid];
    __syncthreads();
    const double xm = fused_xm_blk(j, fun, rec, cm, blk, ev);
    if (tid == 0) {
        const double* hj = rec + 11 * (j - 1);
        const bool lucky = sqrt(hj[8] * hj[8] + hj[9] * hj[9] + hj[10] * hj[10]) < 1e-8;
        st[PS_XM] = xm;
        st[PS_LUCKY] = lucky ? 1.0 : 0.0;
        bool stop = false;
        if (j <= 2) {
            st[PS_X0 + j - 1] = xm;
        } else if (fabs(xm - st[PS_X0]) < tol) {
            stop = true;
        } else {
            st[PS_X0] = st[PS_X1];
            st[PS_X1] = xm;
        }
        if (stop || lucky || j == it) {
            st[PS_DONE] = 1.0;
            st[PS_ITER] = j;
        }
    }
}

size_t pair_fused_lds_bytes(int it) {
    const size_t dense = (size_t)2 * kFusedMaxNN * kFusedMaxNN + 6 * kFusedMaxNN;
    const size_t blk = (size_t)14 * it + 4 * (size_t)it;
    return sizeof(double) * (std::max(dense, blk) + 11 * (size_t)it);
}

// ---------------------------------------------------------------------------
// Register-resident candidate runs (n <= 8 * kFusedThreads): the same
// trace_fun_update as k_pair_fused, but thread t OWNS rows t + q T (q < R,
// T = kFusedThreads) of the candidate's three blocks -- the window P, C and
// the new block W -- in registers for the whole run.  Only the gathered block
// (C, for the next SpMM) and the CSR live in LDS.  So no sweep touches global
// memory: the CGS2 / Householder sweeps are register arithmetic between
// workgroup reductions, and the SpMM gathers from LDS.  Every sum is formed in
// k_pair_fused's order (a thread's rows in q order, waves in id order; long
// rows lane-strided + wave_sum64); the two kernels agree to rounding (the
// compiler contracts a few products into FMAs differently).
// ---------------------------------------------------------------------------
// kRegLongCap (kt_launch.h): long rows handled by whole waves

// fixed-order workgroup sum, one barrier: `red` alternates between two halves
// (a wave cannot run two reductions ahead of a slower one: each has a barrier)
template <int NV>
__device__ __forceinline__ void block_sum1(double (&acc)[NV], double* red /* [2][kFusedWaves][8] */, int& par) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    double* rb = red + par * kFusedWaves * 8;
    par ^= 1;
#pragma unroll
    for (int k = 0; k < NV; ++k) acc[k] = wave_sum64(acc[k]);
    if (lane == 0)
#pragma unroll
        for (int k = 0; k < NV; ++k) rb[wave * 8 + k] = acc[k];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        double s = 0.0;
#pragma unroll
        for (int w = 0; w < kFusedWaves; ++w) s += rb[w * 8 + k];
        acc[k] = s;
    }
}

struct RegRec {  // the step's QR quantities, identical in every thread
    double g[16];  // g1 (8), g2 (8)
    double beta1, r12, beta2;
};

// CGS2 against the window [P C] (has_win) + thin Householder QR of the owned
// rows of W; W <- Q, also written over the LDS gather block X (C's rows are
// held in registers, read from X before the SpMM).  (fused_orth's sweeps A-E, same arithmetic
// and order.)
template <int R>
__device__ __forceinline__ void reg_orth(int n, bool has_p, bool has_win, const double2 (&P)[R],
                                         const double2 (&Cv)[R], double2 (&W)[R], double* X, double* red,
                                         double* bc, int& par, RegRec& o) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int k = 0; k < 16; ++k) o.g[k] = 0.0;
    if (has_win) {
#pragma unroll
        for (int ph = 0; ph < 2; ++ph) {  // sweep A (dots), B (update + dots)
            double acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
            for (int q = 0; q < R; ++q) {
                const int r = tid + q * kFusedThreads;
                const double2 p = has_p ? P[q] : make_double2(0.0, 0.0);
                const double2 u = Cv[q];
                double2 w = W[q];
                if (ph) {
                    const double* g = o.g;
                    w.x -= p.x * g[0] + p.y * g[1] + u.x * g[2] + u.y * g[3];
                    w.y -= p.x * g[4] + p.y * g[5] + u.x * g[6] + u.y * g[7];
                    if (r < n) W[q] = w;
                }
                if (r < n) {
                    acc[0] += p.x * w.x; acc[1] += p.y * w.x; acc[2] += u.x * w.x; acc[3] += u.y * w.x;
                    acc[4] += p.x * w.y; acc[5] += p.y * w.y; acc[6] += u.x * w.y; acc[7] += u.y * w.y;
                }
            }
            block_sum1<8>(acc, red, par);
#pragma unroll
            for (int k = 0; k < 8; ++k) o.g[8 * ph + k] = acc[k];
            FPROF(2 + ph);
        }
    }
    // sweep C: w -= [p c] g2;  s1 = |w0(2:n)|^2, ab = w0(2:n)' w1(2:n); rows 0, 1 broadcast
    double acc2[2] = {0.0, 0.0};
#pragma unroll
    for (int q = 0; q < R; ++q) {
        const int r = tid + q * kFusedThreads;
        double2 w = W[q];
        if (has_win) {
            const double2 p = has_p ? P[q] : make_double2(0.0, 0.0);
            const double2 u = Cv[q];
            const double* g = o.g + 8;
            w.x -= p.x * g[0] + p.y * g[1] + u.x * g[2] + u.y * g[3];
            w.y -= p.x * g[4] + p.y * g[5] + u.x * g[6] + u.y * g[7];
            if (r < n) W[q] = w;
        }
        if (r >= 1 && r < n) {
            acc2[0] += w.x * w.x;
            acc2[1] += w.x * w.y;
        }
    }
    if (tid < 2) {  // rows 0 and 1 are owned by threads 0 and 1 (q = 0)
        bc[2 * tid] = W[0].x;
        bc[2 * tid + 1] = W[0].y;
    }
    block_sum1<2>(acc2, red, par);
    const double w0x = bc[0], w0y = bc[1], w1x = bc[2], w1y = bc[3];
    double beta1, tau1, scal1;
    larfg(w0x, acc2[0], beta1, tau1, scal1);
    const double t = w0y + scal1 * acc2[1];  // v1' w(:,2)
    const double kappa = tau1 * t * scal1;
    const double r12 = w0y - tau1 * t;
    const double v11 = w1x * scal1;
    FPROF(4);
    // sweep D: z = w1 - kappa w0;  s2 = |z(3:n)|^2, dz = w0(3:n)' z(3:n)
    double acc3[2] = {0.0, 0.0};
#pragma unroll
    for (int q = 0; q < R; ++q) {
        const int r = tid + q * kFusedThreads;
        if (r >= 2 && r < n) {
            const double z = W[q].y - kappa * W[q].x;
            acc3[0] += z * z;
            acc3[1] += W[q].x * z;
        }
    }
    block_sum1<2>(acc3, red, par);
    const double z1 = w1y - kappa * w1x;
    double beta2, tau2, scal2;
    larfg(z1, acc3[0], beta2, tau2, scal2);
    const double d = v11 + scal1 * scal2 * acc3[1];  // v1' v2
    const double k2 = tau1 * (v11 - tau2 * d);
    o.beta1 = beta1;
    o.r12 = r12;
    o.beta2 = beta2;
    FPROF(5);
    // sweep E: W <- [q1 q2] = dorg2r(H1, H2), into the gather block
#pragma unroll
    for (int q = 0; q < R; ++q) {
        const int r = tid + q * kFusedThreads;
        if (r < n) {
            const double2 w = W[q];
            double v1, v2;
            if (r == 0) {
                v1 = 1.0;
                v2 = 0.0;
            } else if (r == 1) {
                v1 = v11;
                v2 = 1.0;
            } else {
                v1 = w.x * scal1;
                v2 = (w.y - kappa * w.x) * scal2;
            }
            double2 qq;
            qq.x = (r == 0 ? 1.0 : 0.0) - tau1 * v1;
            qq.y = (r == 1 ? 1.0 : 0.0) - tau2 * v2 - k2 * v1;
            *reinterpret_cast<double2*>(X + 2 * r) = qq;
        }
    }
}

// The register kernel's LDS (bytes, in this order; doubles first):
//   X [n+1][2] (gather block C; row n = 0, the SpMM's unused slots) | G blocks [it] Blk2
//   | ev [2][2 it] | (has_long) wl [kRegLongCap][2] | (csr >= 2) val [nnz]
//   | (has_long) slot [n] int | (csr >= 1) rp [n+1] int, ci [nnz] u16
//   (spec: ws [n][2], the next step's row sums formed during the eigenvalues)
struct RegLds {
    size_t x, ws, gblk, ev, wl, va, slot, rp, ci, total;
};
__host__ __device__ inline RegLds reg_lds_layout(int n, int64_t nnz, int it, bool has_long, int csr,
                                                 bool spec = false) {
    RegLds L;
    size_t o = 0;
    L.x = o;
    o += sizeof(double) * 2 * ((size_t)n + 1);
    L.ws = o;
    if (spec) o += sizeof(double) * 2 * (size_t)n;
    L.gblk = o;
    o += sizeof(Blk2) * (size_t)it;
    L.ev = o;
    o += sizeof(double) * 4 * (size_t)it;
    L.wl = o;
    if (has_long) o += sizeof(double) * 2 * kRegLongCap;
    L.va = o;
    if (csr >= 2) o += sizeof(double) * (size_t)nnz;
    L.slot = o;
    if (has_long) o += sizeof(int) * (size_t)n;
    L.rp = o;
    if (csr >= 1) o += sizeof(int) * ((size_t)n + 1);
    L.ci = o;
    if (csr >= 1) o += sizeof(unsigned short) * (size_t)nnz;
    L.total = o;
    return L;
}

// Xm of step j from the persistent G blocks (T = G but for T's first
// diagonal block t0): fused_xm_blk's arithmetic without rebuilding the
// blocks every step.  Waves 0..W-1 solve T, W..2W-1 G.
// Inlined into k_pair_reg (KT_REG_XM_INLINE=0 builds it as a called function:
// each call then saves callee-saved registers to scratch)
#ifndef KT_REG_XM_INLINE
#define KT_REG_XM_INLINE 1
#endif
// help(): called by every wave once its share of the eigenvalues is done,
// before the phase's first barrier (k_pair_reg: the next step's row sums)
struct NoHelp {
    __device__ void operator()() const {}
};
template <class Help = NoHelp>
#if KT_REG_XM_INLINE
__device__ __forceinline__
#else
__device__ __noinline__
#endif
double reg_xm_blk(int j, int fun, const Blk2* gblk, const double* t0, double* ev, const Help& help = Help()) {
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int nn = 2 * j;
    const int W = xm_waves(nn);  // waves per projection; the rest wait at the barrier
    const int mat = wave / W, wv = wave % W;
    const int per = (nn + W - 1) / W;
    const int k0 = wv * per;
    const int ne = mat < 2 ? min(per, nn - k0) : 0;
    for (int e0 = 0; e0 < ne; e0 += 64) {
        const int cnt = min(64, ne - e0);
        const double lam = mat == 0 ? wave_multisect_blk<KT_BLK_MS, true>(j, gblk, k0 + e0, cnt, t0)
                                    : wave_multisect_blk<KT_BLK_MS, false>(j, gblk, k0 + e0, cnt);
        const int g = group_lanes(cnt);
        if (lane % g == 0 && lane / g < cnt) ev[mat * nn + k0 + e0 + lane / g] = lam;
    }
    help();
    __syncthreads();
    double term = 0.0;  // trace_fun_update.m:85-89 (k-th smallest of each)
    if (wave == 0)
        for (int i = lane; i < nn; i += 64)
            term += (fun == 0) ? exp(ev[i]) * (1.0 - exp(ev[nn + i] - ev[i]))
                               : dev_fscalar(fun, ev[i]) - dev_fscalar(fun, ev[nn + i]);
    term = wave_sum64(term);
    __shared__ double s_xm3;
    if (tid == 0) s_xm3 = term;
    __syncthreads();
    const double xm = s_xm3;
    __syncthreads();
    return xm;
}

// KT_REG_SPEC=0: no row sums formed ahead during the eigenvalues (round 5)
#ifndef KT_REG_SPEC
#define KT_REG_SPEC 1
#endif

// KT_REG_SPEC_DYN=0: only waves 4-7 form the rows ahead (static stride)
#ifndef KT_REG_SPEC_DYN
#define KT_REG_SPEC_DYN 1
#endif

// KT_REG_ZROW=0: unused chunk slots repeat the row's last column (round 5)
#ifndef KT_REG_ZROW
#define KT_REG_ZROW 1
#endif

// One gathered row (2 doubles) of the LDS block X; the KT_REG_DIAG=1
// diagnostic build replaces it by a register value (no gather; its results
// are wrong by construction, only its clocks mean anything)
__device__ __forceinline__ double2 reg_gather(const double* X, int c) {
#if defined(KT_REG_DIAG) && KT_REG_DIAG >= 1
    return make_double2((double)c, 1.0);
#else
    return *reinterpret_cast<const double2*>(X + 2 * c);
#endif
}

// CSR: 0 = CSR in global memory, 1 = row pointers + u16 columns in LDS, 2 = and
// the weights.  A template argument, so every CSR access has a known address
// space (a pointer chosen at run time between LDS and global memory compiles
// to flat loads).
template <int R, int CSR>
__global__ __launch_bounds__(kFusedThreads) void k_pair_reg(int C, int n, int nnz_host, FusedCSR M,
                                                            const int* __restrict__ ii, const int* __restrict__ jj,
                                                            double b00, double b10, double b01, double b11,
                                                            int it, int fun, double tol,
                                                            double* __restrict__ state,
                                                            const int* __restrict__ dyn = nullptr,
                                                            int spec = 0) {
    extern __shared__ double sm[];
    __shared__ double red[2 * kFusedWaves * 8];
    __shared__ double bc[4];
    __shared__ double t0[3];     // T's first diagonal block (a, b, c): G's + Cm
    __shared__ double cm[4];     // Cm = R B R' (column-major)
    __shared__ double lastr[3];  // the previous record's R (beta1, r12, beta2)
    __shared__ int s_spec_next;  // the next block of 64 rows to sum ahead (spec)
    const int c = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // dyn (device-resident greedy loop): {nnz, n_long} of the current CSR,
    // written by the previous step's k_greedy_edit; the LDS was sized for the
    // first step's (larger) matrix
    const int nnz = dyn ? dyn[0] : nnz_host;
    const int nl = min(dyn ? dyn[1] : M.n_long, kRegLongCap);
    const RegLds L = reg_lds_layout(n, nnz, it, nl > 0, CSR, spec != 0);
    char* base = reinterpret_cast<char*>(sm);
    double* X = reinterpret_cast<double*>(base + L.x);
    Blk2* gblk = reinterpret_cast<Blk2*>(base + L.gblk);
    double* ev = reinterpret_cast<double*>(base + L.ev);
    double* wl = reinterpret_cast<double*>(base + L.wl);
    int* slot = reinterpret_cast<int*>(base + L.slot);
    int* lrp = reinterpret_cast<int*>(base + L.rp);
    unsigned short* lci = reinterpret_cast<unsigned short*>(base + L.ci);
    double* lva = reinterpret_cast<double*>(base + L.va);
    double* ws = reinterpret_cast<double*>(base + L.ws);
    if (tid == 0) X[2 * n] = X[2 * n + 1] = 0.0;  // the zero row (SpMM's unused chunk slots)
    // the CSR (shared by every candidate, L2-resident) copied once into LDS
    if (CSR >= 1) {
        for (int t = tid; t <= n; t += kFusedThreads) lrp[t] = M.rp[t];
        for (int t = tid; t < nnz; t += kFusedThreads) lci[t] = (unsigned short)M.ci[t];
    }
    if (CSR >= 2)
        for (int t = tid; t < nnz; t += kFusedThreads) lva[t] = M.va[t];
    const int* rp = CSR >= 1 ? lrp : M.rp;
    const double* va = CSR >= 2 ? lva : M.va;
    auto col = [&](int k) -> int { return CSR >= 1 ? (int)lci[k] : M.ci[k]; };
#ifdef KT_FUSED_PROF
    const unsigned long long clk0 = clock64(), wclk0 = wall_clock64();
    if (c == 0 && tid == 0) {
        for (int k = 0; k < 15; ++k) g_fprof[k] = 0;
        g_fprof[15] = wall_clock64();
    }
#endif
    // long rows handled by waves: slot[r] = position in the wave list, -1 for
    // rows their owner sums
    if (nl > 0) {
        for (int t = tid; t < n; t += kFusedThreads) slot[t] = -1;
        __syncthreads();
        for (int li = tid; li < nl; li += kFusedThreads) slot[M.long_rows[li]] = li;
    }
    __syncthreads();
    double2 P[R], Cv[R], W[R];
    // [V, ~] = qr(U, 0), U = [e_i e_j]   (lanczos_krylov.m:48; krylov_miobi.m:82-84)
    const int ri = ii[c], rj = jj[c];
#pragma unroll
    for (int q = 0; q < R; ++q) {
        const int r = tid + q * kFusedThreads;
        P[q] = Cv[q] = make_double2(0.0, 0.0);
        W[q] = make_double2(r == ri ? 1.0 : 0.0, r == rj ? 1.0 : 0.0);
    }
    int par = 0;
    RegRec o;
    reg_orth<R>(n, false, false, P, Cv, W, X, red, bc, par, o);
    if (tid == 0) {  // Cm = R B R'  (trace_fun_update.m:65-66; V1' U = R for unit selectors)
        const double R00 = o.beta1, R01 = o.r12, R11 = o.beta2;
        const double RB00 = R00 * b00 + R01 * b10, RB01 = R00 * b01 + R01 * b11;
        const double RB10 = R11 * b10, RB11 = R11 * b11;
        cm[0] = RB00 * R00 + RB01 * R01;
        cm[1] = RB10 * R00 + RB11 * R01;
        cm[2] = RB01 * R11;
        cm[3] = RB11 * R11;
    }
    __syncthreads();  // X = V_1
#ifdef KT_FUSED_PROF
    if (c == 0 && tid == 0)
        for (int k = 1; k < 15; ++k) g_fprof[0] += g_fprof[k], g_fprof[k] = 0;
#endif
    FPROF(0);
    double x0 = 0.0, x1 = 0.0, xm = 0.0;
    int iter = it, lucky = 0;
    // one row's sum of W = A C, in CSR order (the owners' loop below, for the
    // rows waves 4-7 sum ahead into ws)
    auto row_sum = [&](int r, double& s0, double& s1) {
        const int rb = rp[r], re = rp[r + 1];
        if (M.unit) {
            for (int k0 = rb; k0 < re; k0 += 4) {
                int cc[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int c0 = col(min(k0 + u, re - 1));
                    cc[u] = (KT_REG_ZROW && k0 + u >= re) ? n : c0;
                }
                double2 v[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) v[u] = reg_gather(X, cc[u]);
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const double a = (k0 + u < re) ? 1.0 : 0.0;
                    s0 = fma(a, v[u].x, s0);
                    s1 = fma(a, v[u].y, s1);
                }
            }
        } else {
            for (int k0 = rb; k0 < re; k0 += 4) {
                int cc[4];
                double a[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int k = min(k0 + u, re - 1);
                    const int c0 = col(k);
                    cc[u] = (KT_REG_ZROW && k0 + u >= re) ? n : c0;
                    a[u] = va[k];
                }
                double2 v[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) v[u] = reg_gather(X, cc[u]);
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const double w = (k0 + u < re) ? a[u] : 0.0;
                    s0 = fma(w, v[u].x, s0);
                    s1 = fma(w, v[u].y, s1);
                }
            }
        }
    };
    bool have_spec = false;  // this step's W = A C already in ws / wl (formed by waves 4-7)
    for (int j = 1; j <= it; ++j) {
        if (have_spec) {
            // the sums waves 4-7 formed during the previous step's eigenvalues
#pragma unroll
            for (int q = 0; q < R; ++q) {
                const int r = tid + q * kFusedThreads;
                Cv[q] = r < n ? *reinterpret_cast<const double2*>(X + 2 * r) : make_double2(0.0, 0.0);
                const int ls = (nl > 0 && r < n) ? slot[r] : -1;
                W[q] = r >= n ? make_double2(0.0, 0.0)
                     : ls >= 0 ? make_double2(wl[2 * ls], wl[2 * ls + 1])
                               : *reinterpret_cast<const double2*>(ws + 2 * r);
            }
        } else {
        // W = A C   (lanczos_krylov.m:81): short rows by their owner, gathers from LDS
#pragma unroll
        for (int q = 0; q < R; ++q) {
            const int r = tid + q * kFusedThreads;
            Cv[q] = r < n ? *reinterpret_cast<const double2*>(X + 2 * r) : make_double2(0.0, 0.0);
            double s0 = 0.0, s1 = 0.0;
#if defined(KT_REG_DIAG) && KT_REG_DIAG >= 2
            if (false) {  // diagnostic: no row sums at all (the phase's fixed cost)
#else
            if (r < n && (nl == 0 || slot[r] < 0)) {
#endif
                const int rb = rp[r], re = rp[r + 1];
                // four nonzeros per round; the indices are clamped into the row
                // (a masked weight drops the repeats) so that every load is
                // unconditional: the four column reads issue together, then the
                // four gathers -- predicated loads compiled to one branch and
                // one LDS round trip EACH (the SpMM took ~13 us per Lanczos step).
                // A slot past the row's end gathers the zero row n instead of
                // repeating the last column: every such lane of the wave reads
                // one address (an LDS broadcast, not one more random access
                // in the instruction's bank conflicts); x + 1 * 0 = x + 0 * v.
                if (M.unit) {
                    for (int k0 = rb; k0 < re; k0 += 4) {
                        int cc[4];
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            const int c0 = col(min(k0 + u, re - 1));
                            cc[u] = (KT_REG_ZROW && k0 + u >= re) ? n : c0;
                        }
                        double2 v[4];
#pragma unroll
                        for (int u = 0; u < 4; ++u) v[u] = reg_gather(X, cc[u]);
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            const double a = (k0 + u < re) ? 1.0 : 0.0;
                            s0 = fma(a, v[u].x, s0);
                            s1 = fma(a, v[u].y, s1);
                        }
                    }
                } else {
                    for (int k0 = rb; k0 < re; k0 += 4) {
                        int cc[4];
                        double a[4];
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            const int k = min(k0 + u, re - 1);
                            const int c0 = col(k);
                            cc[u] = (KT_REG_ZROW && k0 + u >= re) ? n : c0;
                            a[u] = va[k];
                        }
                        double2 v[4];
#pragma unroll
                        for (int u = 0; u < 4; ++u) v[u] = reg_gather(X, cc[u]);
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            const double w = (k0 + u < re) ? a[u] : 0.0;
                            s0 = fma(w, v[u].x, s0);
                            s1 = fma(w, v[u].y, s1);
                        }
                    }
                }
            }
            W[q] = make_double2(s0, s1);
        }
        for (int li = wave; li < nl; li += kFusedWaves) {
            const int r = M.long_rows[li];
            const int b = rp[r], e = rp[r + 1];
            double s0 = 0.0, s1 = 0.0;
            for (int k = b + lane; k < e; k += 64) {
                const int cc = col(k);
                const double a = M.unit ? 1.0 : va[k];
                const double2 v = *reinterpret_cast<const double2*>(X + 2 * cc);
                s0 = fma(a, v.x, s0);
                s1 = fma(a, v.y, s1);
            }
            s0 = wave_sum64(s0);
            s1 = wave_sum64(s1);
            if (lane == 0) {
                wl[2 * li] = s0;
                wl[2 * li + 1] = s1;
            }
        }
        if (nl > 0) {
            __syncthreads();
#pragma unroll
            for (int q = 0; q < R; ++q) {
                const int r = tid + q * kFusedThreads;
                const int ls = r < n ? slot[r] : -1;
                if (ls >= 0) W[q] = make_double2(wl[2 * ls], wl[2 * ls + 1]);
            }
        }
        }  // !have_spec
        FPROF(1);
        // X is overwritten by Q in sweep E: every SpMM read is behind the sweeps' barriers
        reg_orth<R>(n, j > 1, true, P, Cv, W, X, red, bc, par, o);
#pragma unroll
        for (int q = 0; q < R; ++q) P[q] = Cv[q];  // the next step's window block
        if (tid == 0) {  // step j's blocks (fused_xm_blk's entries, appended)
            double h[11];
#pragma unroll
            for (int k = 0; k < 8; ++k) h[k] = o.g[k] + o.g[8 + k];
            h[8] = o.beta1;
            h[9] = o.r12;
            h[10] = o.beta2;
            const int k = j - 1;
            Blk2 m;
            m.a = h[2];
            m.b = 0.5 * (h[3] + h[6]);
            m.c = h[7];
            m.u0 = m.u1 = m.u2 = m.u3 = 0.0;
            gblk[k] = m;
            if (k == 0) {  // T(0:1, 0:1) += Cm (column-major)
                t0[0] = h[2] + cm[0];
                t0[1] = 0.5 * ((h[3] + cm[1]) + (h[6] + cm[2]));
                t0[2] = h[7] + cm[3];
            } else {  // coupling of block k-1 to k: lower block R_{k-1}, upper block from record k
                Blk2& p = gblk[k - 1];
                p.u0 = 0.5 * (lastr[0] + h[0]);
                p.u1 = 0.5 * (0.0 + h[4]);
                p.u2 = 0.5 * (lastr[1] + h[1]);
                p.u3 = 0.5 * (lastr[2] + h[5]);
            }
            lastr[0] = h[8];
            lastr[1] = h[9];
            lastr[2] = h[10];
        }
        if (tid == 0) s_spec_next = 0;
        __syncthreads();  // X = V_{j+1}, blocks of step j visible
        FPROF(6);
        // While waves 0-3 solve step j's eigenvalues (xm_waves: <= 2 waves per
        // projection up to 2j = 32), waves 4-7 would wait at its barrier: they
        // form step j+1's W = A C meanwhile (X = V_{j+1} is final), every row
        // by row_sum in CSR order -- the owners' sums, bit for bit -- into ws
        // and wl.  If step j stops, the sums are simply not used.
        have_spec = spec && j < it && 2 * xm_waves(2 * j) <= kFusedWaves / 2;
        // the short rows in blocks of 64 taken from an LDS counter: waves 4-7
        // start at once, waves 0-3 join as their eigenvalues finish (help())
        auto spec_rows = [&]() {
            if (!have_spec || !KT_REG_SPEC_DYN) return;
            for (;;) {
                int cb = 0;
                if (lane == 0) cb = atomicAdd(&s_spec_next, 1);
                cb = __builtin_amdgcn_readfirstlane(cb);
                if (cb * 64 >= n) break;
                const int r = cb * 64 + lane;
                if (r < n && (nl == 0 || slot[r] < 0)) {
                    double s0 = 0.0, s1 = 0.0;
                    row_sum(r, s0, s1);
                    *reinterpret_cast<double2*>(ws + 2 * r) = make_double2(s0, s1);
                }
            }
        };
        if (have_spec && wave >= kFusedWaves / 2) {
            if (!KT_REG_SPEC_DYN) {  // round-6 first form: waves 4-7 alone, rows strided
                const int t2 = tid - kFusedThreads / 2;
#pragma unroll 1
                for (int r = t2; r < n; r += kFusedThreads / 2) {
                    if (nl == 0 || slot[r] < 0) {
                        double s0 = 0.0, s1 = 0.0;
                        row_sum(r, s0, s1);
                        *reinterpret_cast<double2*>(ws + 2 * r) = make_double2(s0, s1);
                    }
                }
            }
            for (int li = wave - kFusedWaves / 2; li < nl; li += kFusedWaves / 2) {
                const int r = M.long_rows[li];
                const int b = rp[r], e = rp[r + 1];
                double s0 = 0.0, s1 = 0.0;
                for (int k = b + lane; k < e; k += 64) {
                    const int cc = col(k);
                    const double a = M.unit ? 1.0 : va[k];
                    const double2 v = *reinterpret_cast<const double2*>(X + 2 * cc);
                    s0 = fma(a, v.x, s0);
                    s1 = fma(a, v.y, s1);
                }
                s0 = wave_sum64(s0);
                s1 = wave_sum64(s1);
                if (lane == 0) {
                    wl[2 * li] = s0;
                    wl[2 * li + 1] = s1;
                }
            }
        }
#ifdef KT_FUSED_NOEIG
        spec_rows();
        __syncthreads();
        xm = (double)j;
#else
        xm = reg_xm_blk(j, fun, gblk, t0, ev, spec_rows);  // its first barrier: ws / wl complete
#endif
        FPROF(7);
        lucky = sqrt(o.beta1 * o.beta1 + o.r12 * o.r12 + o.beta2 * o.beta2) < 1e-8;  // :91-93
#ifdef KT_FUSED_NOEIG
        lucky = 0;  // diagnostic builds run exactly `it` steps
#endif
        bool stop = false;
        if (j <= 2) {  // :104-118, lag d = 2
            if (j == 1) x0 = xm;
            else x1 = xm;
        } else if (fabs(xm - x0) < tol) {
            stop = true;
        } else {
            x0 = x1;
            x1 = xm;
        }
        FPROF(8);
        if (stop || lucky || j == it) {
            iter = j;
            break;
        }
    }
#ifdef KT_FUSED_PROF
    if (c == 0 && tid == 0)
        printf("reg_prof spec=%d lds=%d n=%d it=%d iter=%d start=%llu spmm=%llu A=%llu B=%llu C=%llu D=%llu E=%llu eig=%llu stop=%llu (x10ns) shader_MHz=%.0f\n",
               spec, (int)L.total, n, it, iter, g_fprof[0], g_fprof[1], g_fprof[2], g_fprof[3], g_fprof[4], g_fprof[5], g_fprof[6],
               g_fprof[7], g_fprof[8], 100.0 * (double)(clock64() - clk0) / (double)(wall_clock64() - wclk0));
#endif
    if (tid == 0) {
        double* st = state + (int64_t)c * PS_N;
        st[PS_XM] = xm;
        st[PS_ITER] = iter;
        st[PS_LUCKY] = lucky ? 1.0 : 0.0;
        st[PS_DONE] = 1.0;
    }
}

// One greedy step's bookkeeping on the device (greedy_krylov.m:80-93 with
// krylov_miobi(A, 1, E, ...), break mode): the candidate with the smallest
// score (the first on ties, as the host loop), its pair dropped from the
// ranking (greedy_krylov.m:84-86), and A with that edge deleted from both
// triangles (krylov_miobi.m:129-135) written to the other CSR buffer -- row
// order and the surviving long rows' order kept, so the next candidate launch
// computes exactly what it computes after the host edit.  One workgroup.
__global__ __launch_bounds__(1024) void k_greedy_edit(int C, const double* __restrict__ state, int* __restrict__ Ti,
                                                     int* __restrict__ Tj, int nT, int n, int long_thresh,
                                                     const int* __restrict__ rp, const int* __restrict__ ci,
                                                     const double* __restrict__ va, const int* __restrict__ lr,
                                                     const int* __restrict__ dyn, int* __restrict__ rp2,
                                                     int* __restrict__ ci2, double* __restrict__ va2,
                                                     int* __restrict__ lr2, int* __restrict__ dyn2, int step,
                                                     int* __restrict__ sel, double* __restrict__ selv) {
    __shared__ double wv[16];
    __shared__ int wi[16];
    __shared__ int s_best, s_ci, s_cj, s_k1, s_k2;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    double v = INFINITY;
    int idx = 0x7fffffff;
    for (int c = tid; c < C; c += 1024) {
        const double x = state[(int64_t)c * PS_N + PS_XM];
        if (x < v) {  // ascending c per thread: the first minimum; NaN never wins (as xm < bv)
            v = x;
            idx = c;
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const double ov = __shfl_xor(v, o, 64);
        const int oi = __shfl_xor(idx, o, 64);
        if (ov < v || (ov == v && oi < idx)) {
            v = ov;
            idx = oi;
        }
    }
    if (lane == 0) {
        wv[wave] = v;
        wi[wave] = idx;
    }
    __syncthreads();
    if (tid == 0) {  // (v, idx) hold wave 0's minimum
        for (int w = 1; w < 16; ++w)
            if (wv[w] < v || (wv[w] == v && wi[w] < idx)) {
                v = wv[w];
                idx = wi[w];
            }
        const bool ok = idx < C;
        s_best = ok ? idx : -1;
        s_ci = ok ? Ti[idx] : -1;
        s_cj = ok ? Tj[idx] : -1;
        sel[2 * step] = s_ci;
        sel[2 * step + 1] = s_cj;
        selv[step] = v;
        // the entries (ci, cj) and (cj, ci): binary search in their sorted rows
        int k1 = -1, k2 = -1;
        if (ok) {
            auto find = [&](int r, int c) {
                int lo = rp[r], hi = rp[r + 1];
                while (lo < hi) {
                    const int mid = (lo + hi) >> 1;
                    if (ci[mid] < c) lo = mid + 1;
                    else hi = mid;
                }
                return (lo < rp[r + 1] && ci[lo] == c) ? lo : -1;
            };
            k1 = find(s_ci, s_cj);
            if (s_cj != s_ci) k2 = find(s_cj, s_ci);
        }
        s_k1 = k1;
        s_k2 = k2;
    }
    __syncthreads();
    const int best = s_best, r1 = s_ci, r2 = s_cj, k1 = s_k1, k2 = s_k2;
    const int nnz = dyn[0];
    // ranking: drop entry `best` (read all, barrier, write shifted)
    int tv[4], tw[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int t = best + 1 + tid + u * 1024;
        tv[u] = (best >= 0 && t < nT) ? Ti[t] : 0;
        tw[u] = (best >= 0 && t < nT) ? Tj[t] : 0;
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int t = best + 1 + tid + u * 1024;
        if (best >= 0 && t < nT) {
            Ti[t - 1] = tv[u];
            Tj[t - 1] = tw[u];
        }
    }
    // the CSR without positions k1, k2 (into the other buffer)
    for (int t = tid; t < nnz; t += 1024) {
        if (t == k1 || t == k2) continue;
        const int d = t - (k1 >= 0 && t > k1) - (k2 >= 0 && t > k2);
        ci2[d] = ci[t];
        va2[d] = va[t];
    }
    for (int r = tid; r <= n; r += 1024)
        rp2[r] = rp[r] - (k1 >= 0 && r > r1) - (k2 >= 0 && r > r2);
    __syncthreads();
    if (tid == 0) {  // long rows that stay long, in their order
        int m = 0;
        for (int l = 0; l < dyn[1]; ++l) {
            const int r = lr[l];
            if (rp2[r + 1] - rp2[r] > long_thresh) lr2[m++] = r;
        }
        dyn2[0] = nnz - (k1 >= 0) - (k2 >= 0);
        dyn2[1] = m;
    }
}

// Rows per thread of k_pair_reg: 2, 4, then exact from 6 (one row more costs
// ~12 VGPRs: at R = 8 the kernel spills 6-18 VGPRs to scratch at 2 waves per
// SIMD, R = 7 and below do not -- India, n = 3,228, takes R = 7).
// KT_REG_R_POW2=1 builds the round-5 choice (2, 4, 8) for A/Bs.
#ifndef KT_REG_R_POW2
#define KT_REG_R_POW2 0
#endif
static int reg_rows(int n) {
    const int rows = (n + kFusedThreads - 1) / kFusedThreads;
    if (KT_REG_R_POW2) return rows <= 2 ? 2 : rows <= 4 ? 4 : 8;
    return rows <= 2 ? 2 : rows <= 4 ? 4 : rows <= 6 ? 6 : rows;
}

// Whether k_pair_reg forms the next step's row sums during the eigenvalues
// (spec: one more n x 2 LDS block); the weights leave the LDS for it (csr 2
// -> 1: read from global memory, L2-resident) when both do not fit.
static int reg_spec_fits(int n, int64_t nnz, int it, bool has_long, int& csr, size_t lds_max) {
    if (!KT_REG_SPEC) return 0;
    if (reg_lds_layout(n, nnz, it, has_long, csr, true).total <= lds_max) return 1;
    if (csr == 2 && reg_lds_layout(n, nnz, it, has_long, 1, true).total <= lds_max) {
        csr = 1;
        return 1;
    }
    return 0;
}

bool pair_reg_applies(int n, int64_t nnz, int it, int n_long, bool unit) {
    const char* de = getenv("KT_PAIRS_DENSE_EIG");
    const char* rg = getenv("KT_PAIRS_REG");
    constexpr size_t kLdsMax = 160 * 1024 - 2048;
    const bool has_long = std::min(n_long, kRegLongCap) > 0;
    (void)unit;
    return !(de && de[0] == '1') && !(rg && rg[0] == '0') && n >= 2 && n <= 8 * kFusedThreads &&
           nnz < (int64_t)1 << 31 && reg_lds_layout(n, nnz, it, has_long, 0).total <= kLdsMax;
}

// k_pair_reg on candidates ii/jj (device) with the CSR's nnz / n_long read
// from dyn; nnz_max / has_long_max size the LDS (the first step's matrix)
hipError_t launch_pair_reg_dyn(int C, int n, int64_t nnz_max, const CsrView& A, bool unit, const int* ii,
                               const int* jj, const double* B, int it, int fun, double tol, double* state,
                               const int* dyn, hipStream_t st) {
    if (C <= 0) return hipSuccess;
    const FusedCSR M{A.rp, A.ci, A.va, A.long_rows, A.n_long, A.long_thresh, unit ? 1 : 0};
    constexpr size_t kLdsMax = 160 * 1024 - 2048;
    const bool has_long = std::min(A.n_long, kRegLongCap) > 0;
    int csr = 0;
    for (int cand = unit ? 1 : 2; cand >= 1; --cand)
        if (reg_lds_layout(n, nnz_max, it, has_long, cand).total <= kLdsMax) {
            csr = cand;
            break;
        }
    const int spec = reg_spec_fits(n, nnz_max, it, has_long, csr, kLdsMax);
    const size_t lds = reg_lds_layout(n, nnz_max, it, has_long, csr, spec).total;
    const int rr = reg_rows(n);
#define KT_REG_LAUNCH(RR, CC)                                                                                  \
    k_pair_reg<RR, CC><<<C, kFusedThreads, lds, st>>>(C, n, (int)nnz_max, M, ii, jj, B[0], B[1], B[2], B[3], it, \
                                                      fun, tol, state, dyn, spec)
#define KT_REG_CSR(RR)                       \
    if (csr == 0) KT_REG_LAUNCH(RR, 0);      \
    else if (csr == 1) KT_REG_LAUNCH(RR, 1); \
    else KT_REG_LAUNCH(RR, 2)
    if (rr == 2) { KT_REG_CSR(2); }
    else if (rr == 4) { KT_REG_CSR(4); }
    else if (rr == 6) { KT_REG_CSR(6); }
    else if (rr == 7) { KT_REG_CSR(7); }
    else { KT_REG_CSR(8); }
#undef KT_REG_CSR
#undef KT_REG_LAUNCH
    return hipGetLastError();
}

hipError_t launch_greedy_edit(int C, const double* state, int* Ti, int* Tj, int nT, int n, int long_thresh,
                              const int* rp, const int* ci, const double* va, const int* lr, const int* dyn,
                              int* rp2, int* ci2, double* va2, int* lr2, int* dyn2, int step, int* sel,
                              double* selv, hipStream_t st) {
    if (nT > 4 * 1024) return hipErrorInvalidValue;
    k_greedy_edit<<<1, 1024, 0, st>>>(C, state, Ti, Tj, nT, n, long_thresh, rp, ci, va, lr, dyn, rp2, ci2, va2,
                                      lr2, dyn2, step, sel, selv);
    return hipGetLastError();
}

hipError_t launch_pair_fused(int C, int n, int64_t nnz, const CsrView& A, bool unit, const int* ii,
                             const int* jj, const double* B, int it, int fun, double tol, double* vec,
                             double* big, int64_t big_stride, double* state, hipStream_t st) {
    if (C <= 0) return hipSuccess;
    const FusedCSR M{A.rp, A.ci, A.va, A.long_rows, A.n_long, A.long_thresh, unit ? 1 : 0};
    // KT_PAIRS_DENSE_EIG=1: the dense tridiagonalisation + multisection in LDS
    // (and the one-thread solver past 2j = 56) instead of block Sturm counts
    const char* de = getenv("KT_PAIRS_DENSE_EIG");
    const int blk_eig = !(de && de[0] == '1');
    // register-resident runs (k_pair_reg) up to 8 rows per thread; KT_PAIRS_REG=0 keeps k_pair_fused.
    // LDS: the gather block and the eigen workspace, then as much of the CSR as
    // fits (row pointers + u16 columns, then the weights).
    const char* rg = getenv("KT_PAIRS_REG");
    constexpr size_t kLdsMax = 160 * 1024 - 2048;  // static __shared__ of the kernel
    const bool has_long = std::min(A.n_long, kRegLongCap) > 0;
    if (blk_eig && !(rg && rg[0] == '0') && n >= 2 && n <= 8 * kFusedThreads && nnz < (int64_t)1 << 31 &&
        reg_lds_layout(n, nnz, it, has_long, 0).total <= kLdsMax) {
        int csr = 0;
        for (int cand = unit ? 1 : 2; cand >= 1; --cand)
            if (reg_lds_layout(n, nnz, it, has_long, cand).total <= kLdsMax) {
                csr = cand;
                break;
            }
        const int spec = reg_spec_fits(n, nnz, it, has_long, csr, kLdsMax);
        const size_t lds = reg_lds_layout(n, nnz, it, has_long, csr, spec).total;
        const int rr = reg_rows(n);
#define KT_REG_LAUNCH(RR, CC)                                                                                  \
    k_pair_reg<RR, CC><<<C, kFusedThreads, lds, st>>>(C, n, (int)nnz, M, ii, jj, B[0], B[1], B[2], B[3], it, fun, \
                                                      tol, state, nullptr, spec)
#define KT_REG_CSR(RR)                       \
    if (csr == 0) KT_REG_LAUNCH(RR, 0);      \
    else if (csr == 1) KT_REG_LAUNCH(RR, 1); \
    else KT_REG_LAUNCH(RR, 2)
        if (rr == 2) { KT_REG_CSR(2); }
        else if (rr == 4) { KT_REG_CSR(4); }
        else if (rr == 6) { KT_REG_CSR(6); }
        else if (rr == 7) { KT_REG_CSR(7); }
        else { KT_REG_CSR(8); }
#undef KT_REG_CSR
#undef KT_REG_LAUNCH
        return hipGetLastError();
    }
    k_pair_fused<<<C, kFusedThreads, pair_fused_lds_bytes(it), st>>>(
        C, n, M, ii, jj, B[0], B[1], B[2], B[3], it, fun, tol, vec, big, big_stride, state, blk_eig);
    return hipGetLastError();
}

// active[0] = number of candidates not done
__global__ void k_pair_active(int C, const double* __restrict__ state, int* __restrict__ active) {
    __shared__ int red[256];
    int cnt = 0;
    for (int c = threadIdx.x; c < C; c += blockDim.x) cnt += state[(int64_t)c * PS_N + PS_DONE] == 0.0;
    red[threadIdx.x] = cnt;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) active[0] = red[0];
}

hipError_t launch_pair_eig(int C, int j, int it, int fun, double tol, const double* hist,
                           const double* Cm, double* scratch, int64_t sstride, double* state,
                           int* active, hipStream_t st) {
    const char* de = getenv("KT_PAIRS_DENSE_EIG");
    if (!(de && de[0] == '1')) {  // block Sturm counts: no LDS limit, no one-thread fallback
        const size_t lds = sizeof(double) * (11 * (size_t)j + 14 * (size_t)j + 4 * (size_t)j);
        k_pair_eig_blk<<<C, kFusedThreads, lds, st>>>(C, j, it, fun, tol, hist, Cm, state);
    } else if (2 * j <= 56) {  // 2 nn^2 + 6 nn doubles <= 52 KB of LDS
        const size_t lds = sizeof(double) * (2 * (size_t)(2 * j) * (2 * j) + 6 * (size_t)(2 * j));
        // W = 1, MS = 4 measured fastest (profiles/r01_greedy_eig_variants.txt):
        // the Sturm rounds are VALU-issue-bound, more waves per SIMD only
        // evaluate more points per round
        k_pair_eig_wave<1, 4><<<C, 128, lds, st>>>(C, j, it, fun, tol, hist, Cm, state);
    } else {
        k_pair_eig<<<(C + 63) / 64, 64, 0, st>>>(C, j, it, fun, tol, hist, Cm, scratch, sstride, state);
    }
    k_pair_active<<<1, 256, 0, st>>>(C, state, active);
    return hipGetLastError();
}

// U_c = [e_i, e_j] (krylov_miobi.m:82-84); X pre-zeroed.
__global__ void k_pair_select(int C, const int* __restrict__ ii, const int* __restrict__ jj,
                              double* __restrict__ X, int ld) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    X[(int64_t)ii[c] * ld + 2 * c] = 1.0;
    X[(int64_t)jj[c] * ld + 2 * c + 1] = 1.0;
}

hipError_t launch_pair_select(int C, const int* ii, const int* jj, double* X, int ld,
                              hipStream_t st) {
    if (C <= 0) return hipSuccess;
    k_pair_select<<<(C + 255) / 256, 256, 0, st>>>(C, ii, jj, X, ld);
    return hipGetLastError();
}

void pairs_orth_geometry(int n, int C, int num_cu, int* nrb, int* rows_per_blk) {
    const int groups = (C + 63) / 64;
    int want = (4 * num_cu + groups - 1) / groups;           // ~4 workgroups per CU
    int rpb = (n + want - 1) / want;
    rpb = ((rpb < 16 ? 16 : rpb) + kSweepWaves - 1) / kSweepWaves * kSweepWaves;
    *rows_per_blk = rpb;
    *nrb = (n + rpb - 1) / rpb;
}

size_t pairs_part_doubles(int n, int C, int num_cu) {
    int nrb, rpb;
    pairs_orth_geometry(n, C, num_cu, &nrb, &rpb);
    return (size_t)8 * C * nrb;
}

size_t pairs_coef_doubles(int C) { return (size_t)CF_NCOEF * C; }

hipError_t launch_pairs_orth(int C, int n, int num_cu, const double* prev, const double* cur,
                             double* W, int ld, double* coef, double* part, double* hr,
                             hipStream_t st, const int* skip) {
    if (C <= 0) return hipSuccess;
    int nrb, rpb;
    pairs_orth_geometry(n, C, num_cu, &nrb, &rpb);
    const dim3 grid((C + 63) / 64, nrb);
    const int cgrid = (C + 3) / 4;
    if (cur) {
        k_pairs_sweep<PH_A><<<grid, kSweepBlock, 0, st>>>(n, C, rpb, prev, cur, W, ld, coef, part, skip);
        k_pairs_coef<PH_A><<<cgrid, 256, 0, st>>>(C, nrb, part, W, ld, coef, hr, skip);
        k_pairs_sweep<PH_B><<<grid, kSweepBlock, 0, st>>>(n, C, rpb, prev, cur, W, ld, coef, part, skip);
        k_pairs_coef<PH_B><<<cgrid, 256, 0, st>>>(C, nrb, part, W, ld, coef, hr, skip);
        k_pairs_sweep<PH_C><<<grid, kSweepBlock, 0, st>>>(n, C, rpb, prev, cur, W, ld, coef, part, skip);
        k_pairs_coef<PH_C><<<cgrid, 256, 0, st>>>(C, nrb, part, W, ld, coef, hr, skip);
    } else {
        k_pairs_sweep<PH_C0><<<grid, kSweepBlock, 0, st>>>(n, C, rpb, nullptr, nullptr, W, ld, coef, part, skip);
        k_pairs_coef<PH_C0><<<cgrid, 256, 0, st>>>(C, nrb, part, W, ld, coef, hr, skip);
    }
    k_pairs_sweep<PH_D><<<grid, kSweepBlock, 0, st>>>(n, C, rpb, nullptr, nullptr, W, ld, coef, part, skip);
    k_pairs_coef<PH_D><<<cgrid, 256, 0, st>>>(C, nrb, part, W, ld, coef, hr, skip);
    k_pairs_sweep<PH_E><<<grid, kSweepBlock, 0, st>>>(n, C, rpb, nullptr, nullptr, W, ld, coef, part, skip);
    return hipGetLastError();
}

}  // namespace kt

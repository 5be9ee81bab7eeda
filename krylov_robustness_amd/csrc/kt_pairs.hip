// kt_pairs.hip -- kernels of the batched greedy candidate evaluation
// (krylov_miobi.m:76-99: one block-2 Lanczos run per candidate edge, all
// candidates of a greedy step advanced together).
//
// Layout: a "pair block" is a row-major n x ld device array; candidate c owns
// columns 2c and 2c+1.  The SpMM that advances every candidate is the shared
// k_spmm_block kernel over all 2C columns; everything per candidate (CGS2
// against the 2-block window, the thin QR, the R factor) is fused into ONE
// workgroup-per-candidate kernel, so a Lanczos step of C candidates is
// spmm + one launch + one small device->host copy.
#include <hip/hip_runtime.h>

#include "kt_launch.h"

namespace kt {

constexpr int kPairBlock = 256;
constexpr int kPairWaves = kPairBlock / 64;

// Deterministic block sum of NV per-thread values: fixed xor tree inside each
// wave, then the waves' partials added in wave order.  Every thread gets the
// totals.  `lds` holds NV * kPairWaves doubles.
template <int NV>
__device__ __forceinline__ void block_sum(double (&v)[NV], double* lds) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        double x = v[k];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
        v[k] = x;
    }
    if (lane == 0)
#pragma unroll
        for (int k = 0; k < NV; ++k) lds[k * kPairWaves + wave] = v[k];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        double s = 0.0;
#pragma unroll
        for (int w = 0; w < kPairWaves; ++w) s += lds[k * kPairWaves + w];
        v[k] = s;
    }
    __syncthreads();
}

// U_c = [e_i, e_j] (krylov_miobi.m:82-84); X pre-zeroed.
__global__ void k_pair_select(int C, const int* __restrict__ ii, const int* __restrict__ jj,
                              double* __restrict__ X, int ld) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    X[(int64_t)ii[c] * ld + 2 * c] = 1.0;
    X[(int64_t)jj[c] * ld + 2 * c + 1] = 1.0;
}

// LAPACK dlarfg on (alpha, ||x||^2 = xx): returns beta, tau and the scale
// 1/(alpha - beta) that turns x into the tail of v (v(1) = 1).
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

// Per candidate c (one workgroup):
//   if cur != nullptr:  CGS2 of W_c against the window [prev_c, cur_c]
//       (lanczos_krylov.m:109-115, two passes h = V'w; w = w - V h), the
//       summed h written to hr[c*11 + 0..7] (column-major 4 x 2, rows
//       prev0, prev1, cur0, cur1; prev rows 0 when prev == nullptr);
//   then  [W_c, R_c] = qr(W_c, 0)  (lanczos_krylov.m:90) as LAPACK does it:
//       dgeqr2 (two dlarfg reflectors) + dorg2r, R to hr[c*11 + 8..10]
//       = (R11, R12, R22).  Exactly rank-deficient blocks get the same
//       Householder completion as MATLAB's qr (tau = 0 reflectors).
__global__ __launch_bounds__(kPairBlock) void k_pair_orth(int n, const double* __restrict__ prev,
                                                          const double* __restrict__ cur,
                                                          double* __restrict__ W, int ld,
                                                          double* __restrict__ hr) {
    __shared__ double lds[8 * kPairWaves];
    const int c = blockIdx.x;
    const int64_t off = 2 * (int64_t)c;
    const int tid = threadIdx.x;
    auto at = [&](const double* B, int r) {
        return *reinterpret_cast<const double2*>(B + (int64_t)r * ld + off);
    };
    double* out = hr + (int64_t)c * 11;
    if (cur) {
        double h[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) h[k] = 0.0;
        for (int pass = 0; pass < 2; ++pass) {
            double g[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) g[k] = 0.0;
            for (int r = tid; r < n; r += kPairBlock) {
                const double2 w = at(W, r), u = at(cur, r);
                const double2 p = prev ? at(prev, r) : make_double2(0.0, 0.0);
                g[0] += p.x * w.x; g[1] += p.y * w.x; g[2] += u.x * w.x; g[3] += u.y * w.x;
                g[4] += p.x * w.y; g[5] += p.y * w.y; g[6] += u.x * w.y; g[7] += u.y * w.y;
            }
            block_sum<8>(g, lds);
            for (int r = tid; r < n; r += kPairBlock) {
                double2 w = at(W, r);
                const double2 u = at(cur, r);
                const double2 p = prev ? at(prev, r) : make_double2(0.0, 0.0);
                w.x -= p.x * g[0] + p.y * g[1] + u.x * g[2] + u.y * g[3];
                w.y -= p.x * g[4] + p.y * g[5] + u.x * g[6] + u.y * g[7];
                *reinterpret_cast<double2*>(W + (int64_t)r * ld + off) = w;
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) h[k] += g[k];
        }
        if (tid == 0)
#pragma unroll
            for (int k = 0; k < 8; ++k) out[k] = h[k];
        __syncthreads();  // rows 0/1 read below were written by other threads
    }
    // --- Householder thin QR of the n x 2 block ---
    const double2 w0 = at(W, 0), w1 = at(W, 1);
    double s[1] = {0.0};
    for (int r = 1 + tid; r < n; r += kPairBlock) {
        const double x = at(W, r).x;
        s[0] += x * x;
    }
    block_sum<1>(s, lds);
    double beta1, tau1, scal1;
    larfg(w0.x, s[0], beta1, tau1, scal1);
    // H1 applied to column 2:  t = v1' w(:,2),  z = w(:,2) - tau1 t v1
    double t[1] = {0.0};
    for (int r = 1 + tid; r < n; r += kPairBlock) {
        const double2 w = at(W, r);
        t[0] += w.x * scal1 * w.y;
    }
    block_sum<1>(t, lds);
    const double tt = w0.y + t[0];
    const double r12 = w0.y - tau1 * tt;
    const double v1_1 = w1.x * scal1;
    const double z1 = w1.y - tau1 * tt * v1_1;
    double s2[1] = {0.0};
    for (int r = 2 + tid; r < n; r += kPairBlock) {
        const double2 w = at(W, r);
        const double z = w.y - tau1 * tt * (w.x * scal1);
        s2[0] += z * z;
    }
    block_sum<1>(s2, lds);
    double beta2, tau2, scal2;
    larfg(z1, s2[0], beta2, tau2, scal2);
    // dorg2r: q1 = H1 e1, q2 = H1 H2 e2 = x - tau1 (v1'x) v1 with x = e2 - tau2 v2
    double d[1] = {0.0};
    for (int r = 2 + tid; r < n; r += kPairBlock) {
        const double2 w = at(W, r);
        const double v1 = w.x * scal1;
        const double v2 = (w.y - tau1 * tt * v1) * scal2;
        d[0] += v1 * v2;
    }
    block_sum<1>(d, lds);  // also orders every read of rows 0/1 before the writes
    const double dd = v1_1 + d[0];
    const double k2 = tau1 * (v1_1 - tau2 * dd);
    for (int r = tid; r < n; r += kPairBlock) {
        const double2 w = at(W, r);
        double v1, v2;
        if (r == 0) {
            v1 = 1.0;
            v2 = 0.0;
        } else if (r == 1) {
            v1 = v1_1;
            v2 = 1.0;
        } else {
            v1 = w.x * scal1;
            v2 = (w.y - tau1 * tt * v1) * scal2;
        }
        double2 q;
        q.x = (r == 0 ? 1.0 : 0.0) - tau1 * v1;
        q.y = (r == 1 ? 1.0 : 0.0) - tau2 * v2 - k2 * v1;
        *reinterpret_cast<double2*>(W + (int64_t)r * ld + off) = q;
    }
    if (tid == 0) {
        out[8] = beta1;
        out[9] = r12;
        out[10] = beta2;
    }
}

hipError_t launch_pair_select(int C, const int* ii, const int* jj, double* X, int ld,
                              hipStream_t st) {
    if (C <= 0) return hipSuccess;
    k_pair_select<<<(C + 255) / 256, 256, 0, st>>>(C, ii, jj, X, ld);
    return hipGetLastError();
}

hipError_t launch_pair_orth(int C, int n, const double* prev, const double* cur, double* W,
                            int ld, double* hr, hipStream_t st) {
    if (C <= 0) return hipSuccess;
    k_pair_orth<<<C, kPairBlock, 0, st>>>(n, prev, cur, W, ld, hr);
    return hipGetLastError();
}

}  // namespace kt

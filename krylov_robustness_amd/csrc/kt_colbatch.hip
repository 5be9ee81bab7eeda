// kt_colbatch.hip -- column-batched single-vector Arnoldi kernels
// (function_multiple_entries.m:84-110: one arnoldi_krylov(A, e_i) run per
// distinct row index i of omega, all runs advanced by one SpMM per step).
//
// Layout: the basis of column c is spread over step blocks; block k is a
// row-major n x P array (P = padded column count), so V[k][r][c] sits at
// k*n*P + r*P + c.  Every kernel maps consecutive lanes to consecutive
// columns (coalesced P*8-byte row segments) and splits rows over threads and
// workgroups; per-column sums go through per-workgroup partials reduced in a
// fixed order (bit-reproducible).
#include <hip/hip_runtime.h>

#include "kt_launch.h"

namespace kt {

constexpr int kColBlock = 256;

// part[(k * P + c) * nrb + blk] = sum over this workgroup's rows r (r >= r_lo)
// of V[k][r][c] * W[r][c], for k in [0, nb).  V == W with nb == 1 gives
// squared norms.
__global__ __launch_bounds__(kColBlock) void k_col_dots(int n, int P, int nb, int64_t vstride,
                                                        const double* __restrict__ V,
                                                        const double* __restrict__ W,
                                                        int rows_per_blk, int r_lo,
                                                        double* __restrict__ part) {
    __shared__ double red[kColBlock];
    const int tpr = kColBlock / P;  // threads per column (P <= 128)
    const int c = threadIdx.x % P;
    const int sub = threadIdx.x / P;
    const int r0 = blockIdx.x * rows_per_blk;
    const int r1 = min(n, r0 + rows_per_blk);
    const int nrb = gridDim.x;
    for (int k = 0; k < nb; ++k) {
        const double* Vk = V + (int64_t)k * vstride;
        double s = 0.0;
        for (int r = max(r0, r_lo) + sub; r < r1; r += tpr)
            s = fma(Vk[(int64_t)r * P + c], W[(int64_t)r * P + c], s);
        red[threadIdx.x] = s;
        __syncthreads();
        if (threadIdx.x < P) {
            double t = 0.0;
            for (int q = 0; q < tpr; ++q) t += red[q * P + c];
            part[((int64_t)k * P + c) * nrb + blockIdx.x] = t;
        }
        __syncthreads();
    }
}

// out[k * P + c] = sum_b part[(k * P + c) * nrb + b]   (one wave per (k, c))
__global__ __launch_bounds__(256) void k_col_reduce(int count, int nrb,
                                                    const double* __restrict__ part,
                                                    double* __restrict__ out) {
    const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (t >= count) return;
    const double* p = part + (int64_t)t * nrb;
    double s = 0.0;
    for (int i = lane; i < nrb; i += 64) s += p[i];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if (lane == 0) out[t] = s;
}

// W[r][c] -= sum_k V[k][r][c] * h[k * P + c]
__global__ __launch_bounds__(kColBlock) void k_col_update(int n, int P, int nb, int64_t vstride,
                                                          const double* __restrict__ V,
                                                          const double* __restrict__ h,
                                                          double* __restrict__ W) {
    const int64_t total = (int64_t)n * P;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (int64_t)gridDim.x * blockDim.x) {
        const int c = (int)(t % P);
        double s = 0.0;
        for (int k = 0; k < nb; ++k) s = fma(V[k * vstride + t], h[k * P + c], s);
        W[t] -= s;
    }
}

// [q, r] = qr(w, 0) for each column (LAPACK dlarfg + dorg2r with one
// reflector): s[c] = ||w(2:n, c)||^2.  Writes Q into `Q` (may alias W) and
// r[c] = beta (the 1x1 R).
__global__ __launch_bounds__(kColBlock) void k_col_householder(int n, int P,
                                                               const double* __restrict__ s,
                                                               const double* W,
                                                               double* Q,
                                                               double* __restrict__ r) {
    const int64_t total = (int64_t)n * P;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (int64_t)gridDim.x * blockDim.x) {
        const int c = (int)(t % P);
        const int64_t row = t / P;
        const double alpha = W[c];  // row 0
        const double xx = s[c];
        double beta, tau, scal;
        if (xx == 0.0) {
            beta = alpha;
            tau = 0.0;
            scal = 1.0;
        } else {
            beta = -copysign(hypot(alpha, sqrt(xx)), alpha);
            tau = (beta - alpha) / beta;
            scal = 1.0 / (alpha - beta);
        }
        const double w = W[t];
        // q = H e1 = e1 - tau v,  v = [1; w(2:n) * scal]
        const double q = row == 0 ? 1.0 - tau : -tau * (w * scal);
        if (row == 0) r[c] = beta;
        // row 0 of W is read by every thread: write it last (below)
        if (row != 0) Q[t] = q;
    }
}

// row 0 of the Householder output (separate launch so no thread reads a
// row-0 value another thread has already replaced)
__global__ void k_col_householder_row0(int P, const double* __restrict__ s, double* Q,
                                       const double* W) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= P) return;
    const double alpha = W[c], xx = s[c];
    double tau = 0.0;
    if (xx != 0.0) {
        const double beta = -copysign(hypot(alpha, sqrt(xx)), alpha);
        tau = (beta - alpha) / beta;
    }
    Q[c] = 1.0 - tau;
}

// X[idx[c] * P + c] = 1 (unit start vectors; X pre-zeroed)
__global__ void k_col_select(int C, int P, const int* __restrict__ idx, double* __restrict__ X) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c < C) X[(int64_t)idx[c] * P + c] = 1.0;
}

// rows per workgroup of k_col_dots: about 4 workgroups per CU, at least rpb_lo
// rows each.  The unit-start runs of function_multiple_entries / the Frechet
// entries take rpb_lo = 32 (config 3's call 4.72 -> 4.17 ms against 64,
// profiles/r03_fme_pipeline.txt: with 64 the launch had ~5 waves per CU);
// the eigs restarts keep 64.  The split fixes the partial-sum order.
static int col_rows_per_blk(int n, int num_cu, int rpb_lo) {
    int want = 4 * num_cu;
    int rpb = (n + want - 1) / want;
    if (rpb < rpb_lo) rpb = rpb_lo;
    return rpb;
}

int col_nrb(int n, int num_cu, int rpb_lo) {
    const int rpb = col_rows_per_blk(n, num_cu, rpb_lo);
    return (n + rpb - 1) / rpb;
}

static int stream_blocks(int64_t total) {
    int64_t g = (total + kColBlock - 1) / kColBlock;
    if (g > 8192) g = 8192;
    return (int)(g < 1 ? 1 : g);
}

hipError_t launch_col_dots(int n, int P, int nb, int64_t vstride, const double* V, const double* W,
                           int r_lo, int num_cu, double* part, double* out, hipStream_t st, int rpb_lo) {
    if (nb <= 0) return hipSuccess;
    const int rpb = col_rows_per_blk(n, num_cu, rpb_lo);
    const int nrb = (n + rpb - 1) / rpb;
    k_col_dots<<<nrb, kColBlock, 0, st>>>(n, P, nb, vstride, V, W, rpb, r_lo, part);
    const int count = nb * P;
    k_col_reduce<<<(count + 3) / 4, 256, 0, st>>>(count, nrb, part, out);
    return hipGetLastError();
}

hipError_t launch_col_update(int n, int P, int nb, int64_t vstride, const double* V,
                             const double* h, double* W, hipStream_t st) {
    if (nb <= 0) return hipSuccess;
    k_col_update<<<stream_blocks((int64_t)n * P), kColBlock, 0, st>>>(n, P, nb, vstride, V, h, W);
    return hipGetLastError();
}

hipError_t launch_col_householder(int n, int P, const double* s, double* W, double* Q, double* r,
                                  hipStream_t st) {
    k_col_householder<<<stream_blocks((int64_t)n * P), kColBlock, 0, st>>>(n, P, s, W, Q, r);
    k_col_householder_row0<<<(P + 63) / 64, 64, 0, st>>>(P, s, Q, W);
    return hipGetLastError();
}

hipError_t launch_col_select(int C, int P, const int* idx, double* X, hipStream_t st) {
    if (C <= 0) return hipSuccess;
    k_col_select<<<(C + 255) / 256, 256, 0, st>>>(C, P, idx, X);
    return hipGetLastError();
}

}  // namespace kt

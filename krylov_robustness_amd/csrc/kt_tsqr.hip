// kt_tsqr.hip -- Householder thin QR of a tall-skinny row-major n x bs block
// (bs <= 128), the factorisation MATLAB's qr(w, 0) computes (LAPACK dgeqr2
// reflectors + dorgqr's Q), for lanczos_krylov.m:90, arnoldi_krylov.m:99 and
// mc_trace.m's qr(., 0).
//
// One launch per column k applies reflector H_k to the trailing columns and,
// in the same pass, accumulates the sums the NEXT column's reflector needs
//   sums[j] = W(k+2:n, k+1)' W(k+2:n, j),  j >= k+1
// (sums[k+1] = ||W(k+2:n, k+1)||^2, dlarfg's xnorm^2; sums[j > k+1] give
// t_j = v' w_j without another pass).  A one-wave-per-column reduce launch
// sums the per-workgroup partials in a fixed order and snapshots the next
// pivot row, so every workgroup of the next step derives identical
// coefficients.  Q = (I - V T V') E is then formed with the compact-WY
// factor T (dlarft, host) in one more pass.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstddef>

#include "kt_launch.h"

namespace kt {

constexpr int kTsBlock = 256;

__device__ __forceinline__ void ts_larfg(double alpha, double xx, double& beta, double& tau,
                                         double& scal) {
    if (xx == 0.0) {
        beta = alpha;
        tau = 0.0;
        scal = 1.0;
        return;
    }
    beta = -copysign(hypot(alpha, sqrt(xx)), alpha);
    tau = (beta - alpha) / beta;
    scal = 1.0 / (alpha - beta);
}

// Step k (k = -1: prologue, no reflector, only the sums for column 0).
// Thread (row slot, column c): c = tid % BP.  V (n x BP, pre-zeroed) receives
// the reflector v_k; W row k column k receives beta_k (R's diagonal).
__global__ __launch_bounds__(kTsBlock) void k_ts_step(int n, int bs, int BP, int k,
                                                      double* __restrict__ W, int ld,
                                                      double* __restrict__ V,
                                                      const double* __restrict__ pivot,
                                                      const double* __restrict__ sums,
                                                      int rows_per_blk, double* __restrict__ part,
                                                      double* __restrict__ taus) {
    __shared__ double red[kTsBlock];
    const int c = threadIdx.x % BP;
    const int sub = threadIdx.x / BP;
    const int rpi = kTsBlock / BP;  // rows per block iteration
    const int kn = k + 1;           // the column whose sums we accumulate
    double beta = 0.0, tau = 0.0, scal = 1.0, tc = 0.0, tn = 0.0;
    if (k >= 0) {
        ts_larfg(pivot[k], sums[k], beta, tau, scal);
        if (c > k && c < bs) tc = pivot[c] + scal * sums[c];
        if (kn < bs) tn = pivot[kn] + scal * sums[kn];
        if (blockIdx.x == 0 && threadIdx.x == 0) taus[k] = tau;
    }
    const int r0 = blockIdx.x * rows_per_blk;
    const int r1 = min(n, r0 + rows_per_blk);
    const int rstart = max(r0, k < 0 ? 0 : k);
    double acc = 0.0;
    // Rows go in chunks of kTsU row slots: every load of a chunk is issued
    // (3 kTsU per thread, one memory round trip) before the barrier that
    // orders the chunk's reads before its writes (a thread's row is read by
    // all BP threads of that row, W(r, kn) is rewritten by one of them); the
    // rows and the accumulation order are the single-slot loop's.  Trip
    // counts are uniform across the workgroup (barrier inside).
    constexpr int kTsU = 8;
    for (int base0 = rstart; base0 < r1; base0 += kTsU * rpi) {
        double wk[kTsU], wn[kTsU], wc[kTsU];
#pragma unroll
        for (int u = 0; u < kTsU; ++u) {
            const int r = base0 + u * rpi + sub;
            const bool live = r < r1 && c < bs;
            wk[u] = (live && k >= 0) ? W[(int64_t)r * ld + k] : 0.0;
            wn[u] = (live && kn < bs) ? W[(int64_t)r * ld + kn] : 0.0;
            wc[u] = live ? W[(int64_t)r * ld + c] : 0.0;
        }
        __syncthreads();  // every read of this chunk before any write
#pragma unroll
        for (int u = 0; u < kTsU; ++u) {
            const int r = base0 + u * rpi + sub;
            if (!(r < r1 && c < bs)) continue;
            double v = 0.0;
            double wcu = wc[u];
            if (k >= 0) {
                v = (r == k) ? 1.0 : wk[u] * scal;
                if (c == k) {
                    V[(int64_t)r * BP + k] = v;
                    if (r == k) W[(int64_t)r * ld + k] = beta;
                } else if (c > k) {
                    wcu -= tau * v * tc;
                    W[(int64_t)r * ld + c] = wcu;
                }
            }
            if (kn < bs && c >= kn && r > kn) {
                const double wn_new = k >= 0 ? wn[u] - tau * v * tn : wn[u];
                acc = fma(wn_new, wcu, acc);
            }
        }
    }
    red[threadIdx.x] = acc;
    __syncthreads();
    if (threadIdx.x < BP && kn < bs) {
        double s = 0.0;
        for (int q = 0; q < rpi; ++q) s += red[q * BP + threadIdx.x];
        part[(int64_t)threadIdx.x * gridDim.x + blockIdx.x] = s;
    }
}

// ---------------------------------------------------------------------------
// The reflector sweep with ONE launch per column (k_ts_step1, default where
// the grid fits): every workgroup first sums the previous launch's
// per-workgroup partials itself -- the same fixed order in every workgroup,
// so every workgroup derives identical coefficients -- and reads the pivot
// row the previous launch snapshotted; then it applies H_k to its rows
// (kTs1Rows per workgroup, 1024 threads) and leaves the next column's
// partials and pivot row in the other half of two ping-pong buffers.  The
// per-column reduce launch of the two-launch form goes away (bs + 1 launches
// instead of 2 bs + 1); the sums group rows by workgroup instead of by
// 64-row block, i.e. rounding-level differences from that form.
// part: 2 x [BP][G] doubles, piv: 2 x BP doubles (slot = (k + 1) & 1 written).
// ---------------------------------------------------------------------------
constexpr int kTs1Block = 1024;
constexpr int kTs1Rows = 384;
constexpr int kTs1MaxG = 128;

__global__ __launch_bounds__(kTs1Block) void k_ts_step1(int n, int bs, int BP, int k, int G, int rows_per_wg,
                                                        double* __restrict__ W, int ld, double* __restrict__ V,
                                                        double* __restrict__ part, double* __restrict__ piv,
                                                        double* __restrict__ taus) {
    __shared__ double s_sums[128], s_piv[128];
    __shared__ double red[kTs1Block];
    const int tid = threadIdx.x;
    const int c = tid % BP;
    const int sub = tid / BP;
    const int rpi = kTs1Block / BP;
    const int kn = k + 1;
    const double* part_in = part + (size_t)(k & 1) * BP * G;   // written by launch k - 1
    double* part_out = part + (size_t)(kn & 1) * BP * G;
    const double* piv_in = piv + (size_t)(k & 1) * BP;
    double* piv_out = piv + (size_t)(kn & 1) * BP;
    double beta = 0.0, tau = 0.0, scal = 1.0, tc = 0.0, tn = 0.0;
    if (k >= 0) {
        // sums[j], j in [k, bs): one wave per column, lanes strided over the
        // G partials, then a fixed xor tree -- identical in every workgroup
        const int lane = tid & 63, wave = tid >> 6;
        for (int j = k + wave; j < bs; j += kTs1Block / 64) {
            double sm = 0.0;
            for (int i = lane; i < G; i += 64) sm += part_in[(size_t)j * G + i];
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) sm += __shfl_xor(sm, o, 64);
            if (lane == 0) s_sums[j] = sm;
        }
        if (tid < bs) s_piv[tid] = piv_in[tid];
        __syncthreads();
        ts_larfg(s_piv[k], s_sums[k], beta, tau, scal);
        if (c > k && c < bs) tc = s_piv[c] + scal * s_sums[c];
        if (kn < bs) tn = s_piv[kn] + scal * s_sums[kn];
        if (blockIdx.x == 0 && tid == 0) taus[k] = tau;
    }
    const int r0 = blockIdx.x * rows_per_wg;
    const int r1 = min(n, r0 + rows_per_wg);
    const int rstart = max(r0, k < 0 ? 0 : k);
    double acc = 0.0;
    constexpr int kTsU = 8;  // as k_ts_step: all loads of a chunk before its barrier
    for (int base0 = rstart; base0 < r1; base0 += kTsU * rpi) {
        double wk[kTsU], wn[kTsU], wc[kTsU];
#pragma unroll
        for (int u = 0; u < kTsU; ++u) {
            const int r = base0 + u * rpi + sub;
            const bool live = r < r1 && c < bs;
            wk[u] = (live && k >= 0) ? W[(int64_t)r * ld + k] : 0.0;
            wn[u] = (live && kn < bs) ? W[(int64_t)r * ld + kn] : 0.0;
            wc[u] = live ? W[(int64_t)r * ld + c] : 0.0;
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < kTsU; ++u) {
            const int r = base0 + u * rpi + sub;
            if (!(r < r1 && c < bs)) continue;
            double v = 0.0;
            double wcu = wc[u];
            if (k >= 0) {
                v = (r == k) ? 1.0 : wk[u] * scal;
                if (c == k) {
                    V[(int64_t)r * BP + k] = v;
                    if (r == k) W[(int64_t)r * ld + k] = beta;
                } else if (c > k) {
                    wcu -= tau * v * tc;
                    W[(int64_t)r * ld + c] = wcu;
                }
            }
            if (kn < bs && r == kn) piv_out[c] = wcu;  // the next pivot row, W(kn, :) after H_k
            if (kn < bs && c >= kn && r > kn) {
                const double wn_new = k >= 0 ? wn[u] - tau * v * tn : wn[u];
                acc = fma(wn_new, wcu, acc);
            }
        }
    }
    if (kn >= bs) return;
    red[tid] = acc;
    __syncthreads();
    if (tid < BP) {
        double sm = 0.0;
        for (int q = 0; q < rpi; ++q) sm += red[q * BP + tid];
        part_out[(size_t)tid * G + blockIdx.x] = sm;
    }
}

// rows per workgroup and grid of the one-launch-per-column sweep; 0 when n
// needs more than kTs1MaxG workgroups (the two-launch form then)
int ts_step1_grid(int n, int* rows_per_wg) {
    const int G = (n + kTs1Rows - 1) / kTs1Rows;
    if (G > kTs1MaxG || G < 1) return 0;
    *rows_per_wg = (n + G - 1) / G;
    return G;
}

hipError_t launch_ts_reflectors1(int n, int bs, int BP, double* W, int ld, double* V, double* part, double* piv,
                                 double* taus, hipStream_t st) {
    int rpw = 0;
    const int G = ts_step1_grid(n, &rpw);
    if (!G || BP > 128) return hipErrorInvalidValue;
    for (int k = -1; k < bs; ++k)
        k_ts_step1<<<G, kTs1Block, 0, st>>>(n, bs, BP, k, G, rpw, W, ld, V, part, piv, taus);
    return hipGetLastError();
}

// sums[j] = sum_b part[j][b] for j in [kn, bs); pivot[j] = W(kn, j) for all j
__global__ __launch_bounds__(256) void k_ts_reduce(int bs, int kn, int nrb,
                                                   const double* __restrict__ part,
                                                   const double* __restrict__ W, int ld,
                                                   double* __restrict__ sums,
                                                   double* __restrict__ pivot) {
    const int j = kn + blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (blockIdx.x == 0 && threadIdx.x < 64)
        for (int q = threadIdx.x; q < bs; q += 64) pivot[q] = W[(int64_t)kn * ld + q];
    if (j >= bs) return;
    const double* p = part + (int64_t)j * nrb;
    double s = 0.0;
    for (int i = lane; i < nrb; i += 64) s += p[i];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if (lane == 0) sums[j] = s;
}

// W[r][j] = (r == j) - sum_k V[r][k] M[k][j]   (Q = E - V (T V1'))
__global__ __launch_bounds__(kTsBlock) void k_ts_formq(int n, int bs, int BP,
                                                       const double* __restrict__ V,
                                                       const double* __restrict__ M,
                                                       double* __restrict__ W, int ld) {
    const int64_t total = (int64_t)n * BP;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (int64_t)gridDim.x * blockDim.x) {
        const int j = (int)(t % BP);
        const int64_t r = t / BP;
        if (j >= bs) continue;
        const double* vr = V + r * BP;
        const int kmax = r < bs ? (int)r + 1 : bs;  // V is unit lower trapezoidal
        double s = 0.0;
        for (int kk = 0; kk < kmax; ++kk) s = fma(vr[kk], M[kk * bs + j], s);
        W[r * ld + j] = (r == j ? 1.0 : 0.0) - s;
    }
}


static int ts_rows_per_blk(int n, int num_cu) {
    int want = 2 * num_cu;
    int rpb = (n + want - 1) / want;
    return rpb < 64 ? 64 : rpb;
}

int ts_nrb(int n, int num_cu) {
    const int rpb = ts_rows_per_blk(n, num_cu);
    return (n + rpb - 1) / rpb;
}

// Reflector sweep: after it, W's top bs x bs upper triangle is R, V holds the
// reflectors (unit lower trapezoidal), taus the scalars.
hipError_t launch_ts_reflectors(int n, int bs, int BP, double* W, int ld, double* V, double* pivot,
                                double* sums, double* part, double* taus, int num_cu,
                                hipStream_t st) {
    const int rpb = ts_rows_per_blk(n, num_cu);
    const int nrb = (n + rpb - 1) / rpb;
    for (int k = -1; k < bs; ++k) {
        k_ts_step<<<nrb, kTsBlock, 0, st>>>(n, bs, BP, k, W, ld, V, pivot, sums, rpb, part, taus);
        const int kn = k + 1;
        if (kn < bs)
            k_ts_reduce<<<(bs - kn + 3) / 4, 256, 0, st>>>(bs, kn, nrb, part, W, ld, sums, pivot);
    }
    return hipGetLastError();
}

hipError_t launch_ts_formq(int n, int bs, int BP, const double* V, const double* M, double* W,
                           int ld, hipStream_t st) {
    int64_t g = ((int64_t)n * BP + kTsBlock - 1) / kTsBlock;
    if (g > 8192) g = 8192;
    k_ts_formq<<<(int)g, kTsBlock, 0, st>>>(n, bs, BP, V, M, W, ld);
    return hipGetLastError();
}

// G = sum_s part[s] (px*py each), fixed order
__global__ void k_sum_slabs(int count, int S, const double* __restrict__ part,
                            double* __restrict__ G) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= count) return;
    double s = 0.0;
    for (int q = 0; q < S; ++q) s += part[(int64_t)q * count + t];
    G[t] = s;
}

hipError_t launch_sum_slabs(int count, int S, const double* part, double* G, hipStream_t st) {
    k_sum_slabs<<<(count + 255) / 256, 256, 0, st>>>(count, S, part, G);
    return hipGetLastError();
}

// out = beta * in + c0 I + c1 X1 + c2 X2 + c3 X3   (n x n column-major; in,
// X2, X3 nullable) -- the Paterson-Stockmeyer blocks of the device expm;
// blockIdx.y = matrix of a batch, consecutive matrices n*n apart
__global__ void k_poly4(int n, double beta, const double* __restrict__ in, double c0, double c1,
                        const double* __restrict__ X1, double c2, const double* __restrict__ X2,
                        double c3, const double* __restrict__ X3, double* __restrict__ out) {
    const int64_t total = (int64_t)n * n;
    const int64_t b = (int64_t)blockIdx.y * total;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = t % n, j = t / n;
        double v = (i == j) ? c0 : 0.0;
        v += c1 * X1[b + t];
        if (X2) v += c2 * X2[b + t];
        if (X3) v += c3 * X3[b + t];
        if (in) v += beta * in[b + t];
        out[b + t] = v;
    }
}

hipError_t launch_poly4(int n, double beta, const double* in, double c0, double c1, const double* X1,
                        double c2, const double* X2, double c3, const double* X3, double* out,
                        hipStream_t st, int batch) {
    int64_t g = ((int64_t)n * n + 255) / 256;
    if (g > 4096) g = 4096;
    k_poly4<<<dim3((unsigned)g, (unsigned)batch), 256, 0, st>>>(n, beta, in, c0, c1, X1, c2, X2, c3, X3,
                                                               out);
    return hipGetLastError();
}

}  // namespace kt

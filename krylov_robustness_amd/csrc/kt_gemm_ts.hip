// kt_gemm_ts.hip -- the two tall-skinny products of block Gram-Schmidt on
// row-major n x p blocks (n ~ 10^4-10^6 rows, p <= a few hundred columns):
//
//   gram:    G (px x py, column-major) = X(:, 0:px)' Y(:, 0:py)
//            the CGS2 coefficients h = V' w (arnoldi_krylov.m:119-125,
//            lanczos_krylov.m:109-115), the QR Gram blocks, mc_trace's
//            projections -- a reduction over the long row dimension
//   combine: Y(:, 0:q) = beta Y + alpha X(:, 0:px) C   (C px x q, column-major)
//            the matching update w = w - V h
//
// rocBLAS runs these shapes as generic GEMMs (split-K batched for gram) at
// 0.7-0.9 TB/s of operand traffic (profiles/r03_fg_step_timeline.txt); the
// shapes are bound by reading X once, so the kernels below are built around
// that read.
//
// gram: f64 MFMA (v_mfma_f64_16x16x4_f64), one wave per 32 x 32 output tile
// (2 x 2 MFMA tiles) walking the rows of a chunk 4 at a time, four waves of a
// workgroup on four adjacent i-tiles of the same chunk (Y's rows shared
// through L1).  Each chunk writes its partial tile to a slab; the slabs are
// summed by k_sum_slabs_wide in a fixed order (deterministic).
// combine: VALU, one row per lane and 8 output columns per wave, X and C
// staged in LDS 64 x 64 at a time (C read as broadcasts).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "kt_launch.h"

namespace kt {

typedef double double4_t __attribute__((ext_vector_type(4)));

constexpr int kGramRowsPerChunk = 128;

__device__ __forceinline__ double4_t mfma_f64(double a, double b, double4_t c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// grid: x = row chunk, y = group of 4 i-tiles (128 columns of X), z = j-tile
// (32 columns of Y).  part: slabs of px*py doubles, slab = chunk.
//
// px <= 32 (one i-tile): the four waves split the chunk's rows instead (wave w
// takes rows rb + 32 w + 128 t), and their four tiles are summed through LDS
// in wave order before the slab is written -- otherwise three of the four
// waves would idle and each CU would have one wave's loads in flight.
__global__ __launch_bounds__(256) void k_gram_mfma(int64_t n, const double* __restrict__ X, int ldx, int px,
                                                   const double* __restrict__ Y, int ldy, int py,
                                                   int rows_per_chunk, double* __restrict__ part) {
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const bool rsplit = px <= 32;  // uniform over the grid
    const int i0 = rsplit ? 0 : (blockIdx.y * 4 + wave) * 32;
    const int j0 = blockIdx.z * 32;
    if (i0 >= px) return;  // whole wave idle (uniform)
    const int64_t cb = (int64_t)blockIdx.x * rows_per_chunk;
    const int64_t re = min(n, cb + rows_per_chunk);
    constexpr int KU = 8;
    const int64_t rb = rsplit ? cb + wave * 4 * KU : cb;
    const int64_t rstep = rsplit ? 4 * 4 * KU : 4 * KU;
    const int li = lane & 15, lk = lane >> 4;
    const int ia = i0 + li, ib = i0 + 16 + li, ja = j0 + li, jb = j0 + 16 + li;
    const bool va = ia < px, vb = ib < px, wa = ja < py, wb = jb < py;
    double4_t c00 = {0, 0, 0, 0}, c01 = c00, c10 = c00, c11 = c00;
    // 4 rows per MFMA k-step; 8 k-steps (32 rows, 32 loads per lane) in flight
    // per iteration: a chunk is 4 round trips, not one per row group
    for (int64_t r0 = rb; r0 < re; r0 += rstep) {
        double xa[KU], xb[KU], ya[KU], yb[KU];
#pragma unroll
        for (int u = 0; u < KU; ++u) {
            const int64_t r = r0 + 4 * u + lk;
            const bool live = r < re;
            const double* xr = X + r * ldx;
            const double* yr = Y + r * ldy;
            xa[u] = (live && va) ? xr[ia] : 0.0;
            xb[u] = (live && vb) ? xr[ib] : 0.0;
            ya[u] = (live && wa) ? yr[ja] : 0.0;
            yb[u] = (live && wb) ? yr[jb] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < KU; ++u) {
            c00 = mfma_f64(xa[u], ya[u], c00);
            c01 = mfma_f64(xa[u], yb[u], c01);
            c10 = mfma_f64(xb[u], ya[u], c10);
            c11 = mfma_f64(xb[u], yb[u], c11);
        }
    }
    if (rsplit) {  // the four waves' tiles summed in wave order (deterministic)
        __shared__ double tl[3][16][64];
        if (wave > 0)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                tl[wave - 1][g][lane] = c00[g];
                tl[wave - 1][4 + g][lane] = c01[g];
                tl[wave - 1][8 + g][lane] = c10[g];
                tl[wave - 1][12 + g][lane] = c11[g];
            }
        __syncthreads();
        if (wave > 0) return;
#pragma unroll
        for (int w = 0; w < 3; ++w)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                c00[g] += tl[w][g][lane];
                c01[g] += tl[w][4 + g][lane];
                c10[g] += tl[w][8 + g][lane];
                c11[g] += tl[w][12 + g][lane];
            }
    }
    // D layout (f64 16x16x4): column = lane & 15 (j), row = (lane >> 4) + 4 reg (i)
    double* slab = part + (int64_t)blockIdx.x * px * py;
    const int jc = lane & 15, ir = lane >> 4;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        const int ii = ir + 4 * g;
        const int iA = i0 + ii, iB = i0 + 16 + ii, jA = j0 + jc, jB = j0 + 16 + jc;
        if (iA < px && jA < py) slab[iA + (int64_t)jA * px] = c00[g];
        if (iA < px && jB < py) slab[iA + (int64_t)jB * px] = c01[g];
        if (iB < px && jA < py) slab[iB + (int64_t)jA * px] = c10[g];
        if (iB < px && jB < py) slab[iB + (int64_t)jB * px] = c11[g];
    }
}

// rows per chunk: 128, or more so that there are at most 256 slabs
static int64_t gram_ts_rows(int64_t n) {
    const int64_t r = (n + 255) / 256;
    return r < kGramRowsPerChunk ? kGramRowsPerChunk : (r + 15) / 16 * 16;
}

int gram_ts_chunks(int64_t n) {
    const int64_t r = gram_ts_rows(n);
    return (int)((n + r - 1) / r);
}

// G[t] = sum_s part[s][t] in a fixed order: 4 waves take the slabs s = w mod 4
// (8 loads in flight per lane), then wave 0 adds the four sums in wave order.
__global__ __launch_bounds__(256) void k_sum_slabs_wide(int count, int S, const double* __restrict__ part,
                                                        double* __restrict__ G) {
    __shared__ double red[4][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int t = blockIdx.x * 64 + lane;
    double acc = 0.0;
    if (t < count) {
        int s = w;
        for (; s + 28 < S; s += 32) {
            double v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = part[(int64_t)(s + 4 * u) * count + t];
#pragma unroll
            for (int u = 0; u < 8; ++u) acc += v[u];
        }
        for (; s < S; s += 4) acc += part[(int64_t)s * count + t];
    }
    red[w][lane] = acc;
    __syncthreads();
    if (w == 0 && t < count) G[t] = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
}

hipError_t launch_gram_ts(int64_t n, const double* X, int ldx, int px, const double* Y, int ldy, int py,
                          double* part, double* G, hipStream_t st) {
    const int S = gram_ts_chunks(n);
    dim3 grid(S, (px + 127) / 128, (py + 31) / 32);
    k_gram_mfma<<<grid, 256, 0, st>>>(n, X, ldx, px, Y, ldy, py, (int)gram_ts_rows(n), part);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const int count = px * py;
    k_sum_slabs_wide<<<(count + 63) / 64, 256, 0, st>>>(count, S, part, G);
    return hipGetLastError();
}

// Y[r][j0 + c] = beta Y + alpha sum_i X[r][i] C[i + (j0 + c) px], c < 8, for the
// 64 rows of this workgroup's x-index; wave w takes columns j0 = 32 y + 8 w.
// X arrives in 64 x 64 tiles staged through LDS by coalesced row loads (a lane
// reading its own row straight from memory touches 64 lines per instruction);
// the tile's row stride of 65 doubles puts a wave's 32-lane half on 64
// distinct banks.  C's 64 x 32 tile is read as broadcasts.
constexpr int kCombRows = 64;
constexpr int kCombI = 64;

// X and Y may alias (apply_rinv and shifted_cholqr3 combine in place, q <= 32):
// with q <= 32 the grid has one y-block, so each workgroup reads all px
// columns of its 64 rows (the tile loop) before its first store, and no other
// workgroup touches those rows -- hence no __restrict__ on X / Y.
__global__ __launch_bounds__(256) void k_combine_ts(int64_t n, const double* X, int ldx, int px,
                                                    const double* __restrict__ C, int q, double alpha,
                                                    double beta, double* Y, int ldy) {
    __shared__ double Xs[kCombRows][kCombI + 1];
    __shared__ double Cs[kCombI][32];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int jw = blockIdx.y * 32 + wave * 8;  // this wave's first output column
    const int64_t rbase = (int64_t)blockIdx.x * kCombRows;
    const int64_t r = rbase + lane;
    const bool live = r < n;
    double acc[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) acc[c] = 0.0;
    for (int ib = 0; ib < px; ib += kCombI) {
        const int ni = min(kCombI, px - ib);
        __syncthreads();
        // X tile: wave w loads rows w, w+4, ...; lane = column (512 B per row).
        // All 16 loads of a lane (and its 8 of C) are issued before the LDS
        // stores, so the staging costs one memory round trip, not 16.
        double xv[kCombRows / 4], cv[kCombI * 32 / 256];
#pragma unroll
        for (int q4 = 0; q4 < kCombRows / 4; ++q4) {
            const int64_t gr = rbase + wave + 4 * q4;
            xv[q4] = (gr < n && lane < ni) ? X[gr * ldx + ib + lane] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < kCombI * 32 / 256; ++u) {
            const int t = threadIdx.x + 256 * u;
            const int ii = t >> 5, jj = t & 31;
            const int j = blockIdx.y * 32 + jj;
            cv[u] = (ii < ni && j < q) ? C[(ib + ii) + (int64_t)j * px] : 0.0;
        }
#pragma unroll
        for (int q4 = 0; q4 < kCombRows / 4; ++q4) Xs[wave + 4 * q4][lane] = xv[q4];
#pragma unroll
        for (int u = 0; u < kCombI * 32 / 256; ++u) {
            const int t = threadIdx.x + 256 * u;
            Cs[t >> 5][t & 31] = cv[u];
        }
        __syncthreads();
        if (jw < q) {
            const int jl = wave * 8;
            for (int ii = 0; ii < ni; ++ii) {
                const double x = Xs[lane][ii];
#pragma unroll
                for (int c = 0; c < 8; ++c) acc[c] = fma(x, Cs[ii][jl + c], acc[c]);
            }
        }
    }
    if (!live || jw >= q) return;
    double* yr = Y + r * ldy;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        const int j = jw + c;
        if (j < q) yr[j] = (beta == 0.0 ? 0.0 : beta * yr[j]) + alpha * acc[c];
    }
}

hipError_t launch_combine_ts(int64_t n, const double* X, int ldx, int px, const double* C, int q, double alpha,
                             double beta, double* Y, int ldy, hipStream_t st) {
    if (n <= 0 || q <= 0) return hipSuccess;
    // in place only within one y-block (see k_combine_ts): with more than one
    // y-block any overlap of X's and Y's address ranges would race, exact
    // aliasing or a Y offset into X's block alike
    if (q > 32) {
        const char* x0 = reinterpret_cast<const char*>(X);
        const char* x1 = reinterpret_cast<const char*>(X + (n - 1) * (int64_t)ldx + px);
        const char* y0 = reinterpret_cast<const char*>(Y);
        const char* y1 = reinterpret_cast<const char*>(Y + (n - 1) * (int64_t)ldy + q);
        if (x0 < y1 && y0 < x1) return hipErrorInvalidValue;
    }
    dim3 grid((unsigned)((n + kCombRows - 1) / kCombRows), (q + 31) / 32);
    k_combine_ts<<<grid, 256, 0, st>>>(n, X, ldx, px, C, q, alpha, beta, Y, ldy);
    return hipGetLastError();
}

// The Frobenius norm^2 and the largest column norm^2 of the n x n
// column-major M into out[0], out[1], then M /= ||M||_F in place (the
// normalised repeated squaring of the fun_update stop test, kt_krylov.cpp).
// Two launches: one wave per column writes its squared norm (lanes down the
// column, coalesced); then every workgroup of the scaling launch reduces the
// n column norms itself in one fixed order (the same f and max everywhere:
// deterministic) and scales its slice.  (One workgroup doing both walked the
// matrix with a memory latency per element: 75 us at n = 225.)
__global__ __launch_bounds__(256) void k_colsq(int n, const double* __restrict__ M, double* __restrict__ colsq) {
    const int lane = threadIdx.x & 63;
    const int j = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (j >= n) return;
    const double* col = M + (int64_t)j * n;
    double c = 0.0;
    for (int i = lane; i < n; i += 64) c = fma(col[i], col[i], c);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    if (lane == 0) colsq[j] = c;
}

__global__ __launch_bounds__(256) void k_fro_scale(int n, double* __restrict__ M, const double* __restrict__ colsq,
                                                   double* __restrict__ out) {
    __shared__ double s_f;
    if (threadIdx.x < 64) {  // wave 0: lanes strided over the columns, then a fixed xor tree
        const int lane = threadIdx.x;
        double f = 0.0, m = 0.0;
        for (int j = lane; j < n; j += 64) {
            const double c = colsq[j];
            f += c;
            m = fmax(m, c);
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            f += __shfl_xor(f, o, 64);
            m = fmax(m, __shfl_xor(m, o, 64));
        }
        if (lane == 0) {
            s_f = f;
            if (blockIdx.x == 0) {
                out[0] = f;
                out[1] = m;
            }
        }
    }
    __syncthreads();
    const double f = s_f;
    if (!(f > 0.0)) return;
    const double inv = 1.0 / sqrt(f);
    const int64_t nn = (int64_t)n * n;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nn; t += (int64_t)gridDim.x * blockDim.x)
        M[t] *= inv;
}

hipError_t launch_fro_colmax_scale(int n, double* M, double* out, double* colsq, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    k_colsq<<<(n + 3) / 4, 256, 0, st>>>(n, M, colsq);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const int64_t nn = (int64_t)n * n;
    const int grid = (int)std::min<int64_t>(256, (nn + 256 * 4 - 1) / (256 * 4));
    k_fro_scale<<<grid, 256, 0, st>>>(n, M, colsq, out);
    return hipGetLastError();
}

// CholeskyQR on the device (kt_block.cpp shifted_cholqr3): one workgroup
// factors the bs x bs Gram G (column-major) as R' R, R upper, with
// shift_coef * trace(G) added to the diagonal, and inverts R; ok[0] = 0 when a
// pivot is not positive.  R and Rinv are column-major bs x bs (zero below the
// diagonal).  Right-looking: the same operations as the host chol_upper up to
// the order of the trailing updates.  bs <= 64 (LDS).
__global__ __launch_bounds__(256) void k_chol_rinv(int bs, const double* __restrict__ G, double shift_coef,
                                                   double* __restrict__ R, double* __restrict__ Rinv,
                                                   int* __restrict__ ok) {
    __shared__ double A[64 * 64];
    __shared__ double X[64 * 64];
    __shared__ double s_shift;
    __shared__ int s_ok;
    const int tid = threadIdx.x;
    for (int t = tid; t < bs * bs; t += blockDim.x) A[t] = G[t];
    __syncthreads();
    if (tid == 0) {
        double tr = 0.0;
        for (int i = 0; i < bs; ++i) tr += A[i + i * bs];
        s_shift = shift_coef * tr;
        s_ok = 1;
    }
    __syncthreads();
    for (int i = tid; i < bs; i += blockDim.x) A[i + i * bs] += s_shift;
    __syncthreads();
    for (int j = 0; j < bs; ++j) {
        if (tid == 0) {
            const double d = A[j + j * bs];
            if (!(d > 0.0)) s_ok = 0;
            A[j + j * bs] = sqrt(d > 0.0 ? d : 1.0);
        }
        __syncthreads();
        const double r = A[j + j * bs];
        for (int q = j + 1 + tid; q < bs; q += blockDim.x) A[j + q * bs] /= r;  // R(j, q)
        __syncthreads();
        const int m = bs - j - 1;  // trailing (p, q), j < p <= q
        for (int t = tid; t < m * m; t += blockDim.x) {
            const int p = j + 1 + t % m, q = j + 1 + t / m;
            if (p <= q) A[p + q * bs] -= A[j + p * bs] * A[j + q * bs];
        }
        __syncthreads();
    }
    // R out (zero below), then Rinv column by column (one thread per column)
    for (int t = tid; t < bs * bs; t += blockDim.x) {
        const int i = t % bs, q = t / bs;
        R[t] = i <= q ? A[t] : 0.0;
    }
    for (int t = tid; t < bs * bs; t += blockDim.x) X[t] = 0.0;
    __syncthreads();
    for (int c = tid; c < bs; c += blockDim.x) {  // back substitution R x = e_c, in LDS
        double* x = X + c * bs;
        x[c] = 1.0 / A[c + c * bs];
        for (int i = c - 1; i >= 0; --i) {
            double sm = 0.0;
            for (int k = i + 1; k <= c; ++k) sm = fma(A[i + k * bs], x[k], sm);
            x[i] = -sm / A[i + i * bs];
        }
    }
    __syncthreads();
    for (int t = tid; t < bs * bs; t += blockDim.x) Rinv[t] = X[t];
    if (tid == 0) ok[0] = s_ok;
}

hipError_t launch_chol_rinv(int bs, const double* G, double shift_coef, double* R, double* Rinv, int* ok,
                            hipStream_t st) {
    if (bs < 1 || bs > 64) return hipErrorInvalidValue;
    k_chol_rinv<<<1, 256, 0, st>>>(bs, G, shift_coef, R, Rinv, ok);
    return hipGetLastError();
}

}  // namespace kt

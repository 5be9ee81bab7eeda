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

// ---------------------------------------------------------------------------
// The reflector sweep as ONE persistent launch (k_ts_qr): workgroup g keeps
// its row slice of W in LDS for the whole factorisation and per column k runs
// k_ts_step's arithmetic on it (apply H_k, write v_k, accumulate the next
// column's sums); the per-column reduce launch becomes a grid barrier after
// which every workgroup sums the G per-workgroup partials itself, in
// workgroup order (the same sums, so the same coefficients, everywhere).
// Partials and the pivot row move write-through (sc1) and are read sc1, so
// the barrier needs no fences (cdna_hip_programming.md Guideline 16, R1).
// 2 bs launches -> 1; the reduction tree differs from the two-launch form's
// (per-workgroup slices of rpb rows, then G partials), i.e. rounding-level
// differences.  Only for n * BP * 8 small enough that the slices fit LDS.
// ---------------------------------------------------------------------------
struct TsBar {  // 128-B lines, zeroed before every launch
    unsigned grp[8][32];
    unsigned top[32];
    unsigned gen[8][32];
    unsigned tmo[32];
};
typedef __attribute__((address_space(1))) unsigned int ts_gu32;
typedef __attribute__((address_space(1))) unsigned long long ts_gu64;

__device__ __forceinline__ double ts_ld(const double* p) {
    return __longlong_as_double((long long)__hip_atomic_load((ts_gu64*)p, __ATOMIC_RELAXED,
                                                             __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ void ts_st(double* p, double v) {
    __hip_atomic_store((ts_gu64*)p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

// grid barrier (per-group counters -> top counter -> per-group generation
// words); every handed-off byte is sc1, so no release / acquire fences.
// Bounded spin: ~2 s, then tmo is raised and every waiter leaves.
__device__ __forceinline__ bool ts_grid_sync(TsBar* B, unsigned e, int G, int g) {
    __shared__ int s_ok;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
    __syncthreads();
    if (threadIdx.x == 0) {
        const int grp = g & 7;
        const int ngrp = G < 8 ? G : 8;
        const unsigned gsz = (unsigned)((G - grp + 7) / 8);
        const unsigned old = __hip_atomic_fetch_add((ts_gu32*)&B->grp[grp][0], 1u, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT);
        if (old == e * gsz - 1u) {
            const unsigned o2 = __hip_atomic_fetch_add((ts_gu32*)&B->top[0], 1u, __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT);
            if (o2 == e * (unsigned)ngrp - 1u)
                for (int q = 0; q < ngrp; ++q)
                    __hip_atomic_store((ts_gu32*)&B->gen[q][0], e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        int ok = 1;
        for (unsigned spins = 0;; ++spins) {
            if (__hip_atomic_load((ts_gu32*)&B->gen[grp][0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= e) break;
            if ((spins & 63u) == 63u &&
                __hip_atomic_load((ts_gu32*)&B->tmo[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                ok = 0;
                break;
            }
            if (spins > (1u << 22)) {
                __hip_atomic_store((ts_gu32*)&B->tmo[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                ok = 0;
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: loads stay below the poll
        s_ok = ok;
    }
    __syncthreads();
    return s_ok != 0;
}

// Workgroup g owns blocks [g bpw, (g+1) bpw) of the two-launch form's row
// blocks (rpb rows each, nrb in all) and keeps their rows in LDS.  Per column
// k: the update and each block's partial sums exactly as k_ts_step computes
// them (block by block) -> barrier -> workgroups 0 .. ceil((bs-kn)/4)-1 sum
// the partials one wave per column exactly as k_ts_reduce does -> barrier ->
// every workgroup reads the sums and the pivot row.  So every value equals
// the two-launch form's, bit for bit.
// pub: [2 slots][BP * nrb partials (column-major, as `part`) | BP sums | BP pivot]
__global__ __launch_bounds__(kTsBlock) void k_ts_qr(int n, int bs, int BP, int rpb, int nrb, int bpw,
                                                    double* __restrict__ W, int ld, double* __restrict__ V,
                                                    double* __restrict__ pub, double* __restrict__ taus,
                                                    TsBar* bar) {
    extern __shared__ double lw[];  // [rows of the workgroup's blocks][BP]
    __shared__ double red[kTsBlock];
    __shared__ double s_sums[128], s_piv[128];
    const int G = (int)gridDim.x, g = (int)blockIdx.x, tid = (int)threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int c = tid % BP, sub = tid / BP, rpi = kTsBlock / BP;
    const int b0 = g * bpw, b1 = min(nrb, b0 + bpw);
    const int r0 = min(n, b0 * rpb), r1 = min(n, b1 * rpb);
    const int nr = r1 - r0;
    const size_t slot_sz = (size_t)BP * nrb + 2 * BP;
    for (int t = tid; t < nr * BP; t += kTsBlock) {
        const int rr = t / BP, cc = t % BP;
        lw[t] = cc < bs ? W[(int64_t)(r0 + rr) * ld + cc] : 0.0;
    }
    __syncthreads();
    unsigned epoch = 0;
    bool ok = true;
    for (int k = -1; k < bs && ok; ++k) {
        const int kn = k + 1;
        double beta = 0.0, tau = 0.0, scal = 1.0, tc = 0.0, tn = 0.0;
        if (k >= 0) {  // as k_ts_step
            ts_larfg(s_piv[k], s_sums[k], beta, tau, scal);
            if (c > k && c < bs) tc = s_piv[c] + scal * s_sums[c];
            if (kn < bs) tn = s_piv[kn] + scal * s_sums[kn];
            if (g == 0 && tid == 0) taus[k] = tau;
        }
        double* slot = pub + (size_t)((epoch + 1) & 1) * slot_sz;
        for (int b = b0; b < b1; ++b) {  // k_ts_step's block b
            const int rb0 = b * rpb, rb1 = min(n, rb0 + rpb);
            const int rstart = max(rb0, k < 0 ? 0 : k);
            double acc = 0.0;
            for (int base = rstart; base < rb1; base += rpi) {  // uniform trip count (barrier inside)
                const int r = base + sub;
                const bool live = r < rb1 && c < bs;
                double* row = lw + (size_t)(r - r0) * BP;
                double wk = 0.0, wn = 0.0, wc = 0.0;
                if (live) {
                    if (k >= 0) wk = row[k];
                    if (kn < bs) wn = row[kn];
                    wc = row[c];
                }
                __syncthreads();  // every read of this row block before any write
                if (live) {
                    double v = 0.0;
                    if (k >= 0) {
                        v = (r == k) ? 1.0 : wk * scal;
                        if (c == k) {
                            V[(int64_t)r * BP + k] = v;
                            if (r == k) row[k] = beta;
                        } else if (c > k) {
                            wc -= tau * v * tc;
                            row[c] = wc;
                        }
                    }
                    if (kn < bs && c >= kn && r > kn) {
                        const double wn_new = k >= 0 ? wn - tau * v * tn : wn;
                        acc = fma(wn_new, wc, acc);
                    }
                }
            }
            if (kn < bs) {
                red[tid] = acc;
                __syncthreads();
                if (tid < BP) {
                    double s = 0.0;
                    for (int q = 0; q < rpi; ++q) s += red[q * BP + tid];
                    ts_st(slot + (size_t)tid * nrb + b, s);
                }
                __syncthreads();
            }
        }
        if (kn >= bs) break;
        if (kn >= r0 && kn < r1 && tid < BP)  // the next pivot row, W(kn, :) after H_k
            ts_st(slot + (size_t)BP * nrb + BP + tid, tid < bs ? lw[(size_t)(kn - r0) * BP + tid] : 0.0);
        ok = ts_grid_sync(bar, ++epoch, G, g);
        if (!ok) break;
        // k_ts_reduce: one wave per column j >= kn, lanes strided over the blocks
        {
            const int j = kn + g * 4 + wave;
            if (j < bs) {
                const double* p = slot + (size_t)j * nrb;
                double s = 0.0;
                for (int i = lane; i < nrb; i += 64) s += ts_ld(p + i);
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
                if (lane == 0) ts_st(slot + (size_t)BP * nrb + j, s);
            }
        }
        ok = ts_grid_sync(bar, ++epoch, G, g);
        if (!ok) break;
        if (tid < BP) {
            s_sums[tid] = (tid >= kn && tid < bs) ? ts_ld(slot + (size_t)BP * nrb + tid) : 0.0;
            s_piv[tid] = ts_ld(slot + (size_t)BP * nrb + BP + tid);
        }
        __syncthreads();
    }
    // R: rows 0..bs-1 of W back to memory (Q is formed from V afterwards)
    for (int t = tid; t < nr * BP; t += kTsBlock) {
        const int rr = t / BP, cc = t % BP;
        if (r0 + rr < bs && cc < bs) W[(int64_t)(r0 + rr) * ld + cc] = lw[t];
    }
}

size_t ts_qr_bar_bytes() { return sizeof(TsBar); }
size_t ts_qr_tmo_offset() { return offsetof(TsBar, tmo); }

// ---------------------------------------------------------------------------
// The persistent sweep with ONE grid barrier per column (k_ts_qr1,
// KT_TSQR_PERSIST=2): every workgroup keeps its row slice in LDS (1024
// threads), publishes one partial per column (its rows summed) and the next
// pivot row write-through (sc1), and after the barrier sums the G partials
// itself in one fixed order -- identical coefficients in every workgroup, no
// second barrier for a reduce.  Rounding-level differences from the
// two-launch form (reductions grouped by workgroup).
// pub: 2 slots x [BP x G partials | BP pivot].
// ---------------------------------------------------------------------------
constexpr int kTsQ1Block = 1024;
constexpr size_t kTsQ1Lds = 136 * 1024;  // the row slice; + 8 KB reduce + 2 KB coefficients

__global__ __launch_bounds__(kTsQ1Block) void k_ts_qr1(int n, int bs, int BP, int rpw, double* __restrict__ W, int ld,
                                                       double* __restrict__ V, double* __restrict__ pub,
                                                       double* __restrict__ taus, TsBar* bar) {
    extern __shared__ double lw[];  // [rows of this workgroup][BP]
    __shared__ double red[kTsQ1Block];
    __shared__ double s_sums[128], s_piv[128];
    const int G = (int)gridDim.x, g = (int)blockIdx.x, tid = (int)threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int c = tid % BP, sub = tid / BP, rpi = kTsQ1Block / BP;
    const int r0 = min(n, g * rpw), r1 = min(n, r0 + rpw);
    const int nr = r1 - r0;
    const size_t slot_sz = (size_t)BP * G + BP;
    for (int t = tid; t < nr * BP; t += kTsQ1Block) {
        const int rr = t / BP, cc = t % BP;
        lw[t] = cc < bs ? W[(int64_t)(r0 + rr) * ld + cc] : 0.0;
    }
    __syncthreads();
    unsigned epoch = 0;
    bool ok = true;
    for (int k = -1; k < bs && ok; ++k) {
        const int kn = k + 1;
        double beta = 0.0, tau = 0.0, scal = 1.0, tc = 0.0, tn = 0.0;
        if (k >= 0) {
            ts_larfg(s_piv[k], s_sums[k], beta, tau, scal);
            if (c > k && c < bs) tc = s_piv[c] + scal * s_sums[c];
            if (kn < bs) tn = s_piv[kn] + scal * s_sums[kn];
            if (g == 0 && tid == 0) taus[k] = tau;
        }
        double* slot = pub + (size_t)((epoch + 1) & 1) * slot_sz;
        const int rstart = max(r0, k < 0 ? 0 : k);
        double acc = 0.0;
        for (int base = rstart; base < r1; base += rpi) {  // uniform trip count (barrier inside)
            const int r = base + sub;
            const bool live = r < r1 && c < bs;
            double* row = lw + (size_t)(r - r0) * BP;
            double wk = 0.0, wn = 0.0, wc = 0.0;
            if (live) {
                if (k >= 0) wk = row[k];
                if (kn < bs) wn = row[kn];
                wc = row[c];
            }
            __syncthreads();  // every read of this row slot before any write
            if (live) {
                double v = 0.0;
                if (k >= 0) {
                    v = (r == k) ? 1.0 : wk * scal;
                    if (c == k) {
                        V[(int64_t)r * BP + k] = v;
                        if (r == k) row[k] = beta;
                    } else if (c > k) {
                        wc -= tau * v * tc;
                        row[c] = wc;
                    }
                }
                if (kn < bs && c >= kn && r > kn) {
                    const double wn_new = k >= 0 ? wn - tau * v * tn : wn;
                    acc = fma(wn_new, wc, acc);
                }
            }
        }
        if (kn >= bs) break;
        red[tid] = acc;
        __syncthreads();
        if (tid < BP) {
            double sm = 0.0;
            for (int q = 0; q < rpi; ++q) sm += red[q * BP + tid];
            ts_st(slot + (size_t)tid * G + g, sm);
        }
        if (kn >= r0 && kn < r1 && tid < BP)  // the next pivot row, W(kn, :) after H_k
            ts_st(slot + (size_t)BP * G + tid, tid < bs ? lw[(size_t)(kn - r0) * BP + tid] : 0.0);
        ok = ts_grid_sync(bar, ++epoch, G, g);
        if (!ok) break;
        // every workgroup: sums[j], j in [kn, bs), one wave per column, lanes
        // over the G partials, a fixed xor tree
        for (int j = kn + wave; j < bs; j += kTsQ1Block / 64) {
            double sm = 0.0;
            for (int i = lane; i < G; i += 64) sm += ts_ld(slot + (size_t)j * G + i);
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) sm += __shfl_xor(sm, o, 64);
            if (lane == 0) s_sums[j] = sm;
        }
        if (tid < BP) s_piv[tid] = ts_ld(slot + (size_t)BP * G + tid);
        __syncthreads();
    }
    // R: rows 0..bs-1 of W back to memory (Q is formed from V afterwards)
    for (int t = tid; t < nr * BP; t += kTsQ1Block) {
        const int rr = t / BP, cc = t % BP;
        if (r0 + rr < bs && cc < bs) W[(int64_t)(r0 + rr) * ld + cc] = lw[t];
    }
}

// grid of k_ts_qr1 (0 when it does not apply): rows per workgroup from the LDS
// budget, at most a quarter of the CUs (one workgroup per CU, co-resident
// next to another context's work)
int ts_qr1_grid(int n, int BP, int num_cu, int* rows_per_wg) {
    const int rpw_max = (int)(kTsQ1Lds / (sizeof(double) * (size_t)BP));
    int G = (n + rpw_max - 1) / rpw_max;
    const int floor_g = std::min(16, num_cu / 4);  // spread small problems over a few CUs
    G = std::max(G, std::min(floor_g, (n + 63) / 64));
    if (G < 1 || G > num_cu / 4 || BP > 128) return 0;
    *rows_per_wg = (n + G - 1) / G;
    if ((size_t)*rows_per_wg * BP * sizeof(double) > kTsQ1Lds) return 0;
    return G;
}

size_t ts_qr1_pub_doubles(int n, int BP, int num_cu) {
    int rpw = 0;
    const int G = ts_qr1_grid(n, BP, num_cu, &rpw);
    return 2 * ((size_t)BP * std::max(G, 1) + BP);
}

hipError_t launch_ts_qr1(int n, int bs, int BP, int num_cu, double* W, int ld, double* V, double* pub, double* taus,
                         void* bar, hipStream_t st) {
    int rpw = 0;
    const int G = ts_qr1_grid(n, BP, num_cu, &rpw);
    if (!G) return hipErrorInvalidValue;
    hipError_t e = hipMemsetAsync(bar, 0, sizeof(TsBar), st);
    if (e != hipSuccess) return e;
    k_ts_qr1<<<G, kTsQ1Block, sizeof(double) * (size_t)rpw * BP, st>>>(n, bs, BP, rpw, W, ld, V, pub, taus,
                                                                     static_cast<TsBar*>(bar));
    return hipGetLastError();
}

static int ts_rows_per_blk(int n, int num_cu);

// blocks per workgroup of the persistent sweep (the two-launch form's blocks,
// ~192 rows per workgroup), 0 when the rows would not fit LDS, the grid would
// not stay resident next to a twin context's run, or the reduce needs more
// workgroups than the grid has
static int ts_qr_bpw(int n, int BP, int num_cu, int* grid) {
    const int rpb = ts_rows_per_blk(n, num_cu);
    const int nrb = (n + rpb - 1) / rpb;
    const size_t lds_rows = (size_t)(144 * 1024) / (sizeof(double) * BP);
    if ((size_t)rpb > lds_rows) return 0;
    int bpw = (192 + rpb - 1) / rpb;
    if ((size_t)bpw * rpb > lds_rows) bpw = (int)(lds_rows / rpb);
    const int G = (nrb + bpw - 1) / bpw;
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessorWithFlags(&per_cu, k_ts_qr, kTsBlock,
                                                              sizeof(double) * (size_t)bpw * rpb * BP, 0) !=
            hipSuccess ||
        per_cu < 1 || G > per_cu * num_cu / 2 || 4 * G < BP)
        return 0;
    *grid = G;
    return bpw;
}

int ts_qr_grid(int n, int BP, int num_cu) {
    int G = 0;
    return ts_qr_bpw(n, BP, num_cu, &G) ? G : 0;
}

size_t ts_qr_pub_doubles(int n, int BP, int num_cu) {
    const int rpb = ts_rows_per_blk(n, num_cu);
    const int nrb = (n + rpb - 1) / rpb;
    return 2 * ((size_t)BP * nrb + 2 * BP);
}

hipError_t launch_ts_qr(int n, int bs, int BP, int num_cu, double* W, int ld, double* V, double* pub,
                        double* taus, void* bar, hipStream_t st) {
    int G = 0;
    const int bpw = ts_qr_bpw(n, BP, num_cu, &G);
    if (!bpw) return hipErrorInvalidValue;
    const int rpb = ts_rows_per_blk(n, num_cu);
    const int nrb = (n + rpb - 1) / rpb;
    hipError_t e = hipMemsetAsync(bar, 0, sizeof(TsBar), st);
    if (e != hipSuccess) return e;
    k_ts_qr<<<G, kTsBlock, sizeof(double) * (size_t)bpw * rpb * BP, st>>>(n, bs, BP, rpb, nrb, bpw, W, ld, V, pub,
                                                                         taus, static_cast<TsBar*>(bar));
    return hipGetLastError();
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

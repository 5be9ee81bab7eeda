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
    const double* __restrict__ coef, double* __restrict__ part) {
    constexpr int NV = PhaseNV<PH>::v;
    __shared__ double lds[NV > 0 ? NV * kSweepWaves * 64 : 1];
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

// sum of the nrb partials of (k, c): one wave, fixed order (lane-strided
// sums, then a fixed xor tree) -> identical result in every lane
__device__ __forceinline__ double wave_sum_part(const double* __restrict__ part, int C, int nrb,
                                                int k, int c) {
    const int lane = threadIdx.x & 63;
    const double* p = part + ((int64_t)k * C + c) * nrb;
    double s = 0.0;
    for (int i = lane; i < nrb; i += 64) s += p[i];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    return s;
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
                                                    double* __restrict__ hr) {
    const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (c >= C) return;
    double* cf = coef + (int64_t)c * CF_NCOEF;
    const int64_t off = 2 * (int64_t)c;
    if (PH == PH_A || PH == PH_B) {
        double v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = wave_sum_part(part, C, nrb, k, c);
        if (lane == 0) {
            const int base = PH == PH_A ? CF_G1 : CF_G2;
#pragma unroll
            for (int k = 0; k < 8; ++k) cf[base + k] = v[k];
        }
    } else if (PH == PH_C || PH == PH_C0) {
        const double s1 = wave_sum_part(part, C, nrb, 0, c);
        const double ab = wave_sum_part(part, C, nrb, 1, c);
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
        const double s2 = wave_sum_part(part, C, nrb, 0, c);
        const double dz = wave_sum_part(part, C, nrb, 1, c);
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
                             hipStream_t st) {
    if (C <= 0) return hipSuccess;
    int nrb, rpb;
    pairs_orth_geometry(n, C, num_cu, &nrb, &rpb);
    const dim3 grid((C + 63) / 64, nrb);
    const int cgrid = (C + 3) / 4;
    if (cur) {
        k_pairs_sweep<PH_A><<<grid, kSweepBlock, 0, st>>>(n, C, rpb, prev, cur, W, ld, coef, part);
        k_pairs_coef<PH_A><<<cgrid, 256, 0, st>>>(C, nrb, part, W, ld, coef, hr);
        k_pairs_sweep<PH_B><<<grid, kSweepBlock, 0, st>>>(n, C, rpb, prev, cur, W, ld, coef, part);
        k_pairs_coef<PH_B><<<cgrid, 256, 0, st>>>(C, nrb, part, W, ld, coef, hr);
        k_pairs_sweep<PH_C><<<grid, kSweepBlock, 0, st>>>(n, C, rpb, prev, cur, W, ld, coef, part);
        k_pairs_coef<PH_C><<<cgrid, 256, 0, st>>>(C, nrb, part, W, ld, coef, hr);
    } else {
        k_pairs_sweep<PH_C0><<<grid, kSweepBlock, 0, st>>>(n, C, rpb, nullptr, nullptr, W, ld, coef, part);
        k_pairs_coef<PH_C0><<<cgrid, 256, 0, st>>>(C, nrb, part, W, ld, coef, hr);
    }
    k_pairs_sweep<PH_D><<<grid, kSweepBlock, 0, st>>>(n, C, rpb, nullptr, nullptr, W, ld, coef, part);
    k_pairs_coef<PH_D><<<cgrid, 256, 0, st>>>(C, nrb, part, W, ld, coef, hr);
    k_pairs_sweep<PH_E><<<grid, kSweepBlock, 0, st>>>(n, C, rpb, nullptr, nullptr, W, ld, coef, part);
    return hipGetLastError();
}

}  // namespace kt

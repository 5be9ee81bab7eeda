// kt_kernels.hip -- CDNA4 (gfx950) kernels for the probe-Lanczos trace path.
//
// Data layout in HBM:
//   A      : CSR, int32 row_ptr[n+1], int32 col[nnz], fp64 val[nnz]; rows
//            relabelled by descending degree (kt_runtime.cpp), hub rows first.
//   blocks : n x P fp64, ROW-MAJOR ("probe-contiguous"): row i of a probe
//            block is P consecutive doubles, so every nonzero a_ic gathers
//            one contiguous 8P-byte row X[c, 0:P] -- a coalesced 16 B/lane
//            load by P/2 lanes.
//
// Wave mapping: a wave64 is split into GPW = 64/LPR "row groups" of
// LPR = P/2 lanes; each group owns one matrix row, each lane two probe
// columns.  P = 128 -> one row per wave (1 KiB gathers); P = 16 -> 8 rows
// per wave (128 B gathers = one cache line).  Rows with degree > 64 are
// instead owned by a whole wave whose groups stride over the nonzeros.
//
// Recurrence (lanczos_krylov.m:73-115 with bs = 1
// per probe column).  Stored vectors are UNNORMALISED, u_j, with a per-probe
// scale s_j (v_j = s_j u_j), so 1/beta is applied inside the next SpMM.
//   K1 spmm_dot  : y = s_j A u_j;             partial  v_j . y
//   coef         : CGS2 against the window [v_{j-1}, v_j] from the Gram
//                  (two classical passes, lanczos_krylov.m:109-115, formed
//                  algebraically: c = 2h - G h)
//   K2 update    : u_{j+1} = y - c0 v_{j-1} - c1 v_j (over u_{j-1});
//                  partials ||u_{j+1}||^2, y . u_{j+1}, u_j . u_{j+1}
//   norm         : beta = ||u_{j+1}||, s_{j+1} = 1/beta (lucky if < 1e-8)
// By the symmetry of A, v_j . (A v_{j+1}) = (A v_j) . v_{j+1}: the K2 dot
// y . u_{j+1} supplies next step's window coefficient, so K1 never reads
// v_{j-1} (48 B of vector traffic per probe-row-step instead of 56).
// All reductions are deterministic: per-block partial slabs summed in a fixed
// order by column-reduction kernels (no float atomics).
#include <hip/hip_runtime.h>

#include "kt_launch.h"
#include "kt_wave.h"
#include <stdint.h>

#include <cstdlib>

#include <type_traits>

namespace kt {

__device__ __forceinline__ uint64_t sm64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

// Lane geometry of a P-wide row-major block: VW doubles per lane, LPR lanes
// per row group, GPW row groups per wave.
template <int P, int VW> struct GeoW {
    static constexpr int VEC = VW;       // doubles per lane
    static constexpr int LPR = P / VEC;  // lanes per row group
    static constexpr int GPW = 64 / LPR; // row groups per wave
};
// streaming kernels and the block SpMM: 16 B per lane
template <int P> using Geo = GeoW<P, (P >= 2) ? 2 : 1>;
// K1: 32 B per lane from P = 16 on -- a 128-B probe row is 4 lanes, 16 rows
// in flight per wave (K1 -4 %, profiles/r01_sweep_vec4.txt; K2 is faster
// with 16 B per lane and keeps Geo)
#ifndef KT_K1_VW
#define KT_K1_VW 4
#endif
template <int P> using GeoK1 = GeoW<P, (P >= 16) ? (KT_K1_VW < P ? KT_K1_VW : P) : (P >= 2) ? 2 : 1>;
// y-form passes (start + step): 16 B per lane, 8 lanes per 128-B probe row.
// 72 VGPRs = 3 workgroups of 512 per CU vs 118 VGPRs = 2 with 32 B per lane:
// +1.4 % evals/s with two sweep lanes (profiles/r02_ab_occupancy.txt); 4 per
// CU (64 VGPRs) is 10 % slower -- more rows in flight thrash the L2.
#ifndef KT_KY_VW
#define KT_KY_VW 2
#endif
template <int P> using GeoKY = GeoW<P, (P >= 16) ? (KT_KY_VW < P ? KT_KY_VW : P) : (P >= 2) ? 2 : 1>;
// block SpMM lane width (doubles per lane) from P = 16 on
#ifndef KT_BLK_VW
#define KT_BLK_VW 2
#endif
template <int P> using GeoB = GeoW<P, (P >= 16) ? KT_BLK_VW : (P >= 2) ? 2 : 1>;

// FLAGS bit 1: unit-weight adjacency (every stored value is 1.0, detected at
// matrix creation): the values array is never read (4 B per nonzero instead
// of 12).
// FLAGS bit 2: deep gather issue -- up to 8 column indices, then up to 8 row
// gathers in flight per row group per round trip (predicated tails, no
// serial remainder loop), for graphs whose rows are mostly short.
// FLAGS bit 0: the CSR index/value streams are loaded nontemporal (read once
// per launch; keeps L2/MALL for the gathered rows).  Bit 3: y is stored
// nontemporal.  The own-row load of u_cur is always a normal load (it is the
// gathered table).
// FLAGS bit 4 (y-form passes): y_{j+1} is stored write-through (buffer store
// with sc1), which drops the line from the XCD's L2 instead of keeping it
// (MI355X_MICROARCH.md: plain / nt stores keep the line), leaving L2 to the
// gathered table.
// FLAGS bit 5 (expmv terms): mu = 0 (no self loops: trace(A) = 0), so a row's
// own b is never read and (A - mu I) b is A b.
// FLAGS bit 6 (y-form passes): also form the Lanczos vector v_{j+1} (the
// basis of f(A) x = ||x|| V f(T) e1) from the pass's own rows.
enum : int { KF_NT = 1, KF_UNIT = 2, KF_MLP = 4, KF_NTY = 8, KF_SC1 = 16, KF_MU0 = 32, KF_VB = 64 };

// KT_KY_DIAG (diagnostic builds of the y-form pass only, tools/ky_diag.sh; their
// results are wrong): 1 = gathers + own row, 2 = gathers only, 3 = row streams only
#ifndef KT_KY_DIAG
#define KT_KY_DIAG 0
#endif

typedef unsigned int kt_u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int kt_u32x2 __attribute__((ext_vector_type(2)));
// VEC doubles of one lane at byte offset `boff` of the buffer, sc1 (write-through)
template <int VEC>
__device__ __forceinline__ void store_sc1(__amdgpu_buffer_rsrc_t r, uint32_t boff, const double* v) {
#pragma unroll
    for (int e = 0; e + 1 < VEC; e += 2) {
        const double2 d = make_double2(v[e], v[e + 1]);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(kt_u32x4, d), r, boff + 8 * e, 0, 16);
    }
    if constexpr (VEC & 1) {
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(kt_u32x2, v[VEC - 1]), r,
                                              boff + 8 * (VEC - 1), 0, 16);
    }
}

template <int VEC> struct VecT;
template <> struct VecT<1> {
    using T = double;
    __device__ static __forceinline__ T load(const double* p) { return *p; }
    __device__ static __forceinline__ T load_nt(const double* p) {
        return __builtin_nontemporal_load(p);
    }
    __device__ static __forceinline__ void store(double* p, const T& v) { *p = v; }
    __device__ static __forceinline__ void store_nt(double* p, const T& v) {
        __builtin_nontemporal_store(v, p);
    }
    __device__ static __forceinline__ double get(const T& v, int) { return v; }
};
template <> struct VecT<2> {
    using T = double2;
    using N = __attribute__((ext_vector_type(2))) double;
    __device__ static __forceinline__ T load(const double* p) {
        return *reinterpret_cast<const double2*>(p);
    }
    __device__ static __forceinline__ T load_nt(const double* p) {
        const N v = __builtin_nontemporal_load(reinterpret_cast<const N*>(p));
        return double2(v[0], v[1]);
    }
    __device__ static __forceinline__ void store(double* p, const T& v) {
        *reinterpret_cast<double2*>(p) = v;
    }
    __device__ static __forceinline__ void store_nt(double* p, const T& v) {
        N w = {v.x, v.y};
        __builtin_nontemporal_store(w, reinterpret_cast<N*>(p));
    }
    __device__ static __forceinline__ double get(const T& v, int e) { return e ? v.y : v.x; }
};

struct Dbl4 {
    double2 a, b;
};
template <> struct VecT<4> {
    using T = Dbl4;
    __device__ static __forceinline__ T load(const double* p) {
        const double2* q = reinterpret_cast<const double2*>(p);
        return Dbl4{q[0], q[1]};
    }
    __device__ static __forceinline__ T load_nt(const double* p) {
        return Dbl4{VecT<2>::load_nt(p), VecT<2>::load_nt(p + 2)};
    }
    __device__ static __forceinline__ void store(double* p, const T& v) {
        double2* q = reinterpret_cast<double2*>(p);
        q[0] = v.a;
        q[1] = v.b;
    }
    __device__ static __forceinline__ void store_nt(double* p, const T& v) {
        VecT<2>::store_nt(p, v.a);
        VecT<2>::store_nt(p + 2, v.b);
    }
    __device__ static __forceinline__ double get(const T& v, int e) {
        return e == 0 ? v.a.x : e == 1 ? v.a.y : e == 2 ? v.b.x : v.b.y;
    }
};

struct Dbl8 {
    Dbl4 a, b;
};
template <> struct VecT<8> {
    using T = Dbl8;
    __device__ static __forceinline__ T load(const double* p) {
        return Dbl8{VecT<4>::load(p), VecT<4>::load(p + 4)};
    }
    __device__ static __forceinline__ T load_nt(const double* p) {
        return Dbl8{VecT<4>::load_nt(p), VecT<4>::load_nt(p + 4)};
    }
    __device__ static __forceinline__ void store(double* p, const T& v) {
        VecT<4>::store(p, v.a);
        VecT<4>::store(p + 4, v.b);
    }
    __device__ static __forceinline__ void store_nt(double* p, const T& v) {
        VecT<4>::store_nt(p, v.a);
        VecT<4>::store_nt(p + 4, v.b);
    }
    __device__ static __forceinline__ double get(const T& v, int e) {
        return e < 4 ? VecT<4>::get(v.a, e) : VecT<4>::get(v.b, e - 4);
    }
};

template <int FLAGS, class T> __device__ __forceinline__ T ld_stream(const T* p) {
    if constexpr (FLAGS & KF_NT) return __builtin_nontemporal_load(p);
    else return *p;
}

// VEC doubles of the gathered block
template <int FLAGS, int VEC>
__device__ __forceinline__ typename VecT<VEC>::T ld_gather(const double* p) {
    return VecT<VEC>::load(p);
}

// ---------------------------------------------------------------------------
// Rademacher probe block: X[r, p] = +-1 from splitmix64(key(seed, base+p) + i),
// i = perm[r] the ORIGINAL row index (oracle/krylov_oracle.py:rademacher,
// oracle/slq_ref.c produce the same stream).
// ---------------------------------------------------------------------------
template <int P>
__global__ __launch_bounds__(256) void k_rademacher(int n, uint64_t seed, int64_t probe_base,
                                                    const int* __restrict__ perm,
                                                    double* __restrict__ X) {
    __shared__ uint64_t keys[P];
    for (int p = threadIdx.x; p < P; p += blockDim.x)
        keys[p] = sm64(sm64(seed) + (uint64_t)(probe_base + p));
    __syncthreads();
    const int64_t total = (int64_t)n * P;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = t / P;
        const int p = (int)(t % P);
        const uint64_t i = perm ? (uint64_t)perm[r] : (uint64_t)r;
        X[t] = (sm64(keys[p] + i) >> 63) ? -1.0 : 1.0;
    }
}

// The same probes written as ncols (<= 64) columns of a wider row-major block
// (X[r * ldx + c] = probe probe_base + c of row r, natural row order): the
// Rademacher columns of mc_trace.m:43-44 straight into their slots of the
// round's probe block, without a staging block and a strided copy.
__global__ __launch_bounds__(256) void k_rademacher_cols(int n, int ncols, uint64_t seed, int64_t probe_base,
                                                         double* __restrict__ X, int ldx) {
    __shared__ uint64_t keys[64];
    for (int p = threadIdx.x; p < ncols; p += blockDim.x) keys[p] = sm64(sm64(seed) + (uint64_t)(probe_base + p));
    __syncthreads();
    const int64_t total = (int64_t)n * ncols;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = t / ncols;
        const int p = (int)(t % ncols);
        X[r * ldx + p] = (sm64(keys[p] + (uint64_t)r) >> 63) ? -1.0 : 1.0;
    }
}

// Packed form of the same probe block for the y-form start pass: bit p of
// S[r * W + p / 32] (W = ceil(P / 32) words per row) is set where X[r, p] = -1.
// n x 4W bytes (2 MB at n = 1M, P = 16) instead of the 8nP-byte fp64 block.
template <int P>
__global__ __launch_bounds__(256) void k_rademacher_signs(int n, uint64_t seed, int64_t probe_base,
                                                          const int* __restrict__ perm,
                                                          uint32_t* __restrict__ S) {
    constexpr int W = (P + 31) / 32;
    __shared__ uint64_t keys[P];
    for (int p = threadIdx.x; p < P; p += blockDim.x)
        keys[p] = sm64(sm64(seed) + (uint64_t)(probe_base + p));
    __syncthreads();
    const int64_t total = (int64_t)n * W;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = t / W;
        const int w = (int)(t % W);
        const uint64_t i = perm ? (uint64_t)perm[r] : (uint64_t)r;
        uint32_t bits = 0;
        for (int b = 0; b < 32 && w * 32 + b < P; ++b)
            bits |= (uint32_t)(sm64(keys[w * 32 + b] + i) >> 63) << b;
        S[t] = bits;
    }
}

// ---------------------------------------------------------------------------
// K1
// ---------------------------------------------------------------------------
// Gather-accumulate nonzeros k = k0, k0 + stride, ... < end of one row.
template <int P, int FLAGS, class G = Geo<P>>
__device__ __forceinline__ void row_gather(int k0, int end, int stride, int p0,
                                           const int* __restrict__ col,
                                           const double* __restrict__ val,
                                           const double* __restrict__ ucur, double* s,
                                           int ld = P) {
    using V = VecT<G::VEC>;
    int k = k0;
    for (; k + 3 * stride < end; k += 4 * stride) {  // 4 independent gathers in flight
        const int c0 = ld_stream<FLAGS>(col + k), c1 = ld_stream<FLAGS>(col + k + stride);
        const int c2 = ld_stream<FLAGS>(col + k + 2 * stride);
        const int c3 = ld_stream<FLAGS>(col + k + 3 * stride);
        double a0 = 1.0, a1 = 1.0, a2 = 1.0, a3 = 1.0;
        if constexpr (!(FLAGS & KF_UNIT)) {
            a0 = ld_stream<FLAGS>(val + k);
            a1 = ld_stream<FLAGS>(val + k + stride);
            a2 = ld_stream<FLAGS>(val + k + 2 * stride);
            a3 = ld_stream<FLAGS>(val + k + 3 * stride);
        }
        const typename V::T x0 = V::load(ucur + (int64_t)c0 * ld + p0);
        const typename V::T x1 = V::load(ucur + (int64_t)c1 * ld + p0);
        const typename V::T x2 = V::load(ucur + (int64_t)c2 * ld + p0);
        const typename V::T x3 = V::load(ucur + (int64_t)c3 * ld + p0);
#pragma unroll
        for (int e = 0; e < G::VEC; ++e) {
            s[e] = fma(a0, V::get(x0, e), s[e]);
            s[e] = fma(a1, V::get(x1, e), s[e]);
            s[e] = fma(a2, V::get(x2, e), s[e]);
            s[e] = fma(a3, V::get(x3, e), s[e]);
        }
    }
    for (; k < end; k += stride) {
        const int c0 = ld_stream<FLAGS>(col + k);
        double a0 = 1.0;
        if constexpr (!(FLAGS & KF_UNIT)) a0 = ld_stream<FLAGS>(val + k);
        const typename V::T x0 = V::load(ucur + (int64_t)c0 * ld + p0);
#pragma unroll
        for (int e = 0; e < G::VEC; ++e) s[e] = fma(a0, V::get(x0, e), s[e]);
    }
}

// Same sum as row_gather, issued D deep (default 8): the D column indices of
// a chunk are loaded together, then the D row gathers (a tail entry re-reads
// the chunk's first row with weight 0, so no lane branches), then the D FMAs.
template <int P, int FLAGS, class G = Geo<P>, int D = 8>
__device__ __forceinline__ void row_gather8(int k0, int end, int stride, int p0,
                                            const int* __restrict__ col,
                                            const double* __restrict__ val,
                                            const double* __restrict__ ucur, double* s,
                                            int ld = P) {
    using V = VecT<G::VEC>;
    for (int k = k0; k < end; k += D * stride) {
        int c[D];
        double a[D];
        const int c0 = ld_stream<FLAGS>(col + k);
        c[0] = c0;
        a[0] = (FLAGS & KF_UNIT) ? 1.0 : ld_stream<FLAGS>(val + k);
#pragma unroll
        for (int i = 1; i < D; ++i) {
            const int idx = k + i * stride;
            const bool ok = idx < end;
            c[i] = ok ? ld_stream<FLAGS>(col + idx) : c0;
            if constexpr (FLAGS & KF_UNIT) a[i] = ok ? 1.0 : 0.0;
            else a[i] = ok ? ld_stream<FLAGS>(val + idx) : 0.0;
        }
        typename V::T x[D];
#pragma unroll
        for (int i = 0; i < D; ++i) x[i] = ld_gather<FLAGS, G::VEC>(ucur + (int64_t)c[i] * ld + p0);
#pragma unroll
        for (int i = 0; i < D; ++i)
#pragma unroll
            for (int e = 0; e < G::VEC; ++e) s[e] = fma(a[i], V::get(x[i], e), s[e]);
    }
}

template <int P, int FLAGS, class G = Geo<P>>
__device__ __forceinline__ void gather_row(int k0, int end, int stride, int p0,
                                           const int* __restrict__ col,
                                           const double* __restrict__ val,
                                           const double* __restrict__ ucur, double* s,
                                           int ld = P) {
    if constexpr (FLAGS & KF_MLP) row_gather8<P, FLAGS, G>(k0, end, stride, p0, col, val, ucur, s, ld);
    else row_gather<P, FLAGS, G>(k0, end, stride, p0, col, val, ucur, s, ld);
}

// y_r = s_cur * sum; accumulate v_cur . y.
template <int P, int FLAGS, class G = Geo<P>>
__device__ __forceinline__ void row_epilogue(int row, int p0, const double* s, const double* sc,
                                             const double* __restrict__ ucur,
                                             double* __restrict__ y, double* acc) {
    using V = VecT<G::VEC>;
    const int64_t off = (int64_t)row * P + p0;
    const typename V::T ui = V::load(ucur + off);
    typename V::T yo;
    double* yp = reinterpret_cast<double*>(&yo);
#pragma unroll
    for (int e = 0; e < G::VEC; ++e) {
        const double yv = s[e] * sc[e];
        yp[e] = yv;
        acc[e] = fma(V::get(ui, e) * sc[e], yv, acc[e]);
    }
    if constexpr (FLAGS & KF_NTY) V::store_nt(y + off, yo);
    else V::store(y + off, yo);
}

// Two modes in one launch.  Blocks [0, long_blocks): one WAVE per long row
// (degree > long_thresh, listed heaviest first), its row groups striding over
// the row's nonzeros and combining by wave shuffles.  Other blocks: one row
// GROUP per short row, rows in order (coalesced y).  partial: [grid][P].
template <int P, int BLOCK, int FLAGS>
__global__ __launch_bounds__(BLOCK) void k_spmm_dot(
    const int* __restrict__ row_ptr, const int* __restrict__ col, const double* __restrict__ val,
    int n, const double* __restrict__ ucur, const double* __restrict__ scale_cur,
    double* __restrict__ y, double* __restrict__ partial, const int* __restrict__ long_rows,
    int n_long, int long_thresh, int long_blocks) {
    using G = GeoK1<P>;
    constexpr int WAVES = BLOCK / 64;
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int sub = lane % G::LPR;
    const int grp = lane / G::LPR;
    const int p0 = sub * G::VEC;

    double sc[G::VEC], acc[G::VEC];
#pragma unroll
    for (int e = 0; e < G::VEC; ++e) {
        sc[e] = scale_cur[p0 + e];
        acc[e] = 0.0;
    }

    if ((int)blockIdx.x < long_blocks) {
        for (int li = blockIdx.x * WAVES + wave; li < n_long; li += long_blocks * WAVES) {
            const int row = long_rows[li];
            const int beg = row_ptr[row];
            const int end = row_ptr[row + 1];
            double s[G::VEC];
#pragma unroll
            for (int e = 0; e < G::VEC; ++e) s[e] = 0.0;
            gather_row<P, FLAGS, G>(beg + grp, end, G::GPW, p0, col, val, ucur, s);
#pragma unroll
            for (int o = G::LPR; o < 64; o <<= 1)
#pragma unroll
                for (int e = 0; e < G::VEC; ++e) s[e] += kt::shfl_xor(s[e], o);
            if (grp == 0) row_epilogue<P, FLAGS, G>(row, p0, s, sc, ucur, y, acc);
        }
    } else {
        const int sb = blockIdx.x - long_blocks;
        const int groups_total = (gridDim.x - long_blocks) * WAVES * G::GPW;
        for (int row = (sb * WAVES + wave) * G::GPW + grp; row < n; row += groups_total) {
            const int beg = ld_stream<FLAGS>(row_ptr + row);
            const int end = ld_stream<FLAGS>(row_ptr + row + 1);
            if (end - beg > long_thresh) continue;  // owned by a long-row wave
            double s[G::VEC];
#pragma unroll
            for (int e = 0; e < G::VEC; ++e) s[e] = 0.0;
            gather_row<P, FLAGS, G>(beg, end, 1, p0, col, val, ucur, s);
            row_epilogue<P, FLAGS, G>(row, p0, s, sc, ucur, y, acc);
        }
    }

    // reduce over the row groups of this wave (lanes sharing `sub`), then waves
#pragma unroll
    for (int o = G::LPR; o < 64; o <<= 1)
#pragma unroll
        for (int e = 0; e < G::VEC; ++e) acc[e] += kt::shfl_xor(acc[e], o);
    __shared__ double red[WAVES][P];
    if (grp == 0) {
#pragma unroll
        for (int e = 0; e < G::VEC; ++e) red[wave][p0 + e] = acc[e];
    }
    __syncthreads();
    for (int t = threadIdx.x; t < P; t += BLOCK) {
        double v = 0.0;
#pragma unroll
        for (int w = 0; w < WAVES; ++w) v += red[w][t];
        partial[(int64_t)t * gridDim.x + blockIdx.x] = v;  // slot-major [P][grid]
    }
}

// One probe's coefficient step from the pass's three sums d0 = X.t,
// d1 = X.Out, d2 = Out.Out.
__device__ __forceinline__ void ycoef_probe(int p, int P, double d0, double d1, double d2, int start,
                                            int last, double s0, double* __restrict__ ys,
                                            double* __restrict__ t_alpha, double* __restrict__ t_up,
                                            double* __restrict__ t_low, double* __restrict__ guard) {
    double an, bn, bnext_sq, ny2, g = 1.0;
    if (start) {
        an = d1 * s0;  // v_0 . y_0 with v_0 = s0 z
        ny2 = d2;
        bn = 0.0;      // beta_0
        bnext_sq = ny2 - an * an;
        ys[1 * P + p] = 0.0;
        ys[2 * P + p] = 0.0;
        ys[4 * P + p] = 0.0;
        guard[p] = 1.0;
    } else {
        const double aj = ys[0 * P + p], bj = ys[1 * P + p], am1 = ys[2 * P + p];
        const double nyj = ys[3 * P + p], ydj = ys[4 * P + p], b1 = ys[5 * P + p];
        g = guard[p];
        const double b1sq = b1 * b1;
        an = (d0 - 2.0 * aj * nyj - 2.0 * bj * ydj + aj * aj * aj + 2.0 * aj * bj * bj + bj * bj * am1) /
             b1sq;
        ny2 = d2;
        bn = b1;
        bnext_sq = ny2 - an * an - b1sq;
        ys[1 * P + p] = b1;
        ys[2 * P + p] = aj;
        ys[4 * P + p] = d1;
    }
    const double bnext = sqrt(fmax(bnext_sq, 0.0));
    ys[0 * P + p] = an;
    ys[3 * P + p] = ny2;
    ys[5 * P + p] = bnext;
    t_alpha[p] = an;
    t_up[p] = bn;
    t_low[p] = bnext;
    if (!last) {
        const double ratio = bnext_sq / ny2;
        guard[p] = (ratio < g || !(ratio == ratio)) ? ratio : g;  // NaN sticks
    }
    const bool ok = bnext > 0.0 && bnext < INFINITY;
    const double inv = ok ? 1.0 / bnext : 0.0;
    ys[6 * P + p] = inv;
    ys[7 * P + p] = an * inv;
    ys[8 * P + p] = bn * inv;
}

// ---------------------------------------------------------------------------
// KY: the A-image ("y-form") probe Lanczos step -- the whole step in ONE
// streaming pass (no K2).  With y_j = A v_j the three-term recurrence
//   beta_{j+1} v_{j+1} = A v_j - alpha_j v_j - beta_j v_{j-1}
// multiplied by A gives
//   y_{j+1} = (A y_j - alpha_j y_j - beta_j y_{j-1}) / beta_{j+1},
// and every coefficient follows from three dots of this pass (symmetry of A,
// see k_ycoef): the v_j are never formed.  The kernel gathers X = y_j,
// reads the own rows X[r], Yold[r] = y_{j-1}[r] (dead after this pass: NT)
// and writes Out[r] = g t_r - a X[r] - b Yold[r] in place over Yold, with
// per-probe (g, a, b) = (1, alpha_j, beta_j) / beta_{j+1}.  Start mode
// (has_old = 0): X = the probe block z, (g, a, b) = (1/||z||, 0, 0), Out =
// y_0 = A v_0.  partial slabs [3][P][grid]: X.t, X.Out, Out.Out.  Out ==
// nullptr (the last pass of a sweep): only X.t is formed -- Yold is not read
// and nothing is stored.
// KF_VB (round 6): the pass also forms the normalised Lanczos vector
//   v_{j+1} = g y_j - a v_j - b v_{j-1}
// with the SAME per-probe (g, a, b): y_i = A v_i for every i (v_0 is the start
// table, y_0 = A v_0), so A applied to the right side is y_{j+1}'s
// recurrence.  y_j[r] is the own row already loaded for alpha; v_j[r] and
// v_{j-1}[r] are read from basis slots Vc, Vo (Vo == nullptr at j = 0) and
// v_{j+1}[r] is written to slot Vn, columns < bcols only -- also in the last
// pass, which still owes v_{m-1}.  No extra gathers: +24 n bcols bytes per
// pass where the explicit sweep's K1 + K2 move 32 n P more.
// ---------------------------------------------------------------------------
template <int P, int FLAGS, class G = Geo<P>, class C = const double*>
__device__ __forceinline__ void row_epilogue_y(int row, int p0, const double* s, C cg,
                                               C ca, C cb, bool has_old,
                                               const double* __restrict__ X,
                                               const double* __restrict__ Yold,
                                               double* __restrict__ Out, double* d0, double* d1,
                                               double* d2, __amdgpu_buffer_rsrc_t orsrc,
                                               const double* __restrict__ Vc = nullptr,
                                               const double* __restrict__ Vo = nullptr,
                                               double* __restrict__ Vn = nullptr, int bcols = 0) {
    using V = VecT<G::VEC>;
    const int64_t off = (int64_t)row * P + p0;
#if KT_KY_DIAG == 2
    // diagnostic build (tools/ky_diag.sh): gathers only -- no own-row read, no
    // y_{j-1} read, no y_{j+1} store; the dots keep the gathered sums live
#pragma unroll
    for (int e = 0; e < G::VEC; ++e) d0[e] = fma(s[e], s[e], d0[e]);
    return;
#endif
    const typename V::T xi = V::load(X + off);
    if constexpr (FLAGS & KF_VB) {
        if (p0 < bcols) {
            const typename V::T vc = V::load(Vc + off);
            typename V::T vo;
            if (Vo) vo = V::load(Vo + off);
#pragma unroll
            for (int e = 0; e < G::VEC; ++e) {
                double v = fma(-ca[e], V::get(vc, e), cg[e] * V::get(xi, e));
                if (Vo) v = fma(-cb[e], V::get(vo, e), v);
                if (p0 + e < bcols) Vn[off + e] = v;
            }
        }
    }
#if KT_KY_DIAG == 1
    // diagnostic build: gathers + the own-row read (alpha's y_j . t), no
    // y_{j-1} read and no y_{j+1} store
#pragma unroll
    for (int e = 0; e < G::VEC; ++e) d0[e] = fma(V::get(xi, e), s[e], d0[e]);
    return;
#endif
    if (!Out) {  // last pass: only alpha (X.t) is still needed
#pragma unroll
        for (int e = 0; e < G::VEC; ++e) d0[e] = fma(V::get(xi, e), s[e], d0[e]);
        return;
    }
    typename V::T yo;
    if (has_old) yo = V::load_nt(Yold + off);
    typename V::T o;
    double* op = reinterpret_cast<double*>(&o);
#pragma unroll
    for (int e = 0; e < G::VEC; ++e) {
        const double x = V::get(xi, e);
        double u = fma(-ca[e], x, cg[e] * s[e]);
        if (has_old) u = fma(-cb[e], V::get(yo, e), u);
        op[e] = u;
        d0[e] = fma(x, s[e], d0[e]);
        d1[e] = fma(x, u, d1[e]);
        d2[e] = fma(u, u, d2[e]);
    }
    if constexpr (FLAGS & KF_SC1) store_sc1<G::VEC>(orsrc, (uint32_t)(off * 8), op);
    else if constexpr (FLAGS & KF_NTY) V::store_nt(Out + off, o);
    else V::store(Out + off, o);
}

// Start-pass gather from the packed sign table: the lane's VEC probe bits of
// column c are one 4-byte load (VEC <= 32, VEC | 32).
template <int P, class G>
__device__ __forceinline__ double sign_of(uint32_t w, int p0, int e) {
    return ((w >> ((p0 + e) & 31)) & 1u) ? -1.0 : 1.0;
}
template <int P, int FLAGS, class G>
__device__ __forceinline__ void row_gather_signs(int k0, int end, int stride, int p0,
                                                 const int* __restrict__ col,
                                                 const double* __restrict__ val,
                                                 const uint32_t* __restrict__ S, double* s) {
    constexpr int W = (P + 31) / 32;
    const int wo = p0 >> 5;
    int k = k0;
    for (; k + 3 * stride < end; k += 4 * stride) {
        const int c0 = ld_stream<FLAGS>(col + k), c1 = ld_stream<FLAGS>(col + k + stride);
        const int c2 = ld_stream<FLAGS>(col + k + 2 * stride);
        const int c3 = ld_stream<FLAGS>(col + k + 3 * stride);
        double a0 = 1.0, a1 = 1.0, a2 = 1.0, a3 = 1.0;
        if constexpr (!(FLAGS & KF_UNIT)) {
            a0 = ld_stream<FLAGS>(val + k);
            a1 = ld_stream<FLAGS>(val + k + stride);
            a2 = ld_stream<FLAGS>(val + k + 2 * stride);
            a3 = ld_stream<FLAGS>(val + k + 3 * stride);
        }
        const uint32_t w0 = S[(int64_t)c0 * W + wo], w1 = S[(int64_t)c1 * W + wo];
        const uint32_t w2 = S[(int64_t)c2 * W + wo], w3 = S[(int64_t)c3 * W + wo];
#pragma unroll
        for (int e = 0; e < G::VEC; ++e) {
            s[e] = fma(a0, sign_of<P, G>(w0, p0, e), s[e]);
            s[e] = fma(a1, sign_of<P, G>(w1, p0, e), s[e]);
            s[e] = fma(a2, sign_of<P, G>(w2, p0, e), s[e]);
            s[e] = fma(a3, sign_of<P, G>(w3, p0, e), s[e]);
        }
    }
    for (; k < end; k += stride) {
        const int c0 = ld_stream<FLAGS>(col + k);
        double a0 = 1.0;
        if constexpr (!(FLAGS & KF_UNIT)) a0 = ld_stream<FLAGS>(val + k);
        const uint32_t w0 = S[(int64_t)c0 * W + wo];
#pragma unroll
        for (int e = 0; e < G::VEC; ++e) s[e] = fma(a0, sign_of<P, G>(w0, p0, e), s[e]);
    }
}

// Start pass (y-form): y_0 = s0 A z from the packed signs; partials as
// k_spmm_lanczos with X = z (X.t, X.y_0, y_0.y_0).
template <int P, int BLOCK, int FLAGS>
__global__ __launch_bounds__(BLOCK) void k_spmm_lanczos_start(
    const int* __restrict__ row_ptr, const int* __restrict__ col, const double* __restrict__ val,
    int n, const uint32_t* __restrict__ S, double s0, double* __restrict__ Out,
    double* __restrict__ partial, const int* __restrict__ long_rows, int n_long, int long_thresh,
    int long_blocks) {
    using G = GeoKY<P>;
    using V = VecT<G::VEC>;
    constexpr int WAVES = BLOCK / 64;
    constexpr int W = (P + 31) / 32;
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int sub = lane % G::LPR;
    const int grp = lane / G::LPR;
    const int p0 = sub * G::VEC;
    double d0[G::VEC], d1[G::VEC], d2[G::VEC];
#pragma unroll
    for (int e = 0; e < G::VEC; ++e) d0[e] = d1[e] = d2[e] = 0.0;
    __amdgpu_buffer_rsrc_t orsrc = __builtin_amdgcn_make_buffer_rsrc(
        Out, 0, (FLAGS & KF_SC1) ? (int)((int64_t)n * P * 8) : 0, 0x00020000);
    auto epilogue = [&](int row, const double* sum) {
        const uint32_t wr = S[(int64_t)row * W + (p0 >> 5)];
        typename V::T o;
        double* op = reinterpret_cast<double*>(&o);
#pragma unroll
        for (int e = 0; e < G::VEC; ++e) {
            const double x = sign_of<P, G>(wr, p0, e);
            const double u = s0 * sum[e];
            op[e] = u;
            d0[e] = fma(x, sum[e], d0[e]);
            d1[e] = fma(x, u, d1[e]);
            d2[e] = fma(u, u, d2[e]);
        }
        if constexpr (FLAGS & KF_SC1) store_sc1<G::VEC>(orsrc, (uint32_t)(((int64_t)row * P + p0) * 8), op);
        else if constexpr (FLAGS & KF_NTY) V::store_nt(Out + (int64_t)row * P + p0, o);
        else V::store(Out + (int64_t)row * P + p0, o);
    };
    if ((int)blockIdx.x < long_blocks) {
        for (int li = blockIdx.x * WAVES + wave; li < n_long; li += long_blocks * WAVES) {
            const int row = long_rows[li];
            double sm[G::VEC];
#pragma unroll
            for (int e = 0; e < G::VEC; ++e) sm[e] = 0.0;
            row_gather_signs<P, FLAGS, G>(row_ptr[row] + grp, row_ptr[row + 1], G::GPW, p0, col, val, S, sm);
#pragma unroll
            for (int o = G::LPR; o < 64; o <<= 1)
#pragma unroll
                for (int e = 0; e < G::VEC; ++e) sm[e] += kt::shfl_xor(sm[e], o);
            if (grp == 0) epilogue(row, sm);
        }
    } else {
        const int sb = blockIdx.x - long_blocks;
        const int groups_total = (gridDim.x - long_blocks) * WAVES * G::GPW;
        for (int row = (sb * WAVES + wave) * G::GPW + grp; row < n; row += groups_total) {
            const int beg = ld_stream<FLAGS>(row_ptr + row);
            const int end = ld_stream<FLAGS>(row_ptr + row + 1);
            if (end - beg > long_thresh) continue;
            double sm[G::VEC];
#pragma unroll
            for (int e = 0; e < G::VEC; ++e) sm[e] = 0.0;
            row_gather_signs<P, FLAGS, G>(beg, end, 1, p0, col, val, S, sm);
            epilogue(row, sm);
        }
    }
#pragma unroll
    for (int o = G::LPR; o < 64; o <<= 1)
#pragma unroll
        for (int e = 0; e < G::VEC; ++e) {
            d0[e] += kt::shfl_xor(d0[e], o);
            d1[e] += kt::shfl_xor(d1[e], o);
            d2[e] += kt::shfl_xor(d2[e], o);
        }
    __shared__ double red[WAVES][3][P];
    if (grp == 0) {
#pragma unroll
        for (int e = 0; e < G::VEC; ++e) {
            red[wave][0][p0 + e] = d0[e];
            red[wave][1][p0 + e] = d1[e];
            red[wave][2][p0 + e] = d2[e];
        }
    }
    __syncthreads();
    for (int t = threadIdx.x; t < 3 * P; t += BLOCK) {
        const int q = t / P, p = t % P;
        double v = 0.0;
#pragma unroll
        for (int w = 0; w < WAVES; ++w) v += red[w][q][p];
        partial[(int64_t)t * gridDim.x + blockIdx.x] = v;
    }
}

// KT_KY_WPE: minimum waves per SIMD the y-form pass is compiled for (register
// budget: 8 -> <= 64 VGPRs = 4 workgroups of 512 per CU; 0 = compiler's choice)
#ifndef KT_KY_WPE
#define KT_KY_WPE 0
#endif
#ifndef KT_KY_CF_LDS
#define KT_KY_CF_LDS 0
#endif
#if KT_KY_WPE > 0
#define KT_KY_BOUNDS(B) __launch_bounds__(B, KT_KY_WPE)
#else
#define KT_KY_BOUNDS(B) __launch_bounds__(B)
#endif
template <int P, int BLOCK, int FLAGS>
__global__ KT_KY_BOUNDS(BLOCK) void k_spmm_lanczos(
    const int* __restrict__ row_ptr, const int* __restrict__ col, const double* __restrict__ val,
    int n, const double* __restrict__ X, const double* __restrict__ Yold, double* __restrict__ Out,
    const double* __restrict__ coef, double* __restrict__ partial,
    const int* __restrict__ long_rows, int n_long, int long_thresh, int long_blocks,
    const double* __restrict__ Vc, const double* __restrict__ Vo, double* __restrict__ Vn, int bcols) {
    using G = GeoKY<P>;
    constexpr int WAVES = BLOCK / 64;
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int sub = lane % G::LPR;
    const int grp = lane / G::LPR;
    const int p0 = sub * G::VEC;
    const bool has_old = Yold != nullptr;
    // Out spans n*P doubles (< 2^32 bytes when KF_SC1 is selected, kt_slq.cpp)
    __amdgpu_buffer_rsrc_t orsrc = __builtin_amdgcn_make_buffer_rsrc(
        Out, 0, (FLAGS & KF_SC1) ? (int)((int64_t)n * P * 8) : 0, 0x00020000);

    double d0[G::VEC], d1[G::VEC], d2[G::VEC];
#pragma unroll
    for (int e = 0; e < G::VEC; ++e) d0[e] = d1[e] = d2[e] = 0.0;
#if KT_KY_CF_LDS
    // (g, a, b) read from LDS per row instead of 3 x VEC registers per lane
    // (volatile: the compiler must not hoist them back into registers)
    __shared__ double s_cf[3 * P];
    for (int t = threadIdx.x; t < 3 * P; t += BLOCK) s_cf[t] = coef[t];
    __syncthreads();
    const volatile double* cg = s_cf + p0;
    const volatile double* ca = s_cf + P + p0;
    const volatile double* cb = s_cf + 2 * P + p0;
#else
    double cg[G::VEC], ca[G::VEC], cb[G::VEC];
#pragma unroll
    for (int e = 0; e < G::VEC; ++e) {
        cg[e] = coef[p0 + e];
        ca[e] = coef[P + p0 + e];
        cb[e] = coef[2 * P + p0 + e];
    }
#endif

    if ((int)blockIdx.x < long_blocks) {
        for (int li = blockIdx.x * WAVES + wave; li < n_long; li += long_blocks * WAVES) {
            const int row = long_rows[li];
            const int beg = row_ptr[row];
            const int end = row_ptr[row + 1];
            double s[G::VEC];
#pragma unroll
            for (int e = 0; e < G::VEC; ++e) s[e] = 0.0;
#if KT_KY_DIAG != 3
            gather_row<P, FLAGS, G>(beg + grp, end, G::GPW, p0, col, val, X, s);
#endif
#pragma unroll
            for (int o = G::LPR; o < 64; o <<= 1)
#pragma unroll
                for (int e = 0; e < G::VEC; ++e) s[e] += kt::shfl_xor(s[e], o);
            if (grp == 0)
                row_epilogue_y<P, FLAGS, G, decltype(cg)>(row, p0, s, cg, ca, cb, has_old, X, Yold, Out, d0, d1, d2,
                                           orsrc, Vc, Vo, Vn, bcols);
        }
    } else {
        const int sb = blockIdx.x - long_blocks;
        const int groups_total = (gridDim.x - long_blocks) * WAVES * G::GPW;
        for (int row = (sb * WAVES + wave) * G::GPW + grp; row < n; row += groups_total) {
            const int beg = ld_stream<FLAGS>(row_ptr + row);
            const int end = ld_stream<FLAGS>(row_ptr + row + 1);
            if (end - beg > long_thresh) continue;  // owned by a long-row wave
            double s[G::VEC];
#pragma unroll
            for (int e = 0; e < G::VEC; ++e) s[e] = 0.0;
#if KT_KY_DIAG != 3  // diagnostic build 3: the row streams alone (no column / gather loads)
            gather_row<P, FLAGS, G>(beg, end, 1, p0, col, val, X, s);
#endif
            row_epilogue_y<P, FLAGS, G, decltype(cg)>(row, p0, s, cg, ca, cb, has_old, X, Yold, Out, d0, d1, d2,
                                           orsrc, Vc, Vo, Vn, bcols);
        }
    }

#pragma unroll
    for (int o = G::LPR; o < 64; o <<= 1)
#pragma unroll
        for (int e = 0; e < G::VEC; ++e) {
            d0[e] += kt::shfl_xor(d0[e], o);
            d1[e] += kt::shfl_xor(d1[e], o);
            d2[e] += kt::shfl_xor(d2[e], o);
        }
    __shared__ double red[WAVES][3][P];
    if (grp == 0) {
#pragma unroll
        for (int e = 0; e < G::VEC; ++e) {
            red[wave][0][p0 + e] = d0[e];
            red[wave][1][p0 + e] = d1[e];
            red[wave][2][p0 + e] = d2[e];
        }
    }
    __syncthreads();
    for (int t = threadIdx.x; t < 3 * P; t += BLOCK) {  // slot t = q * P + p
        const int q = t / P, p = t % P;
        double v = 0.0;
#pragma unroll
        for (int w = 0; w < WAVES; ++w) v += red[w][q][p];
        partial[(int64_t)t * gridDim.x + blockIdx.x] = v;
    }
}

// ---------------------------------------------------------------------------
// Block SpMM for the block-Krylov paths: Y[:, 0:P] = A X[:, 0:P] with row
// strides ldx, ldy (blocks are column slices of a wider row-major basis).
// Same row-group / long-row mapping as K1, no reductions.
// ---------------------------------------------------------------------------
// Rows longer than split_thresh (every long row) are cut into chunks of
// kChunkNnz nonzeros, one WAVE per chunk in blocks [0, chunk_blocks); each
// writes its partial row to ck_part[slice][chunk][P] and k_spmm_combine sums
// a row's chunks in chunk order (deterministic).  With P = 128 a wave holds a
// single row group, so a hub row of 1,500 nonzeros would otherwise be one
// wave's serial gather chain (180 us on as_735 vs 9 us for the rest).
template <int P, int BLOCK, int FLAGS>
__global__ __launch_bounds__(BLOCK) void k_spmm_block(
    const int* __restrict__ row_ptr, const int* __restrict__ col, const double* __restrict__ val,
    int n, const double* __restrict__ X, int ldx, double* __restrict__ Y, int ldy,
    const int* __restrict__ long_rows, int n_long, int long_thresh, int long_blocks,
    const int* __restrict__ skip, const int* __restrict__ ck_beg, const int* __restrict__ ck_end,
    int n_chunks, int chunk_blocks, int split_thresh, double* __restrict__ ck_part) {
    using G = GeoB<P>;
    using V = VecT<G::VEC>;
    constexpr int WAVES = BLOCK / 64;
    if (skip && *skip == 0) return;  // every consumer of this step already stopped
    X += (int64_t)blockIdx.y * P;    // column slice blockIdx.y of a wider block
    Y += (int64_t)blockIdx.y * P;
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int sub = lane % G::LPR;
    const int grp = lane / G::LPR;
    const int p0 = sub * G::VEC;
    if ((int)blockIdx.x < chunk_blocks) {
        double* part = ck_part + (int64_t)blockIdx.y * n_chunks * P;
        for (int ci = blockIdx.x * WAVES + wave; ci < n_chunks; ci += chunk_blocks * WAVES) {
            double s[G::VEC];
#pragma unroll
            for (int e = 0; e < G::VEC; ++e) s[e] = 0.0;
            gather_row<P, FLAGS, G>(ck_beg[ci] + grp, ck_end[ci], G::GPW, p0, col, val, X, s, ldx);
#pragma unroll
            for (int o = G::LPR; o < 64; o <<= 1)
#pragma unroll
                for (int e = 0; e < G::VEC; ++e) s[e] += kt::shfl_xor(s[e], o);
            if (grp == 0) {
#pragma unroll
                for (int e = 0; e < G::VEC; ++e) part[(int64_t)ci * P + p0 + e] = s[e];
            }
        }
    } else if ((int)blockIdx.x < chunk_blocks + long_blocks) {
        const int lb = blockIdx.x - chunk_blocks;
        for (int li = lb * WAVES + wave; li < n_long; li += long_blocks * WAVES) {
            const int row = long_rows[li];
            if (row_ptr[row + 1] - row_ptr[row] > split_thresh) continue;  // chunked
            double s[G::VEC];
#pragma unroll
            for (int e = 0; e < G::VEC; ++e) s[e] = 0.0;
            gather_row<P, FLAGS, G>(row_ptr[row] + grp, row_ptr[row + 1], G::GPW, p0, col, val, X, s,
                                 ldx);
#pragma unroll
            for (int o = G::LPR; o < 64; o <<= 1)
#pragma unroll
                for (int e = 0; e < G::VEC; ++e) s[e] += kt::shfl_xor(s[e], o);
            if (grp == 0) {
                typename V::T yo;
                double* yp = reinterpret_cast<double*>(&yo);
#pragma unroll
                for (int e = 0; e < G::VEC; ++e) yp[e] = s[e];
                V::store(Y + (int64_t)row * ldy + p0, yo);
            }
        }
    } else {
        const int sb = blockIdx.x - chunk_blocks - long_blocks;
        const int groups_total = (gridDim.x - chunk_blocks - long_blocks) * WAVES * G::GPW;
        for (int row = (sb * WAVES + wave) * G::GPW + grp; row < n; row += groups_total) {
            const int beg = row_ptr[row], end = row_ptr[row + 1];
            if (end - beg > long_thresh) continue;
            double s[G::VEC];
#pragma unroll
            for (int e = 0; e < G::VEC; ++e) s[e] = 0.0;
            gather_row<P, FLAGS, G>(beg, end, 1, p0, col, val, X, s, ldx);
            typename V::T yo;
            double* yp = reinterpret_cast<double*>(&yo);
#pragma unroll
            for (int e = 0; e < G::VEC; ++e) yp[e] = s[e];
            V::store(Y + (int64_t)row * ldy + p0, yo);
        }
    }
}

// Y[row, slice P + t] = sum of the row's chunk partials in chunk order
template <int P>
__global__ __launch_bounds__(128) void k_spmm_combine(const int* __restrict__ sp_rows,
                                                      const int* __restrict__ sp_first, int n_chunks,
                                                      const double* __restrict__ ck_part,
                                                      double* __restrict__ Y, int ldy,
                                                      const int* __restrict__ skip) {
    if (skip && *skip == 0) return;
    const int t = threadIdx.x;
    if (t >= P) return;
    const int i = blockIdx.x;
    const double* part = ck_part + (int64_t)blockIdx.y * n_chunks * P;
    double s = 0.0;
    int c = sp_first[i];
    const int ce = sp_first[i + 1];
    for (; c + 8 <= ce; c += 8) {  // 8 loads in flight, summed in chunk order
        double v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = part[(int64_t)(c + u) * P + t];
#pragma unroll
        for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; c < ce; ++c) s += part[(int64_t)c * P + t];
    Y[(int64_t)sp_rows[i] * ldy + (int64_t)blockIdx.y * P + t] = s;
}

// ---------------------------------------------------------------------------
// Deterministic column reduction of per-block slabs [nblk][slots]: 64 slots
// per workgroup (one per lane), 16 waves striding over the slabs in a fixed
// order, LDS combine in wave order.  The sum lands in every lane of wave 0.
// ---------------------------------------------------------------------------
// Slot-major slabs: partial[slot * nblk + b].  One WAVE per slot reads the
// slot's nblk partials with coalesced loads (all in flight at once), sums
// lane-wise in block order, then a fixed xor-tree -- deterministic.
constexpr int kReduceDepth = 32;
__device__ __forceinline__ double wave_reduce_slot(const double* __restrict__ partial, int nblk,
                                                   int slot) {
    const int lane = threadIdx.x & 63;
    const double* base = partial + (int64_t)slot * nblk;
    double v = 0.0;
    // 32 predicated loads in flight per lane before the in-order adds: the
    // slabs are read right after the producing pass, while the other sweep
    // lane's pass loads the memory system, so each round trip costs
    // microseconds (a 4-deep loop over the pass's ~1,500 blocks measured
    // 21.6 us per k_ycoef under two lanes; this 32-deep form measured 25.4 us
    // in a later profile, bench unchanged at 2.54 evals/s, so the slab read
    // is bound by the concurrent pass, not by load depth -- see
    // profiles/r01_final_kernel_stats.csv).  Each lane still adds its blocks
    // in increasing order (out-of-range slots add +0.0), so sums are unchanged.
    for (int b = lane; b < nblk; b += 64 * kReduceDepth) {
        double x[kReduceDepth];
#pragma unroll
        for (int i = 0; i < kReduceDepth; ++i) {
            const int bi = b + 64 * i;
            x[i] = bi < nblk ? base[bi] : 0.0;
        }
#pragma unroll
        for (int i = 0; i < kReduceDepth; ++i) v += x[i];
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += kt::shfl_xor(v, o);
    return v;
}

// k2s[4][P] carries the previous K2's sums: [0] ||u_cur||^2, [1] y_prev . u_cur,
// [2] u_prev . u_cur, [3] ||u_prev||^2.  Window Gram (v = s u):
//   g0 = v_prev.y = (A v_prev).v_cur = s_cur k2s[1]     (symmetry of A)
//   g1 = v_cur.y  (K1 partials)
//   G00 = s_prev^2 k2s[3], G01 = s_prev s_cur k2s[2], G11 = s_cur^2 k2s[0]
// CGS2: h = (g0, g1), h' = h - G h, c = h + h' -> H(j-1,j) = c0, H(j,j) = c1.
template <int P>
__global__ __launch_bounds__(256) void k_coef_cgs2(const double* __restrict__ partial, int nblk,
                                                    int first, const double* __restrict__ k2s,
                                                    const double* __restrict__ scale_cur,
                                                    const double* __restrict__ scale_prev,
                                                    double* __restrict__ coef,
                                                    double* __restrict__ t_alpha,
                                                    double* __restrict__ t_up,
                                                    double* __restrict__ hist) {
    const int p = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (p >= P) return;
    const double g1 = wave_reduce_slot(partial, nblk, p);
    if ((threadIdx.x & 63) == 0) {
        const double sc = scale_cur[p];
        if (hist) hist[p] = sc;  // the basis sweep's scale history: v_j = s_j u_j
        const double G11 = sc * sc * k2s[0 * P + p];
        double g0 = 0.0, G00 = 0.0, G01 = 0.0;
        if (!first) {
            const double sp = scale_prev[p];
            g0 = sc * k2s[1 * P + p];
            G01 = sp * sc * k2s[2 * P + p];
            G00 = sp * sp * k2s[3 * P + p];
        }
        const double h0p = g0 - (G00 * g0 + G01 * g1);
        const double h1p = g1 - (G01 * g0 + G11 * g1);
        const double c0 = g0 + h0p, c1 = g1 + h1p;
        coef[p] = c0;
        coef[P + p] = c1;
        t_alpha[p] = c1;
        t_up[p] = c0;
    }
}

// ---------------------------------------------------------------------------
// K2: u_next = y - c0 s_prev u_prev - c1 s_cur u_cur (in place over u_prev);
// partial slabs [3][P][grid]: ||u_next||^2, y.u_next, u_cur.u_next.  rec
// (optional): u_next's first bcols columns also stored to rec[row * bcols + c]
// (the sweep's basis slot of the next step, kt_slq.cpp).
// Pure streaming: rows are contiguous, so lanes cover 16 B each.
// ---------------------------------------------------------------------------

template <int P, int BLOCK, bool NT>
__global__ __launch_bounds__(BLOCK) void k_update(
    int n, const double* __restrict__ y, double* __restrict__ uprev,
    const double* __restrict__ ucur, const double* __restrict__ scale_cur,
    const double* __restrict__ scale_prev, const double* __restrict__ coef, int first,
    double* __restrict__ partial, double* __restrict__ rec, int bcols) {
    using G = Geo<P>;
    using V = VecT<G::VEC>;
    constexpr int WAVES = BLOCK / 64;
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int sub = lane % G::LPR;
    const int grp = lane / G::LPR;
    const int p0 = sub * G::VEC;
    double a0[G::VEC], a1[G::VEC], nn[G::VEC], yu[G::VEC], cu[G::VEC];
#pragma unroll
    for (int e = 0; e < G::VEC; ++e) {
        a0[e] = first ? 0.0 : coef[p0 + e] * scale_prev[p0 + e];
        a1[e] = coef[P + p0 + e] * scale_cur[p0 + e];
        nn[e] = yu[e] = cu[e] = 0.0;
    }
    const int groups_total = gridDim.x * WAVES * G::GPW;
    for (int row = (blockIdx.x * WAVES + wave) * G::GPW + grp; row < n; row += groups_total) {
        const int64_t off = (int64_t)row * P + p0;
        // y and u_prev are dead after this pass (u_next overwrites u_prev)
        const typename V::T yv = NT ? V::load_nt(y + off) : V::load(y + off);
        const typename V::T cv = V::load(ucur + off);
        typename V::T pv;
        if (!first) pv = NT ? V::load_nt(uprev + off) : V::load(uprev + off);
        typename V::T o;
        double* op = reinterpret_cast<double*>(&o);
#pragma unroll
        for (int e = 0; e < G::VEC; ++e) {
            double u = V::get(yv, e);
            if (!first) u = fma(-a0[e], V::get(pv, e), u);
            u = fma(-a1[e], V::get(cv, e), u);
            op[e] = u;
            nn[e] = fma(u, u, nn[e]);
            yu[e] = fma(V::get(yv, e), u, yu[e]);
            cu[e] = fma(V::get(cv, e), u, cu[e]);
        }
        V::store(uprev + off, o);
        if (rec && p0 < bcols) {
#pragma unroll
            for (int e = 0; e < G::VEC; ++e)
                if (p0 + e < bcols) rec[(int64_t)row * bcols + p0 + e] = op[e];
        }
    }
#pragma unroll
    for (int o = G::LPR; o < 64; o <<= 1)
#pragma unroll
        for (int e = 0; e < G::VEC; ++e) {
            nn[e] += kt::shfl_xor(nn[e], o);
            yu[e] += kt::shfl_xor(yu[e], o);
            cu[e] += kt::shfl_xor(cu[e], o);
        }
    __shared__ double red[WAVES][3][P];
    if (grp == 0) {
#pragma unroll
        for (int e = 0; e < G::VEC; ++e) {
            red[wave][0][p0 + e] = nn[e];
            red[wave][1][p0 + e] = yu[e];
            red[wave][2][p0 + e] = cu[e];
        }
    }
    __syncthreads();
    for (int t = threadIdx.x; t < 3 * P; t += BLOCK) {  // slot t = q * P + p
        const int q = t / P, p = t % P;
        double v = 0.0;
#pragma unroll
        for (int w = 0; w < WAVES; ++w) v += red[w][q][p];
        partial[(int64_t)t * gridDim.x + blockIdx.x] = v;
    }
}

// norm: beta = ||u_next||; s_next = 1/beta (0 after a lucky breakdown,
// lanczos_krylov.m:91-93, lucky_tol = 1e-8); T-record row `low` = beta;
// refresh k2s for the next coef step.
template <int P>
__global__ __launch_bounds__(256) void k_norm(const double* __restrict__ partial, int nblk,
                                               double* __restrict__ k2s,
                                               double* __restrict__ scale_next,
                                               double* __restrict__ t_low) {
    const int slot = blockIdx.x * 4 + (threadIdx.x >> 6);  // slot = q * P + p
    if (slot >= 3 * P) return;
    const double r = wave_reduce_slot(partial, nblk, slot);
    if ((threadIdx.x & 63) == 0) {
        const int q = slot / P, p = slot % P;
        if (q == 0) {
            const double beta = sqrt(r);
            t_low[p] = beta;
            scale_next[p] = (beta < 1e-8) ? 0.0 : 1.0 / beta;
            k2s[3 * P + p] = k2s[0 * P + p];
            k2s[0 * P + p] = r;
        } else {
            k2s[q * P + p] = r;
        }
    }
}

// y-form coefficients (one workgroup per probe, one wave per dot).  State
// ys[k][P]: 0 alpha_j, 1 beta_j, 2 alpha_{j-1}, 3 ||y_j||^2, 4 y_{j-1}.y_j,
// 5 beta_{j+1}, 6..8 the next pass's (g, a, b).  Identities (A = A',
// v_i orthonormal, y_i = A v_i):
//   alpha_0 = v_0.y_0,  beta_1^2 = ||y_0||^2 - alpha_0^2,
//   alpha_{j+1} beta_{j+1}^2 = y_j'A y_j - 2 alpha_j ||y_j||^2
//        - 2 beta_j y_{j-1}.y_j + alpha_j^3 + 2 alpha_j beta_j^2 + beta_j^2 alpha_{j-1},
//   beta_{j+2}^2 = ||y_{j+1}||^2 - alpha_{j+1}^2 - beta_{j+1}^2.
// guard[p] = min over the used beta_k of beta_k^2 / ||y_{k-1}||^2: a small
// ratio (cancellation; a lucky breakdown) sends the sweep back to the
// explicit CGS2 path on the host (kt_slq.cpp), so breakdowns keep the
// reference's semantics (lanczos_krylov.m:91-93).
// Records: alpha[j], up[j] = beta_j, low[j] = beta_{j+1}.
template <int P>
__global__ __launch_bounds__(192) void k_ycoef(const double* __restrict__ partial, int nblk,
                                               int start, int last, double s0,
                                               double* __restrict__ ys,
                                               double* __restrict__ t_alpha,
                                               double* __restrict__ t_up,
                                               double* __restrict__ t_low,
                                               double* __restrict__ guard) {
    const int p = blockIdx.x;
    const int q = threadIdx.x >> 6;
    const double r = wave_reduce_slot(partial, nblk, q * P + p);
    __shared__ double d[3];
    if ((threadIdx.x & 63) == 0) d[q] = r;
    __syncthreads();
    if (threadIdx.x != 0) return;
    ycoef_probe(p, P, d[0], d[1], d[2], start, last, s0, ys, t_alpha, t_up, t_low, guard);
}

// ---------------------------------------------------------------------------
// Small streaming kernels for the Afun paths (mc_trace.m / expmv.m).
// ---------------------------------------------------------------------------
// Y[r, c] = sum_j U[r * ldu + j * sstride + c] * W[j*P + c]
// (f(A)x = ||x|| V f(T) e1; slot j of the basis at U + j * sstride)
__global__ __launch_bounds__(256) void k_weighted_sum(int n, int m, int P, int nc,
                                                      const double* __restrict__ U, int ldu,
                                                      int64_t sstride, const double* __restrict__ W,
                                                      double* __restrict__ Y, int ldy) {
    const int64_t total = (int64_t)n * nc;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = t / nc;
        const int c = (int)(t % nc);
        const double* u = U + r * ldu + c;
        double s = 0.0;
        // the slots' loads of a group of 8 issue together (one memory round
        // trip), then the fma chain in slot order: the sum is bit-identical
        // to the one-slot loop's
        constexpr int kG = 8;
        for (int j0 = 0; j0 < m; j0 += kG) {
            double v[kG];
#pragma unroll
            for (int g = 0; g < kG; ++g) v[g] = (j0 + g < m) ? __builtin_nontemporal_load(u + (int64_t)(j0 + g) * sstride) : 0.0;
#pragma unroll
            for (int g = 0; g < kG; ++g)
                if (j0 + g < m) s = fma(v[g], W[(j0 + g) * P + c], s);
        }
        Y[r * ldy + c] = s;
    }
}

// Row permutation of a row-major block: gather (dst[r] = src[perm[r]]) or
// scatter (dst[perm[r]] = src[r]), cols columns -- natural-order blocks into
// the hubs-first row order of the probe sweep and back (kt_slq.cpp).
__global__ __launch_bounds__(256) void k_perm_rows(int n, int cols, const int* __restrict__ perm, int gather,
                                                   const double* __restrict__ src, int lds,
                                                   double* __restrict__ dst, int ldd) {
    const int64_t total = (int64_t)n * cols;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = t / cols;
        const int c = (int)(t % cols);
        const int64_t p = perm[r];
        if (gather)
            dst[r * ldd + c] = src[p * lds + c];
        else
            dst[p * ldd + c] = src[r * lds + c];
    }
}

// Y[:, 0:nc] = a X + b Y
__global__ __launch_bounds__(256) void k_axpby(int n, int nc, double a, const double* __restrict__ X,
                                               int ldx, double b, double* __restrict__ Y, int ldy) {
    const int64_t total = (int64_t)n * nc;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = t / nc;
        const int c = (int)(t % nc);
        const double y = (b == 0.0) ? 0.0 : b * Y[r * ldy + c];
        Y[r * ldy + c] = fma(a, X[r * ldx + c], y);
    }
}

// per-block partial of the matrix infinity norm max_r sum_c |X[r, c]|
__global__ __launch_bounds__(256) void k_inf_norm(int n, int nc, const double* __restrict__ X,
                                                  int ldx, double* __restrict__ partial) {
    double mx = 0.0;
    for (int r = blockIdx.x * blockDim.x + threadIdx.x; r < n; r += gridDim.x * blockDim.x) {
        double s = 0.0;
        for (int c = 0; c < nc; ++c) s += fabs(X[(int64_t)r * ldx + c]);
        mx = fmax(mx, s);
    }
    for (int o = 32; o > 0; o >>= 1) mx = fmax(mx, kt::shfl_xor(mx, o));
    __shared__ double red[4];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
    __syncthreads();
    if (threadIdx.x == 0) partial[blockIdx.x] = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
}

// normest1 (t = 1, normAm.m:25): statistics of Y = B^m X for the host's
// iteration -- per-block sum |Y| and S_prev . S, with S = mysign(Y)
// (sign(0) = +1) written for the transposed product.  The sign dot is a sum
// of +-1 terms, exact in fp64.
__global__ __launch_bounds__(256) void k_normest1_y(int n, const double* __restrict__ Y,
                                                   const double* __restrict__ Sprev,
                                                   double* __restrict__ S,
                                                   double* __restrict__ partial) {
    double a = 0.0, d = 0.0;
    for (int r = blockIdx.x * blockDim.x + threadIdx.x; r < n; r += gridDim.x * blockDim.x) {
        const double y = Y[r];
        const double s = y < 0.0 ? -1.0 : 1.0;
        a += fabs(y);
        d = fma(Sprev[r], s, d);
        S[r] = s;
    }
    for (int o = 32; o > 0; o >>= 1) {
        a += kt::shfl_xor(a, o);
        d += kt::shfl_xor(d, o);
    }
    __shared__ double red[2][4];
    if ((threadIdx.x & 63) == 0) {
        red[0][threadIdx.x >> 6] = a;
        red[1][threadIdx.x >> 6] = d;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        partial[blockIdx.x] = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
        partial[gridDim.x + blockIdx.x] = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
    }
}

// per-block max |Z| and the smallest row index attaining it (normest1's
// h = abs(Z) and its ordering for t = 1)
__device__ __forceinline__ void absmax_merge(double& v, int& i, double v2, int i2) {
    if (v2 > v || (v2 == v && i2 < i)) {
        v = v2;
        i = i2;
    }
}
__global__ __launch_bounds__(256) void k_absmax_idx(int n, const double* __restrict__ Z,
                                                    double* __restrict__ pval, int* __restrict__ pidx) {
    double v = -1.0;
    int i = 0x7fffffff;
    for (int r = blockIdx.x * blockDim.x + threadIdx.x; r < n; r += gridDim.x * blockDim.x)
        absmax_merge(v, i, fabs(Z[r]), r);
    for (int o = 32; o > 0; o >>= 1) absmax_merge(v, i, kt::shfl_xor(v, o), kt::shfl_xor(i, o));
    __shared__ double sv[4];
    __shared__ int si[4];
    if ((threadIdx.x & 63) == 0) {
        sv[threadIdx.x >> 6] = v;
        si[threadIdx.x >> 6] = i;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < 4; ++w) absmax_merge(v, i, sv[w], si[w]);
        pval[blockIdx.x] = v;
        pidx[blockIdx.x] = i;
    }
}

__global__ void k_fill(double* __restrict__ x, int count, double v) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < count) x[t] = v;
}

// out (nr x cols, column-major) = rows[r] of the row-major block D (ldd)
__global__ __launch_bounds__(256) void k_gather_rows(int nr, int cols, const double* __restrict__ D,
                                                     int ldd, const int64_t* __restrict__ rows,
                                                     double* __restrict__ out) {
    const int64_t total = (int64_t)nr * cols;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (int64_t)gridDim.x * blockDim.x) {
        const int r = (int)(t % nr);
        const int c = (int)(t / nr);
        out[t] = D[rows[r] * ldd + c];
    }
}

// out[i] = D[off[i]]: scattered elements of a device array in one launch
__global__ __launch_bounds__(256) void k_gather_elems(int64_t count, const double* __restrict__ D,
                                                      const int64_t* __restrict__ off,
                                                      double* __restrict__ out) {
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < count;
         t += (int64_t)gridDim.x * blockDim.x)
        out[t] = D[off[t]];
}

// D[off[t]] = val[t]: the nonzeros of a mostly-zero host block (a node
// selector U of fun_and_grad_krylov_*) dropped into a zeroed device block
__global__ __launch_bounds__(256) void k_scatter_elems(int64_t count, const int64_t* __restrict__ off,
                                                       const double* __restrict__ val, double* __restrict__ D) {
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < count;
         t += (int64_t)gridDim.x * blockDim.x)
        D[off[t]] = val[t];
}

// ---------------------------------------------------------------------------
// expmv.m:71-92 Taylor loop with its stop test on the device, so the host
// queues a whole stage without a round trip per term.  State (ExpmvState):
// active = 1 while the stage runs; every kernel of a term (the SpMM through
// its skip flag, k_expmv_term, k_expmv_check) is a no-op once active = 0.
// ---------------------------------------------------------------------------
// term maxima of the fused expmv path: 64 slots per term, one 128-B line
// each (workgroup b folds into slot b % 64), so same-address atomics stay few
// (config 1: 340 workgroups, 31k at n = 1M)
constexpr int kTermSlots = 64, kTermSlotStride = 16;
struct ExpmvState {
    int active;
    int mv;
    double c1;
    double c1s[2];  // fused path: c1 of the check of term j in c1s[j & 1]
    // fused path: term j's row-sum maxima of |b| and |f| in set j % 3, as
    // the bit patterns of the (non-negative) doubles, so an unsigned atomic
    // max is the exact fmax; term j zeroes set (j + 1) % 3 for the next
    // term, k_expmv_begin set 1 for a stage's first term
    unsigned long long term_max[3][kTermSlots][kTermSlotStride];
};

// stage start: c1 = norm(b, inf) from k_inf_norm partials; active = 1   (:73)
__global__ __launch_bounds__(256) void k_expmv_begin(const double* __restrict__ partial, int nb,
                                                     ExpmvState* st) {
    double mx = 0.0;
    for (int i = threadIdx.x; i < nb; i += blockDim.x) mx = fmax(mx, partial[i]);
    for (int o = 32; o > 0; o >>= 1) mx = fmax(mx, kt::shfl_xor(mx, o));
    __shared__ double red[4];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
    __syncthreads();
    if (threadIdx.x == 0) {
        st->c1 = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
        st->c1s[1] = st->c1;
        st->active = 1;
    }
    if (threadIdx.x < kTermSlots) {
        st->term_max[1][threadIdx.x][0] = 0ull;
        st->term_max[1][threadIdx.x][1] = 0ull;
    }
}

// b = coef (Ab - mu b) (in place), f = f + b; partial maxima of the row sums
// of |b| (partial[0, nb)) and |f| (partial[nb, 2 nb))   (:75-78)
__global__ __launch_bounds__(256) void k_expmv_term(int n, int nc, double mu, double coef,
                                                    const double* __restrict__ Ab, double* __restrict__ b,
                                                    double* __restrict__ F, int ld,
                                                    double* __restrict__ partial,
                                                    const ExpmvState* __restrict__ st) {
    if (!st->active) return;
    double mb = 0.0, mf = 0.0;
    for (int r = blockIdx.x * blockDim.x + threadIdx.x; r < n; r += gridDim.x * blockDim.x) {
        double sb = 0.0, sf = 0.0;
        for (int c = 0; c < nc; ++c) {
            const int64_t o = (int64_t)r * ld + c;
            double t = Ab[o];
            if (mu != 0.0) t = fma(-mu, b[o], t);  // (A - mu I) b, as launch_axpby(-mu, b, 1, Ab)
            const double bn = fma(coef, t, 0.0);
            const double f = fma(1.0, bn, F[o]);
            b[o] = bn;
            F[o] = f;
            sb += fabs(bn);
            sf += fabs(f);
        }
        mb = fmax(mb, sb);
        mf = fmax(mf, sf);
    }
    for (int o = 32; o > 0; o >>= 1) {
        mb = fmax(mb, kt::shfl_xor(mb, o));
        mf = fmax(mf, kt::shfl_xor(mf, o));
    }
    __shared__ double red[2][4];
    if ((threadIdx.x & 63) == 0) {
        red[0][threadIdx.x >> 6] = mb;
        red[1][threadIdx.x >> 6] = mf;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        partial[blockIdx.x] = fmax(fmax(red[0][0], red[0][1]), fmax(red[0][2], red[0][3]));
        partial[gridDim.x + blockIdx.x] = fmax(fmax(red[1][0], red[1][1]), fmax(red[1][2], red[1][3]));
    }
}

// bout = coef (A bin - mu bin), F = F + bout on one row (VEC columns from p0);
// row sums of |bout| and |F| of those columns into sb, sf   (expmv.m:75-78)
// The row's own F and b values are loaded before the gathers (expmv_row_prefetch).
template <int VEC>
__device__ __forceinline__ void expmv_row_prefetch(int row, int p0, int nc, int ld, double mu,
                                                   const double* __restrict__ bin,
                                                   const double* __restrict__ F, double* fo, double* bo) {
#pragma unroll
    for (int e = 0; e < VEC; ++e) {
        const int c = p0 + e;
        const int64_t o = (int64_t)row * ld + c;
        fo[e] = (c < nc) ? F[o] : 0.0;
        bo[e] = (c < nc && mu != 0.0) ? bin[o] : 0.0;
    }
}
// PADW = false: the padding columns nc..P-1 of bout are not written (the
// row-blocked kernel: both ping-pong blocks are zeroed when allocated and
// never written there)
template <int VEC, bool PADW = true>
__device__ __forceinline__ void expmv_row_update(int row, int p0, const double* s, const double* fo,
                                                 const double* bo, int nc, int ld, double mu, double coef,
                                                 double* __restrict__ bout, double* __restrict__ F,
                                                 double& sb, double& sf) {
#pragma unroll
    for (int e = 0; e < VEC; ++e) {
        const int c = p0 + e;
        const int64_t o = (int64_t)row * ld + c;
        if (c < nc) {
            double t = s[e];
            if (mu != 0.0) t = fma(-mu, bo[e], t);  // (A - mu I) b, as launch_axpby(-mu, b, 1, Ab)
            const double bn = fma(coef, t, 0.0);
            const double f = fma(1.0, bn, fo[e]);
            bout[o] = bn;
            F[o] = f;
            sb += fabs(bn);
            sf += fabs(f);
        } else if constexpr (PADW) {
            bout[o] = 0.0;
        }
    }
}

// One whole Taylor term in one launch (SpMM fused with the update and with
// the previous term's stop test):
//   the check of term k-1 (expmv.m:79-82) from that term's maxima
//   (the 64 slots of st->term_max[(k-1) % 3], read by wave 0) and
//   c1 = st->c1s[(k-1) & 1] -- stop: st->active = 0; otherwise
//   c1s[k & 1] = c2 (every block stores the same value);
//   bout = coef (A bin - mu bin), F = F + bout, and the workgroup's maxima of
//   the row sums of |bout| and |F| folded into slot blockIdx % 64 of
//   st->term_max[k % 3] by one atomic max each (max is exact: any arrival
//   order gives the same value); block 0 counts the term (mv) and zeroes set
//   (k + 1) % 3.
// Each workgroup reads 64 slots for the check, not the previous term's
// 2 x gridDim.x partials: at n = 1M (31k workgroups) that all-to-all read was
// 15 GB per term (8.3 ms per term on config 4's expmv Afun); one slot per
// term instead serialised 62k same-address atomics (3.5 ms per term, and
// config 1 13.2 -> 30.7 ms).
// A small matrix makes this a chain of dependent memory latencies, so the
// reads of the check and the gathers are issued before anything is decided
// (only the writes wait for the decision), and no row is a long serial
// chain: blocks [0, n_long) take one row longer than long_thresh each (64
// row groups of 32 B per lane, 8 deep, summed through LDS), the next
// ceil(n_med / 4) blocks one row of kMedThresh < degree <= long_thresh per
// WAVE (16 row groups, 8 deep: one round trip), the rest one row of degree
// <= kMedThresh per row group (8 deep).
// bin / bout ping-pong between terms; columns nc..P-1 of the blocks stay zero
// so the P-wide gathers read finite values.
// waves per block of the per-term expmv kernel (a row longer than long_thresh
// is one block's, its gather chain degree / (16 WAVES) deep).  8 waves were
// measured slower than 4 on config 1 (trace_exp 18.1 vs 16.1 ms,
// profiles/r02_expmv_waves.txt): the hub chains are not the term's limit.
#ifndef KT_EXPMV_WAVES
#define KT_EXPMV_WAVES 4
#endif
constexpr int kExpmvWaves = KT_EXPMV_WAVES;
// grids above this many workgroups take the SPLIT term kernel (config 1: 340
// workgroups, fused; n = 1M: 31k, split)
constexpr int kExpmvSplitBlocks = 1024;

//
// SPLIT (large grids, expmv_split_check): the check of term k-1 is not in
// this kernel but in k_expmv_slot_check, launched after term k-1; every
// workgroup reads st->active FIRST and a stopped term returns before its
// gathers.  The fused form issues the gathers before the decision (latency
// hiding on small matrices), which at n = 1M made each of the ~20 no-op terms
// a stage queues ahead of its stop cost a full SpMM (300 us).  The split form
// also loads a row's own F and b after its gathers, not before (94 instead of
// 124 VGPRs; config-4 expmv 6 % faster; compiled for 6 waves per SIMD at 80
// VGPRs it measured no further gain).
template <int P, int FLAGS, bool SPLIT>
__global__ __launch_bounds__(64 * kExpmvWaves) void k_expmv_step(
    const int* __restrict__ rp, const int* __restrict__ ci, const double* __restrict__ va, int n,
    const int* __restrict__ long_rows, int n_long, const int* __restrict__ med_rows, int n_med,
    int nc, int ld, double mu, double coef, double tol, int k, const double* __restrict__ bin,
    double* __restrict__ bout, double* __restrict__ F, ExpmvState* st, int* hflag, int stage) {
    constexpr int WAVES = kExpmvWaves;
    using G = GeoW<P, (P >= 2) ? 2 : 1>;                          // short rows
    using GL = GeoW<P, (P >= 4) ? 4 : (P >= 2) ? 2 : 1>;          // medium / long rows
    __shared__ double red[2][WAVES];
    __shared__ double lred[WAVES][P];
    __shared__ int decide;  // 0 = skip (stopped), 1 = run
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int med_blocks = (n_med + WAVES - 1) / WAVES;
    const int kind = ((int)blockIdx.x < n_long) ? 2 : ((int)blockIdx.x < n_long + med_blocks) ? 1 : 0;
    if constexpr (SPLIT) {
        if (threadIdx.x == 0) decide = st->active;
        __syncthreads();
        if (!decide) return;
    }
    // (1) reads of the check (thread 0), consumed after the gathers
    const int act = (!SPLIT && threadIdx.x == 0) ? st->active : 0;
    const double c1 = (!SPLIT && k > 1) ? st->c1s[(k - 1) & 1] : 0.0;
    unsigned long long pmb = 0ull, pmf = 0ull;
    if (!SPLIT && wave == 0 && k > 1) {
        pmb = st->term_max[(k - 1) % 3][lane][0];
        pmf = st->term_max[(k - 1) % 3][lane][1];
    }
    // (2) the gathers of this term
    const int subL = lane % GL::LPR, grpL = lane / GL::LPR, p0L = subL * GL::VEC;
    const int sub = lane % G::LPR, grp = lane / G::LPR, p0 = sub * G::VEC;
    double sl[GL::VEC], s[G::VEC], fo[GL::VEC], bo[GL::VEC];  // fo / bo: the row's own F, b
#pragma unroll
    for (int e = 0; e < GL::VEC; ++e) sl[e] = fo[e] = bo[e] = 0.0;
#pragma unroll
    for (int e = 0; e < G::VEC; ++e) s[e] = 0.0;
    int row = -1;
    bool mine = false;  // this lane holds a finished row (of its row class)
    if (kind == 2) {
        row = long_rows[blockIdx.x];
        if (!SPLIT && wave == 0 && grpL == 0) expmv_row_prefetch<GL::VEC>(row, p0L, nc, ld, mu, bin, F, fo, bo);
        row_gather8<P, FLAGS, GL>(rp[row] + wave * GL::GPW + grpL, rp[row + 1], WAVES * GL::GPW, p0L, ci,
                                  va, bin, sl, ld);
    } else if (kind == 1) {
        const int mi = ((int)blockIdx.x - n_long) * WAVES + wave;
        if (mi < n_med) {
            row = med_rows[mi];
            if (!SPLIT && grpL == 0) expmv_row_prefetch<GL::VEC>(row, p0L, nc, ld, mu, bin, F, fo, bo);
            row_gather8<P, FLAGS, GL>(rp[row] + grpL, rp[row + 1], GL::GPW, p0L, ci, va, bin, sl, ld);
            mine = grpL == 0;
        }
    } else {
        row = (((int)blockIdx.x - n_long - med_blocks) * WAVES + wave) * G::GPW + grp;
        if (row < n) {
            const int beg = rp[row], end = rp[row + 1];
            if (end - beg <= kMedThresh) {
                if (!SPLIT) expmv_row_prefetch<G::VEC>(row, p0, nc, ld, mu, bin, F, fo, bo);
                row_gather8<P, FLAGS, G>(beg, end, 1, p0, ci, va, bin, s, ld);
                mine = true;
            }
        }
    }
    if (kind != 0) {  // sum the row groups of the wave
#pragma unroll
        for (int o = GL::LPR; o < 64; o <<= 1)
#pragma unroll
            for (int e = 0; e < GL::VEC; ++e) sl[e] += kt::shfl_xor(sl[e], o);
    }
    if (kind == 2 && grpL == 0)
#pragma unroll
        for (int e = 0; e < GL::VEC; ++e) lred[wave][p0L + e] = sl[e];
    // (3) the check, block-uniform
    if constexpr (!SPLIT) {
    if (wave == 0) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const unsigned long long xb = kt::shfl_xor(pmb, o), xf = kt::shfl_xor(pmf, o);
            pmb = xb > pmb ? xb : pmb;
            pmf = xf > pmf ? xf : pmf;
        }
    }
    if (threadIdx.x == 0) decide = act;
    if (threadIdx.x == 0 && act && k > 1) {
        const double c2 = __longlong_as_double((long long)pmb), nf = __longlong_as_double((long long)pmf);
        if (c1 + c2 <= tol * nf) {
            st->active = 0;
            decide = 0;
            // tell the host (pinned, coherent): the rest of this stage's terms
            // are no-ops, it may stop queueing them
            if (hflag && blockIdx.x == 0)
                __hip_atomic_store(hflag, stage, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        } else {
            st->c1s[k & 1] = c2;
        }
    }
    __syncthreads();
    if (!decide) return;
    } else {
        __syncthreads();  // lred (long rows) complete
    }
    if (blockIdx.x == 0) {
        if (threadIdx.x == 0) st->mv += 1;
        if (!SPLIT && threadIdx.x < kTermSlots) {  // the next term's set (last read by term k - 1)
            st->term_max[(k + 1) % 3][threadIdx.x][0] = 0ull;
            st->term_max[(k + 1) % 3][threadIdx.x][1] = 0ull;
        }
    }
    // (4) update, norm partials of this term
    double sb = 0.0, sf = 0.0;
    if (kind == 0) {
        if (mine) {
            // SPLIT (large grids): the row's own F, b after the gathers (fewer live registers)
            if constexpr (SPLIT) expmv_row_prefetch<G::VEC>(row, p0, nc, ld, mu, bin, F, fo, bo);
            expmv_row_update<G::VEC>(row, p0, s, fo, bo, nc, ld, mu, coef, bout, F, sb, sf);
        }
#pragma unroll
        for (int o = 1; o < G::LPR; o <<= 1) {
            sb += kt::shfl_xor(sb, o);
            sf += kt::shfl_xor(sf, o);
        }
    } else {
        if (kind == 2 && wave == 0 && grpL == 0) {
#pragma unroll
            for (int e = 0; e < GL::VEC; ++e)
            {
                double t = lred[0][p0L + e];
#pragma unroll
                for (int w = 1; w < WAVES; ++w) t += lred[w][p0L + e];
                sl[e] = t;
            }
            mine = true;
        }
        if (mine) {
            if constexpr (SPLIT) expmv_row_prefetch<GL::VEC>(row, p0L, nc, ld, mu, bin, F, fo, bo);
            expmv_row_update<GL::VEC>(row, p0L, sl, fo, bo, nc, ld, mu, coef, bout, F, sb, sf);
        }
#pragma unroll
        for (int o = 1; o < GL::LPR; o <<= 1) {
            sb += kt::shfl_xor(sb, o);
            sf += kt::shfl_xor(sf, o);
        }
    }
    double mb = sb, mf = sf;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        mb = fmax(mb, kt::shfl_xor(mb, o));
        mf = fmax(mf, kt::shfl_xor(mf, o));
    }
    if (lane == 0) {
        red[0][wave] = mb;
        red[1][wave] = mf;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double x = red[0][0], y = red[1][0];
#pragma unroll
        for (int w = 1; w < WAVES; ++w) {
            x = fmax(x, red[0][w]);
            y = fmax(y, red[1][w]);
        }
        unsigned long long* slot = st->term_max[k % 3][blockIdx.x % kTermSlots];
        __hip_atomic_fetch_max(slot, (unsigned long long)__double_as_longlong(x), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_max(slot + 1, (unsigned long long)__double_as_longlong(y), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }
}

// ROW-BLOCKED form of the SPLIT term (round 6; large grids, the default there).
// The split kernel above launches one workgroup per long row, one per four
// medium rows and one per 32 short rows: 66k workgroups at config 4 (12.6k
// rows of degree > 64, 90k of 17-64), each paying an `active` read behind a
// barrier, an LDS reduction, a barrier and two atomics for one gather round
// trip.  Here resident workgroups stride over the rows with waves as the
// unit of work, as the probe passes do (k_spmm_lanczos):
//   (0) long rows of degree > kExpmvCoopThresh: one workgroup per row;
//   (1) the other long rows (degree > long_thresh): one wave per row;
//   (2) medium rows (kMedThresh < degree <= long_thresh): one wave per row,
//       the next row's task, chain columns and own f in flight meanwhile;
//   (3) short rows (degree <= kMedThresh) from a task list sorted by degree
//       within windows of 4,096 rows (kt_runtime.cpp build_csr), GPW (= 8 at
//       P = 16) per wave with one row group of 16 B per lane each, pipelined
//       the same way.
// Every row's sum is formed in exactly the order of the split / fused
// kernels, so F, s, m and mv are bit-identical to them:
//   short:  one sequential chain over the row in CSR order (row_gather8, stride 1);
//   medium: 16 chains k = beg + g + 16 i (g < 16), each in i order, summed by
//           the xor butterfly over g (g ^ 1, g ^ 2, g ^ 4, g ^ 8);
//   long:   the fused kernel's 4 waves x 16 chains k = beg + 16 w + g + 64 i,
//           each set butterflied over g, then ((t0 + t1) + t2) + t3 as the
//           fused kernel's LDS sum (one wave per set in (0), the 4 sets in
//           turn in one wave in (1)).
// The row sums of |b| and |F| and their maxima are the split kernel's too
// (the same lane geometry per row class; max is exact in any order).
// Config 4, one MI355X (profiles/r06/expmv_rows_ab): active term 394 us
// (split kernel) -> 293 us; the reference composition 1.58 -> 1.22 s.
// 4 waves per workgroup (108 VGPRs, 4 waves per SIMD); measured flat against
// 5 waves per SIMD at shallower gathers (4-deep short rows, 2-deep medium).
constexpr int kExpmvRowsWaves = 4;
template <int P, int FLAGS, bool CHECK>
__global__ __launch_bounds__(64 * kExpmvRowsWaves) void k_expmv_rows(
    const int* __restrict__ rp, const int* __restrict__ ci, const double* __restrict__ va, int n,
    const int* __restrict__ long_rows, int n_long, int n_heavy, const int4* __restrict__ med_tasks, int n_med,
    const int4* __restrict__ short_tasks, int n_short,
    int nc, int ld, double mu, double coef, int k, const double* __restrict__ bin,
    double* __restrict__ bout, double* __restrict__ F, ExpmvState* st, double tol, int* hflag, int stage) {
    constexpr int WAVES = kExpmvRowsWaves;
    constexpr int VW = 4;                                          // the fused kernel's waves per long row
    using G = GeoW<P, (P >= 2) ? 2 : 1>;                          // short rows
    using GL = GeoW<P, (P >= 4) ? 4 : (P >= 2) ? 2 : 1>;          // medium / long rows
    constexpr bool MU0 = (FLAGS & KF_MU0) != 0;
    if constexpr (MU0) mu = 0.0;  // folds every own-b load and (A - mu I) away
    __shared__ int decide;
    __shared__ double red[2][WAVES];
    __shared__ double lsum[WAVES][P];  // a heavy row's chain-set sums
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    if (wave == 0) {
        // CHECK (fused, round 6): the stop test of term k - 1 (expmv.m:79-82)
        // from its 64 slots, evaluated by every workgroup before any gather
        // (so a term past the stop costs one round trip, not a pass) --
        // the same test k_expmv_slot_check runs as its own launch.  Every
        // workgroup reads the same slots (written by the previous launch) and
        // reaches the same decision; block 0 alone records it (active = 0 and
        // the host flag, or c1s[k & 1] = c2), counts the term and zeroes the
        // next term's slot set (k + 1) % 3, last read by the check of term
        // k - 2 in the previous launch.  Without CHECK the separate launch
        // did all of that and `active` decides.
        int run = st->active;
        if (CHECK && k > 1 && run) {
            unsigned long long pmb = st->term_max[(k - 1) % 3][lane][0], pmf = st->term_max[(k - 1) % 3][lane][1];
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                const unsigned long long xb = kt::shfl_xor(pmb, o), xf = kt::shfl_xor(pmf, o);
                pmb = xb > pmb ? xb : pmb;
                pmf = xf > pmf ? xf : pmf;
            }
            const double c1 = st->c1s[(k - 1) & 1];
            const double c2 = __longlong_as_double((long long)pmb), nf = __longlong_as_double((long long)pmf);
            if (c1 + c2 <= tol * nf) {
                run = 0;
                if (blockIdx.x == 0 && lane == 0) {
                    st->active = 0;
                    if (hflag) __hip_atomic_store(hflag, stage, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                }
            } else if (blockIdx.x == 0 && lane == 0) {
                st->c1s[k & 1] = c2;
            }
        }
        if (run && blockIdx.x == 0) {
            if (lane == 0) st->mv += 1;
            if (CHECK) {
                st->term_max[(k + 1) % 3][lane][0] = 0ull;
                st->term_max[(k + 1) % 3][lane][1] = 0ull;
            }
        }
        if (lane == 0) decide = run;
    }
    __syncthreads();
    if (!decide) return;
    const int gw = blockIdx.x * WAVES + wave, TW = gridDim.x * WAVES;
    __builtin_assume(gw >= 0);
    __builtin_assume(TW > 0);
    const int subL = lane % GL::LPR, grpL = lane / GL::LPR, p0L = subL * GL::VEC;
    const int sub = lane % G::LPR, grp = lane / G::LPR, p0 = sub * G::VEC;
    double mb = 0.0, mf = 0.0;  // running maxima of this lane's row sums
    auto fold = [&](double sb, double sf, int lpr) {
        for (int o = 1; o < lpr; o <<= 1) {
            sb += kt::shfl_xor(sb, o);
            sf += kt::shfl_xor(sf, o);
        }
        mb = fmax(mb, sb);
        mf = fmax(mf, sf);
    };
    // (0) the heaviest long rows (degree > kExpmvCoopThresh, the first n_heavy
    //     of the heaviest-first list): one WORKGROUP per row, wave w running
    //     chain set w -- the fused kernel's own structure and LDS sum -- so a
    //     hub's 4 x 16 chains (49 entries each at degree 3,122) run side by
    //     side instead of one wave's 4 sets in turn (the tail of the launch)
    static_assert(WAVES == VW, "one wave per chain set");
    for (int hi = blockIdx.x; hi < n_heavy; hi += gridDim.x) {
        const int row = long_rows[hi];
        double acc[GL::VEC];
#pragma unroll
        for (int e = 0; e < GL::VEC; ++e) acc[e] = 0.0;
        row_gather8<P, FLAGS, GL, 4>(rp[row] + wave * GL::GPW + grpL, rp[row + 1], VW * GL::GPW, p0L, ci, va, bin,
                                    acc, ld);
#pragma unroll
        for (int o = GL::LPR; o < 64; o <<= 1)
#pragma unroll
            for (int e = 0; e < GL::VEC; ++e) acc[e] += kt::shfl_xor(acc[e], o);
        if (grpL == 0)
#pragma unroll
            for (int e = 0; e < GL::VEC; ++e) lsum[wave][p0L + e] = acc[e];
        __syncthreads();
        double sb = 0.0, sf = 0.0;
        if (wave == 0) {
            if (grpL == 0) {
                double t[GL::VEC], fo[GL::VEC], bo[GL::VEC];
#pragma unroll
                for (int e = 0; e < GL::VEC; ++e) {
                    t[e] = lsum[0][p0L + e];
#pragma unroll
                    for (int w = 1; w < VW; ++w) t[e] += lsum[w][p0L + e];
                }
                expmv_row_prefetch<GL::VEC>(row, p0L, nc, ld, mu, bin, F, fo, bo);
                expmv_row_update<GL::VEC, false>(row, p0L, t, fo, bo, nc, ld, mu, coef, bout, F, sb, sf);
            }
            fold(sb, sf, GL::LPR);
        }
        __syncthreads();  // lsum is rewritten by the next heavy row
    }
    // (1) the other long rows: the fused kernel's 4 waves as 4 chain sets in
    //     turn in one wave (4 deep: the first chain entry of every set is
    //     issued before the butterfly of the previous one is needed)
    for (int li = n_heavy + gw; li < n_long; li += TW) {
        const int row = long_rows[li];
        const int beg = rp[row], end = rp[row + 1];
        double s[GL::VEC];
#pragma unroll 1
        for (int w = 0; w < VW; ++w) {
            double acc[GL::VEC];
#pragma unroll
            for (int e = 0; e < GL::VEC; ++e) acc[e] = 0.0;
            row_gather8<P, FLAGS, GL, 4>(beg + w * GL::GPW + grpL, end, VW * GL::GPW, p0L, ci, va, bin, acc, ld);
#pragma unroll
            for (int o = GL::LPR; o < 64; o <<= 1)
#pragma unroll
                for (int e = 0; e < GL::VEC; ++e) acc[e] += kt::shfl_xor(acc[e], o);
#pragma unroll
            for (int e = 0; e < GL::VEC; ++e) s[e] = w == 0 ? acc[e] : s[e] + acc[e];
        }
        double sb = 0.0, sf = 0.0;
        if (grpL == 0) {
            double fo[GL::VEC], bo[GL::VEC];
            expmv_row_prefetch<GL::VEC>(row, p0L, nc, ld, mu, bin, F, fo, bo);
            expmv_row_update<GL::VEC, false>(row, p0L, s, fo, bo, nc, ld, mu, coef, bout, F, sb, sf);
        }
        fold(sb, sf, GL::LPR);
    }
    // (2) medium rows: one wave per row (16 chains; with MD = 4 a row of
    //     degree <= 64 is one round), pipelined: while row mi gathers, the
    //     chain columns of row mi + TW and the task of row mi + 2 TW are in
    //     flight
    constexpr int MD = 4;
    auto load_mtask = [&](int ii, int& r, int& bg, int& en) {
        r = -1;
        bg = en = 0;
        if (ii < n_med) {
            const int4 v = med_tasks[ii];
            r = v.x;
            bg = v.y;
            en = v.z;
        }
    };
    auto load_mchunk = [&](int bg, int en, int* c) {  // this lane group's first MD chain entries
        const int k0 = bg + grpL;
        const int c0 = k0 < en ? ld_stream<FLAGS>(ci + k0) : 0;
        c[0] = c0;
#pragma unroll
        for (int i = 1; i < MD; ++i) c[i] = (k0 + i * GL::GPW < en) ? ld_stream<FLAGS>(ci + k0 + i * GL::GPW) : c0;
    };
    {
        // mu = 0: the row's own f is loaded one row ahead too (lane group 0)
        auto load_mf = [&](int r, double* f) {
#pragma unroll
            for (int e = 0; e < GL::VEC; ++e) {
                const int c = p0L + e;
                f[e] = (MU0 && grpL == 0 && r >= 0 && c < nc) ? F[(int64_t)r * ld + c] : 0.0;
            }
        };
        int mi = gw;
        int row, beg, end, nrow, nbeg, nend;
        load_mtask(mi, row, beg, end);
        int mc[MD];
        load_mchunk(beg, end, mc);
        double mfc[GL::VEC];
        load_mf(row, mfc);
        load_mtask(mi + TW, nrow, nbeg, nend);
        for (; mi < n_med; mi += TW) {
            int nnrow, nnbeg, nnend;
            load_mtask(mi + 2 * TW, nnrow, nnbeg, nnend);
            int mn[MD];
            load_mchunk(nbeg, nend, mn);
            double mfn[GL::VEC];
            load_mf(nrow, mfn);
            using VL = VecT<GL::VEC>;
            double s[GL::VEC];
#pragma unroll
            for (int e = 0; e < GL::VEC; ++e) s[e] = 0.0;
            const int k0 = beg + grpL;
            {
                double a[(FLAGS & KF_UNIT) ? 1 : MD];
                if constexpr (!(FLAGS & KF_UNIT)) {
#pragma unroll
                    for (int i = 0; i < MD; ++i)
                        a[i] = (k0 + i * GL::GPW < end) ? ld_stream<FLAGS>(va + k0 + i * GL::GPW) : 0.0;
                }
                typename VL::T x[MD];
#pragma unroll
                for (int i = 0; i < MD; ++i) x[i] = VL::load(bin + (int64_t)mc[i] * ld + p0L);
#pragma unroll
                for (int i = 0; i < MD; ++i)
#pragma unroll
                    for (int e = 0; e < GL::VEC; ++e) {
                        if constexpr (FLAGS & KF_UNIT)
                            s[e] = (k0 + i * GL::GPW < end) ? s[e] + VL::get(x[i], e) : s[e];
                        else s[e] = fma(a[i], VL::get(x[i], e), s[e]);
                    }
            }
            // (rows longer than 16 MD: the rest of each chain, same order)
            row_gather8<P, FLAGS, GL, MD>(k0 + MD * GL::GPW, end, GL::GPW, p0L, ci, va, bin, s, ld);
#pragma unroll
            for (int o = GL::LPR; o < 64; o <<= 1)
#pragma unroll
                for (int e = 0; e < GL::VEC; ++e) s[e] += kt::shfl_xor(s[e], o);
            double sb = 0.0, sf = 0.0;
            if (grpL == 0) {
                double fo[GL::VEC], bo[GL::VEC];
                if constexpr (MU0) {
#pragma unroll
                    for (int e = 0; e < GL::VEC; ++e) fo[e] = mfc[e];
                } else {
                    expmv_row_prefetch<GL::VEC>(row, p0L, nc, ld, mu, bin, F, fo, bo);
                }
                expmv_row_update<GL::VEC, false>(row, p0L, s, fo, bo, nc, ld, mu, coef, bout, F, sb, sf);
            }
            fold(sb, sf, GL::LPR);
#pragma unroll
            for (int e = 0; e < GL::VEC; ++e) mfc[e] = mfn[e];
            row = nrow;
            beg = nbeg;
            end = nend;
            nrow = nnrow;
            nbeg = nnbeg;
            nend = nnend;
#pragma unroll
            for (int i = 0; i < MD; ++i) mc[i] = mn[i];
        }
    }
    constexpr int SD = 8;            // short rows: gathers in flight per row group
    // short rows: column indices loaded one block ahead (all 16 of a short
    // row measured equal to 8: 1,070-1,076 vs 1,067-1,070 ms per warm
    // trace_exp, profiles/r06/expmv_rows_ab)
    constexpr int SCOL = 8;
    // (3) short rows, in the task list's order (degree-descending, so the
    //     GPW rows of a wave take the same number of gather rounds), GPW
    //     tasks per wave, software-pipelined: while block b gathers, the
    //     first SCOL column indices of block b + TW (every column of a short
    //     row at SCOL = 16) and the tasks of block b + 2 TW are in flight
    const int nblk = (n_short + G::GPW - 1) / G::GPW;
    auto load_task = [&](int bb, int& r, int& bg, int& en) {
        const int t = bb * G::GPW + grp;
        r = -1;
        bg = en = 0;
        if (bb < nblk && t < n_short) {
            const int4 v = short_tasks[t];
            r = v.x;
            bg = v.y;
            en = v.z;
        }
    };
    auto load_chunk = [&](int bg, int en, int* c) {  // a row's first SCOL columns (tail: its first)
        const int c0 = bg < en ? ld_stream<FLAGS>(ci + bg) : 0;
        c[0] = c0;
#pragma unroll
        for (int i = 1; i < SCOL; ++i) c[i] = (bg + i < en) ? ld_stream<FLAGS>(ci + bg + i) : c0;
    };
    // mu = 0: the rows' own f is loaded one block ahead too
    auto load_f = [&](int r, double* f) {
#pragma unroll
        for (int e = 0; e < G::VEC; ++e) {
            const int c = p0 + e;
            f[e] = (MU0 && r >= 0 && c < nc) ? F[(int64_t)r * ld + c] : 0.0;
        }
    };
    int b = gw;
    int row, beg, end, nrow, nbeg, nend;
    load_task(b, row, beg, end);
    int cc[SCOL];
    load_chunk(beg, end, cc);
    double fc[G::VEC];
    load_f(row, fc);
    load_task(b + TW, nrow, nbeg, nend);
    for (; b < nblk; b += TW) {
        int nnrow, nnbeg, nnend;
        load_task(b + 2 * TW, nnrow, nnbeg, nnend);
        int cn[SCOL];
        load_chunk(nbeg, nend, cn);
        double fn[G::VEC];
        load_f(nrow, fn);
        double sb = 0.0, sf = 0.0;
        if (row >= 0) {
            using VV = VecT<G::VEC>;
            double s[G::VEC], fo[G::VEC], bo[G::VEC];
#pragma unroll
            for (int e = 0; e < G::VEC; ++e) s[e] = 0.0;
            // the prefetched columns in rounds of SD gathers, then (rows longer
            // than SCOL) the rest as row_gather8 -- one chain in CSR order
#pragma unroll
            for (int h = 0; h < SCOL / SD; ++h) {
                const int k0 = beg + h * SD;
                if (h > 0 && k0 >= end) break;
                // unit weights: fma(1, x, s) = s + x and fma(0, x, s) = s (a
                // masked tail entry), so the weights are predicates, not registers
                double a[(FLAGS & KF_UNIT) ? 1 : SD];
                if constexpr (!(FLAGS & KF_UNIT)) {
#pragma unroll
                    for (int i = 0; i < SD; ++i) a[i] = (k0 + i < end) ? ld_stream<FLAGS>(va + k0 + i) : 0.0;
                }
                typename VV::T x[SD];
#pragma unroll
                for (int i = 0; i < SD; ++i) x[i] = VV::load(bin + (int64_t)cc[h * SD + i] * ld + p0);
#pragma unroll
                for (int i = 0; i < SD; ++i)
#pragma unroll
                    for (int e = 0; e < G::VEC; ++e) {
                        if constexpr (FLAGS & KF_UNIT) s[e] = (k0 + i < end) ? s[e] + VV::get(x[i], e) : s[e];
                        else s[e] = fma(a[i], VV::get(x[i], e), s[e]);
                    }
            }
            row_gather8<P, FLAGS, G, SD>(beg + SCOL, end, 1, p0, ci, va, bin, s, ld);
            if constexpr (MU0) {
#pragma unroll
                for (int e = 0; e < G::VEC; ++e) fo[e] = fc[e];
            } else {
                expmv_row_prefetch<G::VEC>(row, p0, nc, ld, mu, bin, F, fo, bo);
            }
            expmv_row_update<G::VEC, false>(row, p0, s, fo, bo, nc, ld, mu, coef, bout, F, sb, sf);
        }
        fold(sb, sf, G::LPR);
#pragma unroll
        for (int e = 0; e < G::VEC; ++e) fc[e] = fn[e];
        row = nrow;
        beg = nbeg;
        end = nend;
        nrow = nnrow;
        nbeg = nnbeg;
        nend = nnend;
#pragma unroll
        for (int i = 0; i < SCOL; ++i) cc[i] = cn[i];
    }
    // (4) this workgroup's maxima into slot blockIdx % 64 of set k % 3
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        mb = fmax(mb, kt::shfl_xor(mb, o));
        mf = fmax(mf, kt::shfl_xor(mf, o));
    }
    if (lane == 0) {
        red[0][wave] = mb;
        red[1][wave] = mf;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double x = red[0][0], y = red[1][0];
#pragma unroll
        for (int w = 1; w < WAVES; ++w) {
            x = fmax(x, red[0][w]);
            y = fmax(y, red[1][w]);
        }
        unsigned long long* slot = st->term_max[k % 3][blockIdx.x % kTermSlots];
        __hip_atomic_fetch_max(slot, (unsigned long long)__double_as_longlong(x), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_max(slot + 1, (unsigned long long)__double_as_longlong(y), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }
}

// The check of term k (expmv.m:79-82) for the SPLIT term kernel, one wave:
// c2 / nf = the maxima in the 64 slots of set k % 3, c1 = st->c1s[k & 1];
// stop: active = 0 (and the host flag); else c1s[(k + 1) & 1] = c2.  Zeroes
// set (k + 1) % 3 for term k + 1 (its last reader was the check of term k - 2).
__global__ __launch_bounds__(64) void k_expmv_slot_check(ExpmvState* st, int k, double tol, int* hflag,
                                                         int stage) {
    const int lane = threadIdx.x;
    st->term_max[(k + 1) % 3][lane][0] = 0ull;
    st->term_max[(k + 1) % 3][lane][1] = 0ull;
    if (!st->active) return;
    unsigned long long mb = st->term_max[k % 3][lane][0], mf = st->term_max[k % 3][lane][1];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long xb = kt::shfl_xor(mb, o), xf = kt::shfl_xor(mf, o);
        mb = xb > mb ? xb : mb;
        mf = xf > mf ? xf : mf;
    }
    if (lane != 0) return;
    const double c1 = st->c1s[k & 1];
    const double c2 = __longlong_as_double((long long)mb), nf = __longlong_as_double((long long)mf);
    if (c1 + c2 <= tol * nf) {
        st->active = 0;
        if (hflag) __hip_atomic_store(hflag, stage, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    } else {
        st->c1s[(k + 1) & 1] = c2;
    }
}

// mv = mv + 1; c2 = norm(b, inf); if c1 + c2 <= tol*norm(f, inf) break; c1 = c2   (:76-82)
__global__ __launch_bounds__(256) void k_expmv_check(const double* __restrict__ partial, int nb,
                                                     double tol, ExpmvState* st) {
    if (!st->active) return;
    double mb = 0.0, mf = 0.0;
    for (int i = threadIdx.x; i < nb; i += blockDim.x) {
        mb = fmax(mb, partial[i]);
        mf = fmax(mf, partial[nb + i]);
    }
    for (int o = 32; o > 0; o >>= 1) {
        mb = fmax(mb, kt::shfl_xor(mb, o));
        mf = fmax(mf, kt::shfl_xor(mf, o));
    }
    __shared__ double red[2][4];
    if ((threadIdx.x & 63) == 0) {
        red[0][threadIdx.x >> 6] = mb;
        red[1][threadIdx.x >> 6] = mf;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const double c2 = fmax(fmax(red[0][0], red[0][1]), fmax(red[0][2], red[0][3]));
        const double nf = fmax(fmax(red[1][0], red[1][1]), fmax(red[1][2], red[1][3]));
        st->mv += 1;
        if (st->c1 + c2 <= tol * nf) st->active = 0;
        else st->c1 = c2;
    }
}

}  // namespace kt

// ---------------------------------------------------------------------------
// host-side launchers (C++ linkage, used by the runtime)
// ---------------------------------------------------------------------------
#include "kt_launch.h"

namespace kt {

static constexpr int kBlock = 512;

int long_blocks_for(int n_long, int max_blocks) {
    const int waves = kBlock / 64;
    int b = (n_long + waves - 1) / waves;
    return b < max_blocks ? b : max_blocks;
}

int spmm_grid(int n, int P, int max_blocks) {
    const int gpw = (P >= 2) ? 64 / (P / 2) : 64;
    const int rows_per_block = (kBlock / 64) * gpw;
    int g = (n + rows_per_block - 1) / rows_per_block;
    if (g > max_blocks) g = max_blocks;
    if (g < 1) g = 1;
    return g;
}

template <class F>
static hipError_t dispatch_p(int P, F&& f) {
    switch (P) {
    case 1: f(std::integral_constant<int, 1>{}); break;
    case 2: f(std::integral_constant<int, 2>{}); break;
    case 4: f(std::integral_constant<int, 4>{}); break;
    case 8: f(std::integral_constant<int, 8>{}); break;
    case 16: f(std::integral_constant<int, 16>{}); break;
    case 32: f(std::integral_constant<int, 32>{}); break;
    case 64: f(std::integral_constant<int, 64>{}); break;
    case 128: f(std::integral_constant<int, 128>{}); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_rademacher(int P, int n, uint64_t seed, int64_t probe_base, const int* perm,
                             double* X, hipStream_t st) {
    int64_t total = (int64_t)n * P;
    int grid = (int)((total + 255) / 256);
    if (grid > 8192) grid = 8192;
    if (grid < 1) grid = 1;
    return dispatch_p(P, [&](auto c) {
        k_rademacher<decltype(c)::value><<<grid, 256, 0, st>>>(n, seed, probe_base, perm, X);
    });
}

hipError_t launch_rademacher_cols(int n, int ncols, uint64_t seed, int64_t probe_base, double* X, int ldx,
                                  hipStream_t st) {
    if (ncols < 1 || ncols > 64 || ldx < ncols) return hipErrorInvalidValue;
    int64_t total = (int64_t)n * ncols;
    int grid = (int)((total + 255) / 256);
    if (grid > 8192) grid = 8192;
    if (grid < 1) grid = 1;
    k_rademacher_cols<<<grid, 256, 0, st>>>(n, ncols, seed, probe_base, X, ldx);
    return hipGetLastError();
}

hipError_t launch_spmm_dot(int P, int flags, int grid, const int* rp, const int* ci,
                           const double* va, int n, const double* ucur, const double* sc,
                           double* y, double* partial, const int* long_rows, int n_long,
                           int long_thresh, int long_blocks, hipStream_t st) {
    return dispatch_p(P, [&](auto c) {
        constexpr int PP = decltype(c)::value;
#define KT_K1(F)                                                                              \
    k_spmm_dot<PP, kBlock, F><<<grid, kBlock, 0, st>>>(rp, ci, va, n, ucur, sc, y, partial,      \
                                                       long_rows, n_long, long_thresh, long_blocks)
        switch (flags & 15) {
        case 0: KT_K1(0); break;
        case KF_UNIT: KT_K1(KF_UNIT); break;
        case KF_NT: KT_K1(KF_NT); break;
        case KF_NT | KF_UNIT: KT_K1(KF_NT | KF_UNIT); break;
        case KF_NTY | KF_UNIT: KT_K1(KF_NTY | KF_UNIT); break;
        case KF_NT | KF_NTY | KF_UNIT: KT_K1(KF_NT | KF_NTY | KF_UNIT); break;
        case KF_MLP: KT_K1(KF_MLP); break;
        case KF_MLP | KF_UNIT: KT_K1(KF_MLP | KF_UNIT); break;
        case KF_MLP | KF_NTY | KF_UNIT: KT_K1(KF_MLP | KF_NTY | KF_UNIT); break;
        default:  // unsupported combination: keep only the unit bit (exactness)
            if (flags & KF_UNIT) KT_K1(KF_UNIT);
            else KT_K1(0);
            break;
        }
#undef KT_K1
    });
}

hipError_t launch_spmm_block(int P, int flags, int grid, const CsrView& M, const double* X, int ldx,
                             double* Y, int ldy, int long_blocks, int chunk_blocks, double* ck_part,
                             hipStream_t st, int slices, const int* skip) {
    const dim3 g(grid, slices);
    hipError_t e = dispatch_p(P, [&](auto c) {
        constexpr int PP = decltype(c)::value;
#define KT_SB(F)                                                                                   \
    k_spmm_block<PP, kBlock, F><<<g, kBlock, 0, st>>>(                                              \
        M.rp, M.ci, M.va, M.n, X, ldx, Y, ldy, M.long_rows, M.n_long, M.long_thresh, long_blocks, skip, \
        M.ck_beg, M.ck_end, M.n_chunks, chunk_blocks, M.split_thresh, ck_part)
        switch (flags & (KF_UNIT | KF_MLP)) {
        case 0: KT_SB(0); break;
        case KF_UNIT: KT_SB(KF_UNIT); break;
        case KF_MLP: KT_SB(KF_MLP); break;
        default: KT_SB(KF_UNIT | KF_MLP); break;
        }
#undef KT_SB
    });
    if (e != hipSuccess || M.n_split == 0 || chunk_blocks == 0) return e;
    return dispatch_p(P, [&](auto c) {
        constexpr int PP = decltype(c)::value;
        k_spmm_combine<PP><<<dim3(M.n_split, slices), 128, 0, st>>>(M.sp_rows, M.sp_first, M.n_chunks, ck_part,
                                                                    Y, ldy, skip);
    });
}

hipError_t launch_coef_cgs2(int P, const double* partial, int nblk, int first, const double* k2s,
                            const double* sc, const double* sp, double* coef, double* t_alpha,
                            double* t_up, double* hist, hipStream_t st) {
    return dispatch_p(P, [&](auto c) {
        constexpr int PP = decltype(c)::value;
        k_coef_cgs2<PP><<<(PP + 3) / 4, 256, 0, st>>>(partial, nblk, first, k2s, sc, sp, coef,
                                                      t_alpha, t_up, hist);
    });
}

hipError_t launch_update(int P, int grid, int n, const double* y, double* uprev,
                         const double* ucur, const double* sc, const double* sp,
                         const double* coef, int first, double* partial, hipStream_t st, bool nt,
                         double* rec, int bcols) {
    return dispatch_p(P, [&](auto c) {
        if (nt)
            k_update<decltype(c)::value, kBlock, true><<<grid, kBlock, 0, st>>>(
                n, y, uprev, ucur, sc, sp, coef, first, partial, rec, bcols);
        else
            k_update<decltype(c)::value, kBlock, false><<<grid, kBlock, 0, st>>>(
                n, y, uprev, ucur, sc, sp, coef, first, partial, rec, bcols);
    });
}

hipError_t launch_norm(int P, const double* partial, int nblk, double* k2s, double* scale_next,
                       double* t_low, hipStream_t st) {
    return dispatch_p(P, [&](auto c) {
        constexpr int PP = decltype(c)::value;
        k_norm<PP><<<(3 * PP + 3) / 4, 256, 0, st>>>(partial, nblk, k2s, scale_next, t_low);
    });
}


hipError_t launch_spmm_lanczos(int P, int flags, int grid, const int* rp, const int* ci,
                               const double* va, int n, const double* X, const double* Yold,
                               double* Out, const double* coef, double* partial,
                               const int* long_rows, int n_long, int long_thresh, int long_blocks,
                               hipStream_t st, const double* Vc, const double* Vo, double* Vn, int bcols) {
    return dispatch_p(P, [&](auto c) {
        constexpr int PP = decltype(c)::value;
#define KT_KY(F)                                                                                   \
    k_spmm_lanczos<PP, kBlock, F><<<grid, kBlock, 0, st>>>(rp, ci, va, n, X, Yold, Out, coef, partial, \
                                                           long_rows, n_long, long_thresh, long_blocks, \
                                                           Vc, Vo, Vn, bcols)
        if (Vn) {  // the basis-forming pass (KF_VB)
            if (flags & KF_UNIT) {
                if (flags & KF_SC1) KT_KY(KF_UNIT | KF_SC1 | KF_VB);
                else KT_KY(KF_UNIT | KF_VB);
            } else {
                if (flags & KF_SC1) KT_KY(KF_SC1 | KF_VB);
                else KT_KY(KF_VB);
            }
            return;
        }
        switch (flags & (KF_UNIT | KF_NTY | KF_SC1)) {
        case 0: KT_KY(0); break;
        case KF_UNIT: KT_KY(KF_UNIT); break;
        case KF_NTY: KT_KY(KF_NTY); break;
        case KF_UNIT | KF_NTY: KT_KY(KF_UNIT | KF_NTY); break;
        case KF_SC1:
        case KF_SC1 | KF_NTY: KT_KY(KF_SC1); break;
        default: KT_KY(KF_UNIT | KF_SC1); break;
        }
#undef KT_KY
    });
}

hipError_t launch_rademacher_signs(int P, int n, uint64_t seed, int64_t probe_base,
                                  const int* perm, uint32_t* S, hipStream_t st) {
    const int64_t total = (int64_t)n * ((P + 31) / 32);
    int grid = (int)((total + 255) / 256);
    if (grid > 8192) grid = 8192;
    if (grid < 1) grid = 1;
    return dispatch_p(P, [&](auto c) {
        k_rademacher_signs<decltype(c)::value><<<grid, 256, 0, st>>>(n, seed, probe_base, perm, S);
    });
}

hipError_t launch_spmm_lanczos_start(int P, int flags, int grid, const int* rp, const int* ci,
                                     const double* va, int n, const uint32_t* S, double s0,
                                     double* Out, double* partial, const int* long_rows, int n_long,
                                     int long_thresh, int long_blocks, hipStream_t st) {
    return dispatch_p(P, [&](auto c) {
        constexpr int PP = decltype(c)::value;
#define KT_KS(F)                                                                                 \
    k_spmm_lanczos_start<PP, kBlock, F><<<grid, kBlock, 0, st>>>(rp, ci, va, n, S, s0, Out, partial, \
                                                                 long_rows, n_long, long_thresh,  \
                                                                 long_blocks)
        switch (flags & (KF_UNIT | KF_NTY | KF_SC1)) {
        case 0: KT_KS(0); break;
        case KF_UNIT: KT_KS(KF_UNIT); break;
        case KF_NTY: KT_KS(KF_NTY); break;
        case KF_UNIT | KF_NTY: KT_KS(KF_UNIT | KF_NTY); break;
        case KF_SC1:
        case KF_SC1 | KF_NTY: KT_KS(KF_SC1); break;
        default: KT_KS(KF_UNIT | KF_SC1); break;
        }
#undef KT_KS
    });
}

hipError_t launch_ycoef(int P, const double* partial, int nblk, int start, int last, double s0,
                        double* ys, double* t_alpha, double* t_up, double* t_low, double* guard,
                        hipStream_t st) {
    return dispatch_p(P, [&](auto c) {
        constexpr int PP = decltype(c)::value;
        k_ycoef<PP><<<PP, 192, 0, st>>>(partial, nblk, start, last, s0, ys, t_alpha, t_up, t_low,
                                        guard);
    });
}

static int stream_grid(int64_t total) {
    int64_t g = (total + 255) / 256;
    if (g > 4096) g = 4096;
    return g < 1 ? 1 : (int)g;
}

hipError_t launch_weighted_sum(int n, int m, int P, int nc, const double* U, int ldu, int64_t sstride,
                               const double* W, double* Y, int ldy, hipStream_t st) {
    k_weighted_sum<<<stream_grid((int64_t)n * nc), 256, 0, st>>>(n, m, P, nc, U, ldu, sstride, W, Y, ldy);
    return hipGetLastError();
}

hipError_t launch_perm_rows(int n, int cols, const int* perm, int gather, const double* src, int lds,
                            double* dst, int ldd, hipStream_t st) {
    if (n <= 0 || cols <= 0) return hipSuccess;
    k_perm_rows<<<stream_grid((int64_t)n * cols), 256, 0, st>>>(n, cols, perm, gather, src, lds, dst, ldd);
    return hipGetLastError();
}

hipError_t launch_axpby(int n, int nc, double a, const double* X, int ldx, double b, double* Y,
                        int ldy, hipStream_t st) {
    k_axpby<<<stream_grid((int64_t)n * nc), 256, 0, st>>>(n, nc, a, X, ldx, b, Y, ldy);
    return hipGetLastError();
}

int inf_norm_blocks() { return 1024; }

hipError_t launch_inf_norm(int n, int nc, const double* X, int ldx, double* partial,
                           hipStream_t st) {
    k_inf_norm<<<inf_norm_blocks(), 256, 0, st>>>(n, nc, X, ldx, partial);
    return hipGetLastError();
}

// one row per thread: no idle blocks on small matrices (the check reduces
// only these partials)
static int expmv_term_blocks(int n) {
    const int b = (n + 255) / 256;
    return b < 1 ? 1 : (b > inf_norm_blocks() ? inf_norm_blocks() : b);
}

hipError_t launch_expmv_begin(const double* partial, int nb, void* state, hipStream_t st) {
    k_expmv_begin<<<1, 256, 0, st>>>(partial, nb, static_cast<ExpmvState*>(state));
    return hipGetLastError();
}

hipError_t launch_expmv_term(int n, int nc, double mu, double coef, const double* Ab, double* b,
                             double* F, int ld, double* partial, const void* state, hipStream_t st) {
    k_expmv_term<<<expmv_term_blocks(n), 256, 0, st>>>(n, nc, mu, coef, Ab, b, F, ld, partial,
                                                       static_cast<const ExpmvState*>(state));
    return hipGetLastError();
}

hipError_t launch_expmv_check(int n, const double* partial, double tol, void* state, hipStream_t st) {
    k_expmv_check<<<1, 256, 0, st>>>(partial, expmv_term_blocks(n), tol, static_cast<ExpmvState*>(state));
    return hipGetLastError();
}

size_t expmv_state_bytes() { return sizeof(ExpmvState); }

int expmv_step_blocks(int n, int P, int n_long, int n_med, int waves) {
    if (waves <= 0) waves = kExpmvWaves;
    const int gpw = (P >= 2) ? 64 / (P / 2) : 64;
    return n_long + (n_med + waves - 1) / waves + (n + waves * gpw - 1) / (waves * gpw);
}

bool expmv_split_check(int n, int P, int n_long, int n_med) {
    return expmv_step_blocks(n, P, n_long, n_med) > kExpmvSplitBlocks;
}

hipError_t launch_expmv_slot_check(void* state, int k, double tol, hipStream_t st, int* hflag, int stage) {
    k_expmv_slot_check<<<1, 64, 0, st>>>(static_cast<ExpmvState*>(state), k, tol, hflag, stage);
    return hipGetLastError();
}

// form: 0 fused, 1 split (a workgroup per long row / 4 medium rows / 32 short
// rows), 2 row-blocked split (k_expmv_rows, resident workgroups)
static int expmv_rows_grid(int n_tasks_hint) {
    static int per_cu = 0, cus = 0;
    if (!per_cu) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        int occ = 0;
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_expmv_rows<16, KF_UNIT | KF_MU0, true>,
                                                           64 * kExpmvRowsWaves, 0);
        per_cu = occ > 0 ? occ : 2;
        if (cus <= 0) cus = 256;
    }
    int g = per_cu * cus;
    if (g > n_tasks_hint) g = n_tasks_hint;
    return g < 1 ? 1 : g;
}

hipError_t launch_expmv_step(int P, bool unit, const CsrView& M, const int* med_rows, int n_med, int nc,
                             int ld, double mu, double coef, double tol, int k, const double* bin,
                             double* bout, double* F, void* state, hipStream_t st, int form, int* hflag,
                             int stage) {
    ExpmvState* s = static_cast<ExpmvState*>(state);
    if ((form == 2 || form == 3) && !(M.short_tasks && M.med_tasks)) form = 1;  // no task lists: the split kernel
    if (form == 2 || form == 3) {
        const bool fused_check = form == 3;
        // KT_EXPMV_CLASSES (timing diagnostics only; the results are WRONG):
        // bit mask of the row classes the term processes, 1 long, 2 medium, 4 short
        static const int classes = [] {
            const char* e = std::getenv("KT_EXPMV_CLASSES");
            return e ? std::atoi(e) : 7;
        }();
        const int nl = (classes & 1) ? M.n_long : 0, nh = (classes & 1) ? M.n_heavy : 0, nm = (classes & 2) ? n_med : 0,
                  ns = (classes & 4) ? M.n_short : 0;
        // no more waves than tasks (long rows, medium rows, blocks of 8 short rows)
        const int tasks = nl + nm + (ns + 7) / 8;
        const int grid = expmv_rows_grid((tasks + kExpmvRowsWaves - 1) / kExpmvRowsWaves);
#define KT_EXPMV_ROWS(PP, F_)                                                                      \
    if (fused_check)                                                                               \
        k_expmv_rows<PP, F_, true><<<grid, 64 * kExpmvRowsWaves, 0, st>>>(M.rp, M.ci, M.va, M.n, M.long_rows, \
            nl, nh, reinterpret_cast<const int4*>(M.med_tasks), nm, reinterpret_cast<const int4*>(M.short_tasks), \
            ns, nc, ld, mu, coef, k, bin, bout, F, s, tol, hflag, stage);                          \
    else                                                                                           \
        k_expmv_rows<PP, F_, false><<<grid, 64 * kExpmvRowsWaves, 0, st>>>(M.rp, M.ci, M.va, M.n, M.long_rows, \
            nl, nh, reinterpret_cast<const int4*>(M.med_tasks), nm, reinterpret_cast<const int4*>(M.short_tasks), \
            ns, nc, ld, mu, coef, k, bin, bout, F, s, tol, hflag, stage)
#define KT_EXPMV_ROWS_P(PP)                                                                        \
    if (mu == 0.0) {                                                                               \
        if (unit) KT_EXPMV_ROWS(PP, KF_UNIT | KF_MU0);                                             \
        else KT_EXPMV_ROWS(PP, KF_MU0);                                                            \
    } else {                                                                                       \
        if (unit) KT_EXPMV_ROWS(PP, KF_UNIT);                                                      \
        else KT_EXPMV_ROWS(PP, 0);                                                                 \
    }
        switch (P) {
        case 1: KT_EXPMV_ROWS_P(1) break;
        case 2: KT_EXPMV_ROWS_P(2) break;
        case 4: KT_EXPMV_ROWS_P(4) break;
        case 8: KT_EXPMV_ROWS_P(8) break;
        case 16: KT_EXPMV_ROWS_P(16) break;
        case 32: KT_EXPMV_ROWS_P(32) break;
        default: return hipErrorInvalidValue;
        }
#undef KT_EXPMV_ROWS_P
#undef KT_EXPMV_ROWS
        return hipGetLastError();
    }
    const bool split = form == 1;
    const int grid = expmv_step_blocks(M.n, P, M.n_long, n_med);
#define KT_EXPMV_LAUNCH(PP, F_, SP)                                                                \
    k_expmv_step<PP, F_, SP><<<grid, 64 * kExpmvWaves, 0, st>>>(M.rp, M.ci, M.va, M.n, M.long_rows, \
                                                               M.n_long, med_rows, n_med, nc, ld, mu, \
                                                               coef, tol, k, bin, bout, F, s, hflag, stage)
#define KT_EXPMV_STEP(PP)                                                                          \
    if (unit) {                                                                                    \
        if (split) KT_EXPMV_LAUNCH(PP, KF_UNIT, true);                                             \
        else KT_EXPMV_LAUNCH(PP, KF_UNIT, false);                                                  \
    } else {                                                                                       \
        if (split) KT_EXPMV_LAUNCH(PP, 0, true);                                                   \
        else KT_EXPMV_LAUNCH(PP, 0, false);                                                        \
    }
    switch (P) {
    case 1: KT_EXPMV_STEP(1) break;
    case 2: KT_EXPMV_STEP(2) break;
    case 4: KT_EXPMV_STEP(4) break;
    case 8: KT_EXPMV_STEP(8) break;
    case 16: KT_EXPMV_STEP(16) break;
    case 32: KT_EXPMV_STEP(32) break;
    default: return hipErrorInvalidValue;
    }
#undef KT_EXPMV_STEP
#undef KT_EXPMV_LAUNCH
    return hipGetLastError();
}

hipError_t launch_gather_rows(int nr, int cols, const double* D, int ldd, const int64_t* rows, double* out,
                              hipStream_t st) {
    k_gather_rows<<<stream_grid((int64_t)nr * cols), 256, 0, st>>>(nr, cols, D, ldd, rows, out);
    return hipGetLastError();
}

hipError_t launch_gather_elems(int64_t count, const double* D, const int64_t* off, double* out,
                               hipStream_t st) {
    if (count <= 0) return hipSuccess;
    k_gather_elems<<<stream_grid(count), 256, 0, st>>>(count, D, off, out);
    return hipGetLastError();
}

hipError_t launch_scatter_elems(int64_t count, const int64_t* off, const double* val, double* D,
                                hipStream_t st) {
    if (count <= 0) return hipSuccess;
    k_scatter_elems<<<stream_grid(count), 256, 0, st>>>(count, off, val, D);
    return hipGetLastError();
}

int normest1_blocks(int n) {
    const int b = (n + 255) / 256;
    return b < 1 ? 1 : (b > 1024 ? 1024 : b);
}

hipError_t launch_normest1_y(int n, const double* Y, const double* Sprev, double* S, double* partial,
                             hipStream_t st) {
    k_normest1_y<<<normest1_blocks(n), 256, 0, st>>>(n, Y, Sprev, S, partial);
    return hipGetLastError();
}

hipError_t launch_absmax_idx(int n, const double* Z, double* pval, int* pidx, hipStream_t st) {
    k_absmax_idx<<<normest1_blocks(n), 256, 0, st>>>(n, Z, pval, pidx);
    return hipGetLastError();
}

// Start scales of a sweep seeded by a device block, from the columns'
// squared norms n2 (device, nc of them; zero norm: a zero column):
//   mode 0 (explicit sweep): a = sc[P] = 1/||x_c||, b = k2s[P] = ||x_c||^2;
//   mode 1 (y-form sweep):   a = ys[9P] = [1/||x_c|| | 0 (5P) | 1 (P) | 0 (2P)]
// so the sweep is queued without the host reading the norms first.
__global__ __launch_bounds__(256) void k_sweep_scales(const double* __restrict__ n2, int nc, int P, int mode,
                                                      double* __restrict__ a, double* __restrict__ b) {
    for (int t = threadIdx.x; t < (mode ? 9 * P : P); t += blockDim.x) {
        const int c = t % P, q = t / P;
        const double v = c < nc ? n2[c] : 0.0;
        const double s = v > 0.0 ? 1.0 / sqrt(v) : 0.0;
        if (mode == 0) {
            a[t] = s;
            b[t] = v > 0.0 ? v : 0.0;
        } else {
            a[t] = q == 0 ? s : (q == 6 ? 1.0 : 0.0);
        }
    }
}

// n2[c] = G[c + c ld] (the diagonal of a Gram block)
__global__ __launch_bounds__(64) void k_gram_diag(const double* __restrict__ G, int ld, int nc,
                                                  double* __restrict__ n2) {
    for (int c = threadIdx.x; c < nc; c += blockDim.x) n2[c] = G[c + (int64_t)c * ld];
}

hipError_t launch_sweep_scales(const double* n2, int nc, int P, int mode, double* a, double* b, hipStream_t st) {
    k_sweep_scales<<<1, 256, 0, st>>>(n2, nc, P, mode, a, b);
    return hipGetLastError();
}

hipError_t launch_gram_diag(const double* G, int ld, int nc, double* n2, hipStream_t st) {
    k_gram_diag<<<1, 64, 0, st>>>(G, ld, nc, n2);
    return hipGetLastError();
}

// test hook (kt_debug_delay): one wave that waits `ticks` of the 100 MHz
// constant clock, so a stream is busy for a known time; every wave exits
__global__ __launch_bounds__(64) void k_delay(long long ticks) {
    const long long t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(64);
}

hipError_t launch_delay(double microseconds, hipStream_t st) {
    const long long ticks = (long long)(microseconds * 100.0);  // 100 MHz
    k_delay<<<1, 64, 0, st>>>(ticks);
    return hipGetLastError();
}

hipError_t launch_fill(double* x, int count, double v, hipStream_t st) {
    int grid = (count + 255) / 256;
    if (grid < 1) grid = 1;
    k_fill<<<grid, 256, 0, st>>>(x, count, v);
    return hipGetLastError();
}

}  // namespace kt

// hub_split.hip -- can the L2 be kept for the hub rows of the probe table?
//
// The y-form pass (k_spmm_lanczos<16>) gathers 128-B probe rows by a
// power-law column stream (Chung-Lu gamma = 2.5, hubs first); the XCD L2
// hit rate is ~11 % although the top 32K rows (4 MB, one L2) carry ~30 % of
// the gathers: the cold rows evict the hub rows under LRU.  This probe times
// the same access pattern (gather 10 rows per output row + own-row read +
// previous-row read + output store, 32 B per lane, 4 lanes per row) with the
// table split in two allocations -- rows < H in ordinary device memory,
// rows >= H in memory of another kind -- to see whether the cold rows can be
// kept out of L2 without losing the Infinity-Cache rate.
//
//   hipcc -O3 --offload-arch=gfx950 hub_split.hip -o hub_split && ./hub_split
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                \
        }                                                                           \
    } while (0)

constexpr int P = 16, VEC = 4, LPR = P / VEC, GPW = 64 / LPR;
typedef double d4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ d4 ld4(const double* p) { return *reinterpret_cast<const d4*>(p); }
__device__ __forceinline__ d4 ld4_nt(const double* p) {
    return __builtin_nontemporal_load(reinterpret_cast<const d4*>(p));
}

// MODE 0: one table; MODE 1: rows >= H from `cold` (split allocation);
// MODE 2: one table, rows >= H loaded nontemporal; MODE 3: columns folded
// into the first H rows (c & (H-1): an L2-resident table, same instruction
// stream); MODE 4: column = row + k - beg (each row gathers its own and the
// next 9 rows: streaming locality, same instruction stream)
template <int MODE, bool STREAMS = true>
__global__ __launch_bounds__(512) void k_probe(const int* __restrict__ rp, const int* __restrict__ col,
                                               int n, int H, const double* __restrict__ hot,
                                               const double* __restrict__ cold,
                                               const double* __restrict__ yold, double* __restrict__ out,
                                               double* __restrict__ part) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int sub = lane % LPR, grp = lane / LPR;
    const int p0 = sub * VEC;
    const int groups = gridDim.x * (blockDim.x / 64) * GPW;
    double acc = 0.0;
    for (int row = (blockIdx.x * (blockDim.x / 64) + wave) * GPW + grp; row < n; row += groups) {
        const int beg = rp[row], end = rp[row + 1];
        d4 s = {0, 0, 0, 0};
        for (int k = beg; k < end; ++k) {
            const int c = col[k];
            d4 x;
            if constexpr (MODE == 0) x = ld4(hot + (int64_t)c * P + p0);
            else if constexpr (MODE == 1)
                x = (c < H) ? ld4(hot + (int64_t)c * P + p0) : ld4(cold + (int64_t)(c - H) * P + p0);
            else if constexpr (MODE == 2)
                x = (c < H) ? ld4(hot + (int64_t)c * P + p0) : ld4_nt(hot + (int64_t)c * P + p0);
            else if constexpr (MODE == 3)
                x = ld4(hot + (int64_t)(c & (H - 1)) * P + p0);
            else
                x = ld4(hot + (int64_t)((row + k - beg + (c & 0)) & (n - 1)) * P + p0);
            s += x;
        }
        if constexpr (!STREAMS) {  // gathers only
            acc += s.x + s.y + s.z + s.w;
            continue;
        }
        const double* own = (MODE == 1 && row >= H) ? cold + (int64_t)(row - H) * P : hot + (int64_t)row * P;
        const d4 xi = ld4(own + p0);
        const d4 yo = ld4_nt(yold + (int64_t)row * P + p0);
        const d4 u = s - 0.5 * xi - 0.25 * yo;
        __builtin_nontemporal_store(u, reinterpret_cast<d4*>(out + (int64_t)row * P + p0));
        acc += u.x * xi.x + u.y * xi.y + u.z * xi.z + u.w * xi.w;
    }
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
    if (lane == 0) part[blockIdx.x * (blockDim.x / 64) + wave] = acc;
}

template <int MODE, bool STREAMS = true>
float run(int grid, const int* rp, const int* col, int n, int H, const double* hot, const double* cold,
          const double* yold, double* out, double* part) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    k_probe<MODE, STREAMS><<<grid, 512>>>(rp, col, n, H, hot, cold, yold, out, part);
    CK(hipEventRecord(a));
    const int reps = 20;
    for (int r = 0; r < reps; ++r) k_probe<MODE, STREAMS><<<grid, 512>>>(rp, col, n, H, hot, cold, yold, out, part);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps * 1e3f;
}

int main() {
    const int n = 1 << 20, deg = 10;
    int num_cu = 0;
    CK(hipDeviceGetAttribute(&num_cu, hipDeviceAttributeMultiprocessorCount, 0));
    // power-law columns (Chung-Lu weights (i+1)^(-2/3), hubs first), 10 per row
    std::vector<double> cdf(n);
    double accw = 0.0;
    for (int i = 0; i < n; ++i) cdf[i] = (accw += std::pow(i + 1.0, -2.0 / 3.0));
    for (auto& c : cdf) c /= accw;
    std::vector<int> hrp(n + 1), hcol((size_t)n * deg);
    uint64_t s = 88172645463325252ull;
    for (int r = 0; r <= n; ++r) hrp[r] = r * deg;
    for (auto& v : hcol) {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        const double u = (double)(s >> 11) * (1.0 / 9007199254740992.0);
        v = std::min((int)(std::lower_bound(cdf.begin(), cdf.end(), u) - cdf.begin()), n - 1);
    }
    int *rp, *col;
    double *hot, *yold, *out, *part;
    const size_t row_bytes = sizeof(double) * P;
    CK(hipMalloc(&rp, sizeof(int) * (n + 1)));
    CK(hipMalloc(&col, sizeof(int) * hcol.size()));
    CK(hipMalloc(&hot, row_bytes * n));
    CK(hipMalloc(&yold, row_bytes * n));
    CK(hipMalloc(&out, row_bytes * n));
    CK(hipMalloc(&part, sizeof(double) * 1 << 20));
    CK(hipMemcpy(rp, hrp.data(), sizeof(int) * (n + 1), hipMemcpyHostToDevice));
    int* rp0;  // every row empty: the own-row / previous-row / output streams alone
    CK(hipMalloc(&rp0, sizeof(int) * (n + 1)));
    CK(hipMemset(rp0, 0, sizeof(int) * (n + 1)));
    CK(hipMemcpy(col, hcol.data(), sizeof(int) * hcol.size(), hipMemcpyHostToDevice));
    CK(hipMemset(hot, 0, row_bytes * n));
    CK(hipMemset(yold, 0, row_bytes * n));
    const int grid = num_cu * 4;
    printf("# n=%d deg=%d P=%d grid=%d (times in us per pass; gathered %.0f MB)\n", n, deg, P, grid,
           (double)n * deg * row_bytes / 1e6);
    printf("single table, plain loads         %8.1f\n",
           run<0>(grid, rp, col, n, 0, hot, nullptr, yold, out, part));
    printf("gathers only (no row streams)      %8.1f\n",
           run<0, false>(grid, rp, col, n, 0, hot, nullptr, yold, out, part));
    printf("H=  1024 folded, gathers only      %8.1f\n",
           run<3, false>(grid, rp, col, n, 1024, hot, nullptr, yold, out, part));
    printf("streams only (deg 0)               %8.1f\n",
           run<3>(grid, rp, col, n, 1024, hot, nullptr, yold, out, part) * 0.0f +
           run<0>(grid, rp0, col, n, 0, hot, nullptr, yold, out, part));
    for (int H : {1024, 8192, 32768, 262144})
        printf("H=%6d  columns folded into rows < H  %8.1f\n", H,
               run<3>(grid, rp, col, n, H, hot, nullptr, yold, out, part));
    printf("neighbouring rows (streaming)      %8.1f\n",
           run<4>(grid, rp, col, n, 0, hot, nullptr, yold, out, part));
    for (int H : {32768}) {
        printf("H=%6d  cold rows nontemporal    %8.1f\n", H,
               run<2>(grid, rp, col, n, H, hot, nullptr, yold, out, part));
        for (unsigned flag : {hipDeviceMallocDefault, hipDeviceMallocFinegrained, hipDeviceMallocUncached}) {
            double* cold = nullptr;
            CK(hipExtMallocWithFlags((void**)&cold, row_bytes * (n - H), flag));
            CK(hipMemset(cold, 0, row_bytes * (n - H)));
            const char* name = flag == hipDeviceMallocDefault ? "default" :
                               flag == hipDeviceMallocFinegrained ? "finegrained" : "uncached";
            printf("H=%6d  cold rows split, %-11s %8.1f\n", H, name,
                   run<1>(grid, rp, col, n, H, hot, cold, yold, out, part));
            fflush(stdout);
            CK(hipFree(cold));
        }
    }
    return 0;
}

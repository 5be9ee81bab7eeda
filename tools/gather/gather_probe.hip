// gather_probe.hip -- measures the MI355X's attainable rate for the access
// pattern of the SLQ SpMM (K1): rows of a row-major fp64 table gathered by a
// uniformly random index stream, RB bytes per row (8 lanes x 16 B for 128-B
// rows), U gathers in flight per row group, summed into registers and written
// once per output row (like y = A u with degree `deg`).
//
//   hipcc -O3 --offload-arch=gfx950 gather_probe.hip -o gather_probe
//   ./gather_probe            -> one line per configuration
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <string>
#include <vector>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                \
        }                                                                           \
    } while (0)

// P doubles per row (P/2 lanes x 16 B), U gathers in flight, deg gathers per output row
template <int P, int U>
__global__ __launch_bounds__(512) void k_gather(const int* __restrict__ idx, int nout, int deg,
                                                const double* __restrict__ table,
                                                double* __restrict__ out) {
    constexpr int LPR = P / 2, GPW = 64 / LPR;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int sub = lane % LPR, grp = lane / LPR;
    const int groups = gridDim.x * (blockDim.x / 64) * GPW;
    for (int row = (blockIdx.x * (blockDim.x / 64) + wave) * GPW + grp; row < nout; row += groups) {
        double sx = 0.0, sy = 0.0;
        const int* ix = idx + (int64_t)row * deg;
        for (int k = 0; k < deg; k += U) {
            double2 x[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int c = (k + u < deg) ? ix[k + u] : ix[k];
                x[u] = *reinterpret_cast<const double2*>(table + (int64_t)c * P + 2 * sub);
            }
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (k + u < deg) {
                    sx += x[u].x;
                    sy += x[u].y;
                }
        }
        *reinterpret_cast<double2*>(out + (int64_t)row * P + 2 * sub) = make_double2(sx, sy);
    }
}

template <int P, int U>
double run(int nrows, int nout, int deg, int blocks_per_cu, int num_cu, const int* idx,
           const double* table, double* out) {
    const int grid = blocks_per_cu * num_cu;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    k_gather<P, U><<<grid, 512>>>(idx, nout, deg, table, out);  // warm
    CK(hipEventRecord(a));
    const int reps = 10;
    for (int r = 0; r < reps; ++r) k_gather<P, U><<<grid, 512>>>(idx, nout, deg, table, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, a, b));
    const double gathered = (double)nout * deg * P * 8.0;
    return gathered / (ms / reps * 1e-3) / 1e9;  // GB/s of gathered rows
}

int main(int argc, char** argv) {
    // argv[1] = "powerlaw": indices drawn with probability ~ (i+1)^(-2/3)
    // (the Chung-Lu gamma = 2.5 weights of the SLQ benchmark graph, hubs
    // first as after the degree relabelling); default uniform
    const bool powerlaw = argc > 1 && std::string(argv[1]) == "powerlaw";
    int num_cu = 0;
    CK(hipDeviceGetAttribute(&num_cu, hipDeviceAttributeMultiprocessorCount, 0));
    const int deg = 10;
    printf("# num_cu=%d  deg=%d  indices=%s  (GB/s = gathered row bytes / kernel time)\n", num_cu, deg,
           powerlaw ? "powerlaw" : "uniform");
    for (int table_mb : {16, 64, 128, 512}) {
        for (int P : {16, 32, 128}) {
            if (powerlaw && table_mb != 128 && table_mb != 256) continue;
            const int nrows = (int)((int64_t)table_mb * (1 << 20) / (8 * P));
            const int nout = nrows;  // one output row per table row (like y = A u)
            std::vector<int> h((size_t)nout * deg);
            uint64_t s = 88172645463325252ull;
            std::vector<double> cdf;
            if (powerlaw) {
                cdf.resize(nrows);
                // Chung-Lu weights w_i = c (i+1)^(-2/3), sum ~ nnz, capped at sqrt(nnz)
                const double nnz = (double)nrows * deg;
                const double c = nnz / (3.0 * std::cbrt((double)nrows));
                double acc = 0.0, cap = std::sqrt(nnz);
                for (int i = 0; i < nrows; ++i) {
                    acc += std::fmin(c * std::pow(i + 1.0, -2.0 / 3.0), cap);
                    cdf[i] = acc;
                }
                for (auto& c : cdf) c /= acc;
            }
            for (auto& v : h) {
                s ^= s << 13; s ^= s >> 7; s ^= s << 17;
                if (powerlaw) {
                    const double u = (double)(s >> 11) * (1.0 / 9007199254740992.0);
                    v = (int)(std::lower_bound(cdf.begin(), cdf.end(), u) - cdf.begin());
                    if (v >= nrows) v = nrows - 1;
                } else {
                    v = (int)(s % (uint64_t)nrows);
                }
            }
            int* idx;
            double *table, *out;
            CK(hipMalloc(&idx, sizeof(int) * h.size()));
            CK(hipMalloc(&table, sizeof(double) * (size_t)nrows * P));
            CK(hipMalloc(&out, sizeof(double) * (size_t)nout * P));
            CK(hipMemcpy(idx, h.data(), sizeof(int) * h.size(), hipMemcpyHostToDevice));
            CK(hipMemset(table, 0, sizeof(double) * (size_t)nrows * P));
            for (int bpc : {2, 4}) {
                double g4 = 0, g8 = 0;
                if (P == 16) { g4 = run<16, 4>(nrows, nout, deg, bpc, num_cu, idx, table, out);
                               g8 = run<16, 8>(nrows, nout, deg, bpc, num_cu, idx, table, out); }
                if (P == 32) { g4 = run<32, 4>(nrows, nout, deg, bpc, num_cu, idx, table, out);
                               g8 = run<32, 8>(nrows, nout, deg, bpc, num_cu, idx, table, out); }
                if (P == 128) { g4 = run<128, 4>(nrows, nout, deg, bpc, num_cu, idx, table, out);
                                g8 = run<128, 8>(nrows, nout, deg, bpc, num_cu, idx, table, out); }
                printf("table %4d MB  row %4d B  blocks/CU %d  U=4 %7.0f GB/s  U=8 %7.0f GB/s\n",
                       table_mb, P * 8, bpc, g4, g8);
                fflush(stdout);
            }
            CK(hipFree(idx));
            CK(hipFree(table));
            CK(hipFree(out));
        }
    }
    return 0;
}

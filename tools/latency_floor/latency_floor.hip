// Latency floors for the secondary configs' dependent chains.
// Measures on the MI355X, with HIP events / hipGraphs (no profiler):
//   1. dependent launch interval of a chain of N launches of an empty kernel
//      of grid G (256 threads), host-queued (wall / N) and replayed from a
//      hipGraph (the device-side floor, host issue removed);
//   2. the same chain when each thread does a dependent chain of H loads
//      through an L2-resident table (row_ptr -> col -> row -> ... shape);
//   3. inside one 512-thread workgroup (k_pair_reg's shape): cycles per
//      __syncthreads round and per dependent LDS load, by clock64.
// Build: hipcc -O3 --offload-arch=gfx950 latency_floor.hip -o latency_floor
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);            \
            return 1;                                                                          \
        }                                                                                      \
    } while (0)

__global__ void k_empty(int* sink) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && sink[0] == 12345) sink[1] = 1;
}

// each thread: H dependent loads idx = next[idx] over a small (L2-resident) table
__global__ void k_chase(const int* __restrict__ next, int mask, int H, int* out) {
    int i = (blockIdx.x * blockDim.x + threadIdx.x) & mask;
    for (int h = 0; h < H; ++h) i = next[i];
    if (i == -1) out[0] = i;
}

// one workgroup of 512: R rounds of (LDS write, barrier, dependent LDS read)
__global__ __launch_bounds__(512) void k_lds(int R, int H, unsigned long long* cyc, int* out) {
    __shared__ int s[1024];
    const int t = threadIdx.x;
    s[t] = (t * 7 + 1) & 1023;
    s[t + 512] = (t * 13 + 5) & 1023;
    __syncthreads();
    unsigned long long c0 = clock64();
    int v = t;
    for (int r = 0; r < R; ++r) {
        s[t] = v & 1023;
        __syncthreads();
        v = s[(t + 1) & 511];
    }
    unsigned long long c1 = clock64();
    int w = t;
    for (int h = 0; h < H; ++h) w = s[w & 1023];
    unsigned long long c2 = clock64();
    if (t == 0) {
        cyc[0] = c1 - c0;
        cyc[1] = c2 - c1;
    }
    if (v + w == -7) out[0] = 1;
}

static double chain_ms(hipStream_t st, int N, int grid, int H, const int* next, int* sink, bool graph) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    auto body = [&] {
        for (int i = 0; i < N; ++i) {
            if (H == 0)
                k_empty<<<grid, 256, 0, st>>>(sink);
            else
                k_chase<<<grid, 256, 0, st>>>(next, 4095, H, sink);
        }
    };
    float ms = 0.f;
    if (!graph) {
        body();  // warm
        (void)hipStreamSynchronize(st);
        (void)hipEventRecord(a, st);
        body();
        (void)hipEventRecord(b, st);
        (void)hipEventSynchronize(b);
        (void)hipEventElapsedTime(&ms, a, b);
    } else {
        hipGraph_t g;
        hipGraphExec_t ge;
        (void)hipStreamBeginCapture(st, hipStreamCaptureModeGlobal);
        body();
        (void)hipStreamEndCapture(st, &g);
        (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
        (void)hipGraphLaunch(ge, st);
        (void)hipStreamSynchronize(st);
        (void)hipEventRecord(a, st);
        (void)hipGraphLaunch(ge, st);
        (void)hipEventRecord(b, st);
        (void)hipEventSynchronize(b);
        (void)hipEventElapsedTime(&ms, a, b);
        (void)hipGraphExecDestroy(ge);
        (void)hipGraphDestroy(g);
    }
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    return ms;
}

int main() {
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    int *next, *sink;
    std::vector<int> h(4096);
    for (int i = 0; i < 4096; ++i) h[i] = (int)((i * 2654435761u + 12345u) & 4095u);
    CK(hipMalloc(&next, sizeof(int) * 4096));
    CK(hipMalloc(&sink, sizeof(int) * 4));
    CK(hipMemcpy(next, h.data(), sizeof(int) * 4096, hipMemcpyHostToDevice));
    CK(hipMemset(sink, 0, sizeof(int) * 4));
    const int N = 2000;
    std::printf("# 1-2. dependent launch chains, %d launches, 256 threads per workgroup\n", N);
    for (int grid : {64, 400, 1024}) {
        for (int H : {0, 4, 8}) {
            const double q = chain_ms(st, N, grid, H, next, sink, false) * 1e3 / N;
            const double g = chain_ms(st, N, grid, H, next, sink, true) * 1e3 / N;
            std::printf("grid %5d  dependent L2 loads per thread %d: %.2f us per launch host-queued, "
                        "%.2f us from a hipGraph\n", grid, H, q, g);
        }
    }
    unsigned long long* cyc;
    CK(hipMalloc(&cyc, sizeof(unsigned long long) * 2));
    std::printf("# 3. one 512-thread workgroup (k_pair_reg's shape)\n");
    for (int R : {256, 1024}) {
        k_lds<<<1, 512, 0, st>>>(R, 1024, cyc, sink);
        CK(hipStreamSynchronize(st));
        unsigned long long hc[2];
        CK(hipMemcpy(hc, cyc, sizeof(hc), hipMemcpyDeviceToHost));
        std::printf("rounds %d: %.1f cycles per (LDS write + __syncthreads + LDS read) round; "
                    "%.1f cycles per dependent LDS load\n", R, (double)hc[0] / R, (double)hc[1] / 1024);
    }
    int clk = 0;
    CK(hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0));
    std::printf("# device clock attribute %d kHz\n", clk);
    return 0;
}

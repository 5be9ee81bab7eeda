// Host cost of kernel launches from 1..T threads, each on its own stream
// (config 1's expmv chains launch ~1 kernel per Taylor term from 3 host
// threads).  Prints per-launch host time and the wall time per launch per
// stream for a dependent chain of tiny kernels.
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <thread>
#include <vector>

__global__ void k_tiny(double* x, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) x[i] = x[i] * 0.5 + 1.0;
}

static void run(int T, int launches, int grid) {
    std::vector<hipStream_t> st(T);
    std::vector<double*> buf(T);
    for (int t = 0; t < T; ++t) {
        (void)hipStreamCreateWithFlags(&st[t], hipStreamNonBlocking);
        (void)hipMalloc(&buf[t], sizeof(double) * 256 * grid);
    }
    (void)hipDeviceSynchronize();
    std::vector<double> host_us(T), wall_us(T);
    std::atomic<int> ready{0};
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
        th.emplace_back([&, t] {
            (void)hipSetDevice(0);
            ready.fetch_add(1);
            while (ready.load() < T) {
            }
            auto t0 = std::chrono::steady_clock::now();
            for (int i = 0; i < launches; ++i) k_tiny<<<grid, 256, 0, st[t]>>>(buf[t], 256 * grid);
            auto t1 = std::chrono::steady_clock::now();
            (void)hipStreamSynchronize(st[t]);
            auto t2 = std::chrono::steady_clock::now();
            host_us[t] = std::chrono::duration<double, std::micro>(t1 - t0).count() / launches;
            wall_us[t] = std::chrono::duration<double, std::micro>(t2 - t0).count() / launches;
        });
    for (auto& x : th) x.join();
    double h = 0, w = 0;
    for (int t = 0; t < T; ++t) {
        h += host_us[t] / T;
        w += wall_us[t] / T;
    }
    std::printf("threads %d grid %d: host %.2f us per launch, wall %.2f us per launch per stream\n", T, grid, h, w);
    for (int t = 0; t < T; ++t) {
        (void)hipFree(buf[t]);
        (void)hipStreamDestroy(st[t]);
    }
}

int main() {
    for (int grid : {64, 512})
        for (int T : {1, 2, 3, 4}) run(T, 4000, grid);
    return 0;
}

// TEST INFRASTRUCTURE: ThreadSanitizer stress test of the host worker pool
// (krylov_robustness_amd/csrc/kt_pool.h) -- built by `make -C
// krylov_robustness_amd/csrc tsan`, run by tools/sanitize.sh.
//
// Several caller threads (the contexts / twin workers of the library) submit
// jobs to the one process-wide pool at once, as mc_trace's twin and
// speculative threads and kt_slq_collect's quadratures do; every job writes
// disjoint slots and the caller checks them after run() returns, so any
// missing happens-before edge between the workers' writes and the caller's
// reads (or between successive jobs' job_/count_ fields) is a data race
// TSan reports.  Exit 0 and no report: clean.
#include <atomic>
#include <cstdio>
#include <thread>
#include <vector>

#include "kt_pool.h"

int main() {
    constexpr int kCallers = 4, kRounds = 200;
    std::atomic<int> bad{0};
    std::vector<std::thread> callers;
    for (int c = 0; c < kCallers; ++c) {
        callers.emplace_back([c, &bad] {
            for (int r = 0; r < kRounds; ++r) {
                const int count = 8 + (r * 7 + c * 13) % 120;  // above and below min_parallel
                std::vector<double> out(count, -1.0);
                kt::HostPool::get().run(count, [&](int i) { out[i] = (double)(i * (c + 1) + r); }, 8);
                for (int i = 0; i < count; ++i)
                    if (out[i] != (double)(i * (c + 1) + r)) bad.fetch_add(1);
            }
        });
    }
    for (auto& t : callers) t.join();
    std::printf("pool_stress: %d callers x %d jobs, pool threads %d, wrong slots %d\n", kCallers, kRounds,
                kt::HostPool::get().threads(), bad.load());
    return bad.load() == 0 ? 0 : 1;
}

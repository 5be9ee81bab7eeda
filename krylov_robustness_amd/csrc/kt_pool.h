// kt_pool.h -- persistent host worker pool for small per-column / per-
// candidate dense work between device steps (the greedy host-eig path,
// the Frechet entries of hessianfcn); spawning threads every Krylov step
// would cost more than the work.  Sized by host_pool_threads().
#pragma once
#include <sched.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <condition_variable>
#include <cstdlib>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace kt {

// CPUs this process may use: the affinity mask capped by the cgroup CPU
// quota (v2 cpu.max, v1 cfs_quota_us / cfs_period_us), as bench.py cpu_share
inline int process_cpus() {
    int aff = 0;
    cpu_set_t set;
    CPU_ZERO(&set);
    if (sched_getaffinity(0, sizeof(set), &set) == 0) aff = CPU_COUNT(&set);
    if (aff <= 0) aff = (int)std::max(1u, std::thread::hardware_concurrency());
    double quota = -1.0;
    if (FILE* f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {
        char q[32] = {0};
        long per = 100000;
        if (std::fscanf(f, "%31s %ld", q, &per) >= 1 && std::string(q) != "max" && per > 0)
            quota = std::atof(q) / (double)per;
        std::fclose(f);
    } else if (FILE* g = std::fopen("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", "r")) {
        long q = -1, per = 100000;
        if (std::fscanf(g, "%ld", &q) == 1 && q > 0) {
            if (FILE* h = std::fopen("/sys/fs/cgroup/cpu/cpu.cfs_period_us", "r")) {
                if (std::fscanf(h, "%ld", &per) != 1 || per <= 0) per = 100000;
                std::fclose(h);
            }
            quota = (double)q / (double)per;
        }
        std::fclose(g);
    }
    if (quota > 0.0) aff = std::max(1, std::min(aff, (int)std::floor(quota + 1e-9)));
    return aff;
}

// The pool's threads (caller included): min(16, process_cpus() /
// LOCAL_WORLD_SIZE), >= 1 -- torchrun's ranks on one node share its CPUs;
// KT_HOST_THREADS overrides
inline int host_pool_threads() {
    if (const char* e = std::getenv("KT_HOST_THREADS")) {
        const int v = std::atoi(e);
        if (v > 0) return std::min(v, 256);
    }
    int lws = 1;
    if (const char* e = std::getenv("LOCAL_WORLD_SIZE")) lws = std::max(1, std::atoi(e));
    return std::max(1, std::min(16, process_cpus() / lws));
}

class HostPool {
   public:
    static HostPool& get() {
        static HostPool pool;
        return pool;
    }
    // f(i) for i in [0, count); the caller thread participates.  One job at a
    // time: callers on other threads (other contexts) wait their turn; f must
    // not call run() itself.
    void run(int count, const std::function<void(int)>& f, int min_parallel = 8) {
        if (count <= 0) return;
        if (workers_.empty() || count < min_parallel) {
            for (int i = 0; i < count; ++i) f(i);
            return;
        }
        std::lock_guard<std::mutex> job_lock(run_m_);
        {
            std::lock_guard<std::mutex> lk(m_);
            job_ = &f;
            count_ = count;
            next_.store(0);
            pending_ = (int)workers_.size();
            ++gen_;
        }
        cv_.notify_all();
        drain(f, count);
        std::unique_lock<std::mutex> lk(m_);
        done_cv_.wait(lk, [&] { return pending_ == 0; });
        job_ = nullptr;
    }
    int threads() const { return (int)workers_.size() + 1; }
    ~HostPool() {
        {
            std::lock_guard<std::mutex> lk(m_);
            stop_ = true;
            ++gen_;
        }
        cv_.notify_all();
        for (auto& t : workers_) t.join();
    }

   private:
    HostPool() {
        const int nt = host_pool_threads() - 1;
        for (int t = 0; t < nt; ++t) workers_.emplace_back([this] { loop(); });
    }
    void drain(const std::function<void(int)>& f, int count) {
        for (int i = next_.fetch_add(1); i < count; i = next_.fetch_add(1)) f(i);
    }
    void loop() {
        uint64_t seen = 0;
        for (;;) {
            const std::function<void(int)>* f;
            int count;
            {
                std::unique_lock<std::mutex> lk(m_);
                cv_.wait(lk, [&] { return gen_ != seen; });
                seen = gen_;
                if (stop_) return;
                f = job_;
                count = count_;
            }
            if (f) drain(*f, count);
            std::lock_guard<std::mutex> lk(m_);
            if (--pending_ == 0) done_cv_.notify_one();
        }
    }
    std::vector<std::thread> workers_;
    std::mutex run_m_, m_;
    std::condition_variable cv_, done_cv_;
    const std::function<void(int)>* job_ = nullptr;
    int count_ = 0, pending_ = 0;
    std::atomic<int> next_{0};
    uint64_t gen_ = 0;
    bool stop_ = false;
};

}  // namespace kt

// kt_pool.h -- persistent host worker pool for small per-column / per-
// candidate dense work between device steps (the greedy host-eig path,
// the Frechet entries of hessianfcn); spawning threads every Krylov step
// would cost more than the work.  Sized min(16, cores).
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace kt {

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
        int nt = (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency())) - 1;
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

// kt_worker.h -- persistent host worker threads of a context (kt_krylov.cpp,
// kt_mctrace.cpp): in-order job queues whose threads live as long as the
// context.
#pragma once
#include <hip/hip_runtime.h>

#include <condition_variable>
#include <deque>
#include <exception>
#include <functional>
#include <mutex>
#include <thread>

#include "kt_internal.h"

namespace kt {

// ---------------------------------------------------------------------------
// In-order worker thread for the projected-matrix work of a block-Krylov run
// (trace_fun_update / fun_update): job k runs while the caller's thread
// extends the basis by one more step.  wait(k) blocks until jobs 0..k of the
// current run have finished and rethrows the first failure; once a job failed
// the rest are skipped.  finish() ends a run: it drops the jobs not yet
// started, waits for the running one and resets the job count, so the thread
// serves the next run (threads per context: ctx_worker below).
// ---------------------------------------------------------------------------
class StepWorker {
   public:
    explicit StepWorker(int device) : device_(device) { th_ = std::thread([this] { loop(); }); }
    StepWorker(const StepWorker&) = delete;
    StepWorker& operator=(const StepWorker&) = delete;
    ~StepWorker() {
        {
            std::lock_guard<std::mutex> lk(m_);
            stop_ = true;
            q_.clear();
        }
        cv_.notify_all();
        th_.join();
    }
    void finish() {
        std::unique_lock<std::mutex> lk(m_);
        q_.clear();
        done_cv_.wait(lk, [&] { return !busy_; });
        done_ = 0;
        err_ = nullptr;
    }
    void submit(std::function<void()> f) {
        {
            std::lock_guard<std::mutex> lk(m_);
            q_.push_back(std::move(f));
        }
        cv_.notify_all();
    }
    void wait(int k) {
        std::unique_lock<std::mutex> lk(m_);
        done_cv_.wait(lk, [&] { return done_ > k || err_; });
        if (err_) std::rethrow_exception(err_);
    }

   private:
    void loop() {
        (void)hipSetDevice(device_);
        for (;;) {
            std::function<void()> f;
            bool skip;
            {
                std::unique_lock<std::mutex> lk(m_);
                cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
                if (q_.empty()) return;  // stop_ with nothing queued
                f = std::move(q_.front());
                q_.pop_front();
                busy_ = true;
                skip = err_ != nullptr;  // read under the lock: finish() / the failing job write it
            }
            std::exception_ptr e;
            if (!skip) {
                try {
                    f();
                } catch (...) {
                    e = std::current_exception();
                }
            }
            {
                std::lock_guard<std::mutex> lk(m_);
                if (e && !err_) err_ = e;
                ++done_;
                busy_ = false;
            }
            done_cv_.notify_all();
        }
    }
    int device_;
    std::mutex m_;
    std::condition_variable cv_, done_cv_;
    std::deque<std::function<void()>> q_;
    int done_ = 0;
    bool stop_ = false, busy_ = false;
    std::exception_ptr err_;
    std::thread th_;
};

// The context's persistent worker threads (created on first use), slot
// kWorkerPipeline for a block-Krylov run's projected work, kWorkerTwin /
// kWorkerSpec for the concurrent Afun calls of fun_and_grad_krylov_fun and
// mc_trace.  A thread that made HIP calls and EXITED stalled the device's
// other streams for 6-30 ms (profiles/r03_thread_exit_stall.txt), so these
// threads live as long as the context; a run ends with RunWorker's finish(),
// so the next run starts with an idle worker.
enum { kWorkerPipeline = 0, kWorkerTwin = 1, kWorkerSpec = 2 };
inline StepWorker* ctx_worker(kt_context_s* ctx, int slot) {
    if (!ctx->workers[slot]) {
        ctx->workers[slot] = new StepWorker(ctx->device);
        ctx->workers_free = [](void* p) { delete static_cast<StepWorker*>(p); };
    }
    return static_cast<StepWorker*>(ctx->workers[slot]);
}
// Scoped use of it by one run: finish() on every exit path, before the run's
// steps / Xstop (captured by reference in the queued jobs) go out of scope.
struct RunWorker {
    StepWorker* w = nullptr;
    RunWorker() = default;
    RunWorker(const RunWorker&) = delete;
    RunWorker& operator=(const RunWorker&) = delete;
    ~RunWorker() { reset(); }
    void reset(StepWorker* nw = nullptr) {
        if (w) w->finish();
        w = nw;
    }
    StepWorker* operator->() const { return w; }
    explicit operator bool() const { return w != nullptr; }
};

}  // namespace kt

// psgpu_pool.h -- the blocking export's host thread pool (std only: tests/cpp/pool_check.cpp
// builds it without HIP).
#pragma once
#include <stdint.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace psgpu {
// Host threads kept for the blocking export's scatter (psgpu_host.cpp export_scatter): spawning
// them per call cost more than the scatter of a small mesh.  run(n, f) calls f(0 .. n-1) over
// the workers and the caller and returns when every call has returned.  A task is claimed by a
// compare-exchange on one word holding (job, count, next), so a worker still leaving the last
// job can never take a task of the next one.
class ScatterPool {
public:
    explicit ScatterPool(unsigned workers) {
        for (unsigned i = 0; i < workers; ++i) th_.emplace_back([this] { work(); });
    }
    ~ScatterPool() {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (std::thread& t : th_) t.join();
    }
    unsigned workers() const { return (unsigned)th_.size(); }
    void run(unsigned n, const std::function<void(unsigned)>& f) {
        if (!n) return;
        {
            std::lock_guard<std::mutex> g(mu_);
            f_ = &f;
            left_.store(n, std::memory_order_relaxed);
            ++gen_;
            state_.store(((uint64_t)gen_ << 32) | ((uint64_t)n << 16), std::memory_order_release);
        }
        cv_.notify_all();
        drain(gen_);
        std::unique_lock<std::mutex> l(mu_);
        done_.wait(l, [&] { return left_.load(std::memory_order_acquire) == 0; });
    }

private:
    void drain(uint32_t gen) {
        uint64_t v = state_.load(std::memory_order_acquire);
        for (;;) {
            if ((uint32_t)(v >> 32) != gen || (v & 0xffffu) >= ((v >> 16) & 0xffffu)) return;
            if (!state_.compare_exchange_weak(v, v + 1, std::memory_order_acq_rel)) continue;
            (*f_)((unsigned)(v & 0xffffu));
            if (left_.fetch_sub(1, std::memory_order_acq_rel) == 1) {
                std::lock_guard<std::mutex> g(mu_);
                done_.notify_all();
            }
            v = state_.load(std::memory_order_acquire);
        }
    }
    void work() {
        uint32_t seen = 0;
        for (;;) {
            // a short spin for the next job (back-to-back calls), then sleep
            const auto t0 = std::chrono::steady_clock::now();
            while ((uint32_t)(state_.load(std::memory_order_acquire) >> 32) == seen &&
                   std::chrono::steady_clock::now() - t0 < std::chrono::microseconds(200))
                std::this_thread::yield();
            {
                std::unique_lock<std::mutex> l(mu_);
                cv_.wait(l, [&] { return stop_ || (uint32_t)(state_.load(std::memory_order_acquire) >> 32) != seen; });
                if (stop_) return;
            }
            seen = (uint32_t)(state_.load(std::memory_order_acquire) >> 32);
            drain(seen);
        }
    }
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_, done_;
    const std::function<void(unsigned)>* f_ = nullptr;
    std::atomic<uint64_t> state_{0};  // job << 32 | count << 16 | next
    std::atomic<uint32_t> left_{0};
    uint32_t gen_ = 0;
    bool stop_ = false;
};
}  // namespace psgpu

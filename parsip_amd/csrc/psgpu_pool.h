// psgpu_pool.h -- the blocking export's host thread pool (std only: tests/cpp/pool_check.cpp
// builds it without HIP).
#pragma once
#include <pthread.h>
#include <sched.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <unistd.h>

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
    // `cpus`: where the workers may run (null: anywhere the process may)
    // If a thread cannot be started, the ones already running are stopped and joined before
    // the exception leaves (a destroyed joinable std::thread would terminate the process), so
    // the caller's fallback (scatter on its own thread) can run.
    explicit ScatterPool(unsigned workers, const cpu_set_t* cpus = nullptr) {
        try {
            th_.reserve(workers);
            for (unsigned i = 0; i < workers; ++i) {
                th_.emplace_back([this] { work(); });
                if (cpus) (void)pthread_setaffinity_np(th_.back().native_handle(), sizeof(cpu_set_t), cpus);
            }
        } catch (...) {
            stop_all();
            throw;
        }
    }
    // The CPUs of the NUMA node the calling thread runs on, within the process's affinity set
    // (Linux sysfs); false if that cannot be read.  The export's threads stay on one node: spread
    // over both sockets of the box, their traffic slowed the device's writes into the staging
    // 3-4x in some calls (C3 blocking 0.5 -> 1.6-2.0 ms, bimodal; on one node, either one, 0.52-0.55).
    static bool caller_node_cpus(cpu_set_t* out) {
        unsigned cpu = 0, node = 0;
        if (getcpu(&cpu, &node) != 0) return false;
        char path[96];
        snprintf(path, sizeof(path), "/sys/devices/system/node/node%u/cpulist", node);
        FILE* f = fopen(path, "r");
        if (!f) return false;
        cpu_set_t allowed, mine;
        CPU_ZERO(&mine);
        if (sched_getaffinity(0, sizeof(allowed), &allowed) != 0) {
            fclose(f);
            return false;
        }
        unsigned a = 0, b = 0;
        char sep = 0;
        while (fscanf(f, "%u", &a) == 1) {  // "0-63,128-191"
            b = a;
            int c = fgetc(f);
            if (c == '-') {
                if (fscanf(f, "%u", &b) != 1) break;
                c = fgetc(f);
            }
            for (unsigned x = a; x <= b && x < CPU_SETSIZE; ++x)
                if (CPU_ISSET(x, &allowed)) CPU_SET(x, &mine);
            sep = (char)c;
            if (sep != ',') break;
        }
        fclose(f);
        if (CPU_COUNT(&mine) == 0) return false;
        *out = mine;
        return true;
    }
    ~ScatterPool() { stop_all(); }
    unsigned workers() const { return (unsigned)th_.size(); }

    // callerDrains: the calling thread takes tasks too (false: it only waits -- when the
    // workers are pinned to a node the caller may not be on)
    void run(unsigned n, const std::function<void(unsigned)>& f, bool callerDrains = true) {
        if (!n) return;
        {
            std::lock_guard<std::mutex> g(mu_);
            f_ = &f;
            left_.store(n, std::memory_order_relaxed);
            ++gen_;
            state_.store(((uint64_t)gen_ << 32) | ((uint64_t)n << 16), std::memory_order_release);
        }
        cv_.notify_all();
        if (callerDrains || th_.empty()) drain(gen_);
        std::unique_lock<std::mutex> l(mu_);
        done_.wait(l, [&] { return left_.load(std::memory_order_acquire) == 0; });
    }

private:
    void stop_all() {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (std::thread& t : th_)
            if (t.joinable()) t.join();
        th_.clear();
    }
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

// The blocking export's thread pool (parsip_amd/csrc/psgpu_pool.h), host only: every run(n, f)
// calls f(0 .. n-1) exactly once each and returns only after all of them, run after run, with
// runs back to back (the workers still spinning) and after pauses (the workers asleep).
#include <cstdio>
#include <cstdlib>

#include "psgpu_pool.h"

int main() {
    cpu_set_t node;
    const bool haveNode = psgpu::ScatterPool::caller_node_cpus(&node);
    for (unsigned workers : {1u, 3u, 16u}) {
        psgpu::ScatterPool pool(workers, haveNode && workers == 16 ? &node : nullptr);
        std::vector<std::atomic<int>> hits(16);
        for (int run = 0; run < 20000; ++run) {
            const unsigned n = 1 + (unsigned)(run * 7) % 16;
            for (auto& h : hits) h.store(0);
            std::atomic<int> inside{0};
            std::function<void(unsigned)> f = [&](unsigned k) {
                inside.fetch_add(1);
                if (k >= n) std::abort();
                hits[k].fetch_add(1);
                inside.fetch_sub(1);
            };
            pool.run(n, f, run % 2 == 0);  // the caller draining or only waiting
            if (inside.load() != 0) {
                std::printf("run %d returned with a task in flight\n", run);
                return 1;
            }
            for (unsigned k = 0; k < 16; ++k)
                if (hits[k].load() != (k < n ? 1 : 0)) {
                    std::printf("workers %u run %d n %u: task %u ran %d times\n", workers, run, n, k, hits[k].load());
                    return 1;
                }
            if (run % 5000 == 4999) std::this_thread::sleep_for(std::chrono::milliseconds(5));  // workers asleep
        }
    }
    std::printf("ok\n");
    return 0;
}

// Host-side launch floor of the library: ms per step of a rank's share of a
// config, E engines (contexts, one stream each) taking the steps in turn, enqueued
//   (a) from one host thread, round-robin (what bench.py does from Python), and
//   (b) from E host threads, one per engine (each enqueues every E-th step),
// through the C-ABI directly (no Python).  Launch cost is per host thread (tools/launch_cost:
// ~3.7 us per launch from one thread, ~1 us aggregate from four), so (b) shows what the
// device sustains once the host stops being the bound.
// Build: g++ -O2 -std=c++17 -I include tools/engine_threads.cpp -L parsip_amd -l:libparsip_gpu.so
//        -Wl,-rpath,$PWD/parsip_amd -lpthread -o tools/_bin/engine_threads
// Input: a model file (PsSoaBlobPrims, PsSoaPrimMatrices, PsSoaBlobOps bytes, then float cs),
// written by tools/dump_model.py.
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "parsip_gpu.h"

static double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

#define OK(x)                                                             \
    do {                                                                  \
        int rc_ = (x);                                                    \
        if (rc_ != PSGPU_RET_SUCCESS) {                                   \
            fprintf(stderr, "%s -> %d\n", #x, rc_);                       \
            exit(1);                                                      \
        }                                                                 \
    } while (0)

int main(int argc, char** argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: engine_threads model.bin [engines] [shares,..] [K]\n");
        return 2;
    }
    static PsSoaBlobPrims P;
    static PsSoaPrimMatrices M;
    static PsSoaBlobOps O;
    float cs = 0.0f;
    FILE* f = fopen(argv[1], "rb");
    if (!f || fread(&P, sizeof P, 1, f) != 1 || fread(&M, sizeof M, 1, f) != 1 || fread(&O, sizeof O, 1, f) != 1 ||
        fread(&cs, 4, 1, f) != 1) {
        fprintf(stderr, "bad model file\n");
        return 2;
    }
    fclose(f);
    const int E = argc > 2 ? atoi(argv[2]) : 4;
    std::vector<int> shares;
    for (const char* s = argc > 3 ? argv[3] : "1,8"; *s;) {
        shares.push_back(atoi(s));
        while (*s && *s != ',') ++s;
        if (*s) ++s;
    }
    const int K = argc > 4 ? atoi(argv[4]) : 800;
    const int vb = getenv("VB") ? atoi(getenv("VB")) : 8, fb = getenv("FB") ? atoi(getenv("FB")) : 4;
    psgpu_ctx* plan = nullptr;
    OK(psgpu_create(0, &plan));
    OK(psgpu_set_model(plan, &P, &M, &O));
    psgpu_jit_wait(plan);
    OK(psgpu_polygonize(plan, cs, 0, 0xffffffffu, nullptr));
    PsMeshInfo full;
    OK(psgpu_finish(plan, &full));
    std::vector<uint32_t> costs(full.ctMPUs);
    OK(psgpu_mpu_costs(plan, costs.data()));
    std::vector<psgpu_ctx*> eng(E);
    for (auto& c : eng) {
        OK(psgpu_create(0, &c));
        if (E > 1) {
            OK(psgpu_set_option(c, PSGPU_OPT_VERTEX_BLOCKS_PER_CU, vb));
            OK(psgpu_set_option(c, PSGPU_OPT_FINISH_BLOCKS_PER_CU, fb));
        }
        OK(psgpu_set_model(c, &P, &M, &O));
        psgpu_jit_wait(c);
    }
    for (int S : shares) {
        std::vector<uint32_t> b(S + 1);
        OK(psgpu_split_costs(costs.data(), (uint32_t)costs.size(), (uint32_t)S, 0, b.data()));
        double worst1 = 0, worstE = 0;
        for (int r = 0; r < S; ++r) {
            const uint32_t lo = b[r], hi = b[r + 1];
            for (auto* c : eng) {  // warm-up: the range's buffers and k_mpu grid
                for (int k = 0; k < 3; ++k) OK(psgpu_polygonize(c, cs, lo, hi, nullptr));
                OK(psgpu_finish(c, nullptr));
            }
            // (a) one host thread, round-robin
            double t0 = now_s(), enq = 0;
            for (int k = 0; k < K; ++k) {
                const double a = now_s();
                OK(psgpu_polygonize(eng[k % E], cs, lo, hi, nullptr));
                enq += now_s() - a;
            }
            for (auto* c : eng) OK(psgpu_finish(c, nullptr));
            const double one = (now_s() - t0) / K * 1e6;
            // (b) one host thread per engine
            std::atomic<int> go{0};
            std::vector<std::thread> th;
            t0 = now_s();
            for (int e = 0; e < E; ++e)
                th.emplace_back([&, e] {
                    while (!go.load()) {
                    }
                    for (int k = e; k < K; k += E) OK(psgpu_polygonize(eng[e], cs, lo, hi, nullptr));
                    OK(psgpu_finish(eng[e], nullptr));
                });
            t0 = now_s();
            go = 1;
            for (auto& t : th) t.join();
            const double thr = (now_s() - t0) / K * 1e6;
            PsMeshInfo I;
            OK(psgpu_finish(eng[0], &I));
            printf("share 1/%d rank %d (MPUs %u, V %u): %d engines: one thread %.1f us/step (enqueue %.1f us), "
                   "%d threads %.1f us/step\n",
                   S, r, hi - lo, I.ctVertices, E, one, enq / K * 1e6, E, thr);
            fflush(stdout);
            if (one > worst1) worst1 = one;
            if (thr > worstE) worstE = thr;
        }
        printf("share 1/%d: slowest rank one thread %.1f us/step, %d threads %.1f us/step\n", S, worst1, E, worstE);
        fflush(stdout);
    }
    for (auto* c : eng) psgpu_destroy(c);
    psgpu_destroy(plan);
    return 0;
}

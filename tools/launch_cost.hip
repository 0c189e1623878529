// Launch-cost probe: what one kernel launch costs the host and the device on MI355X, to
// size the per-polygonization launch floor.  Empty kernels with a
// 320-byte argument block (the size of psgpu::Params), launched through
// hipModuleLaunchKernel-equivalent paths (hipLaunchKernel of a static kernel here),
//   - back to back on one stream, on 4 streams round-robin, from 4 host threads;
//   - in "steps" of L dependent launches (L = 1..4) on E engines (streams) in turn,
//     with 1 block and with a persistent-sized grid (2048 blocks of 256 threads).
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/_bin/launch_cost tools/launch_cost.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <thread>
#include <vector>

struct Arg {
    unsigned int w[80];  // 320 B
};

__global__ void k_empty(Arg a) {
    if (a.w[0] == 0xdeadbeefu && threadIdx.x == 1234567) a.w[1] = 0;  // never true
}

#define CHECK(x)                                                                  \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
            return 1;                                                             \
        }                                                                         \
    } while (0)

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
    Arg a{};
    CHECK(hipFree(nullptr));
    (void)hipDeviceSynchronize();
    std::vector<hipStream_t> st(8);
    for (auto& s : st) CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const int K = 20000;
    // warm-up
    for (int i = 0; i < 200; ++i) hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st[0], a);
    CHECK(hipDeviceSynchronize());
    for (int grid : {1, 2048}) {
        for (int E : {1, 2, 4, 6}) {
            for (int L : {1, 2, 3, 4}) {
                const int steps = K / L;
                const double t0 = now_us();
                for (int s = 0; s < steps; ++s)
                    for (int l = 0; l < L; ++l) hipLaunchKernelGGL(k_empty, dim3(grid), dim3(256), 0, st[s % E], a);
                const double t1 = now_us();
                CHECK(hipDeviceSynchronize());
                const double t2 = now_us();
                printf("grid %4d engines %d launches/step %d: %.2f us/step (%.2f us/launch), host enqueue %.2f us/launch\n",
                       grid, E, L, (t2 - t0) / steps, (t2 - t0) / (steps * L), (t1 - t0) / (steps * L));
                fflush(stdout);
            }
        }
    }
    // 4 host threads, one stream each, 1 block
    for (int T : {2, 4}) {
        const int per = K / T;
        const double t0 = now_us();
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t)
            th.emplace_back([&, t] {
                for (int i = 0; i < per; ++i) hipLaunchKernelGGL(k_empty, dim3(1), dim3(256), 0, st[t], a);
            });
        for (auto& x : th) x.join();
        CHECK(hipDeviceSynchronize());
        const double t1 = now_us();
        printf("%d host threads x 1 stream each, grid 1: %.2f us/launch overall\n", T, (t1 - t0) / (per * T));
        fflush(stdout);
    }
    // hipModuleLaunchKernel (how the library launches its per-tree kernels), 1 and 4 threads
    hipModule_t mod = nullptr;
    hipFunction_t fn = nullptr;
    if (hipModuleLoad(&mod, "tools/_bin/empty.co") == hipSuccess &&
        hipModuleGetFunction(&fn, mod, "k_empty_mod") == hipSuccess) {
        for (int T : {1, 2, 4}) {
            const int per = K / T;
            const double t0 = now_us();
            std::vector<std::thread> th;
            for (int t = 0; t < T; ++t)
                th.emplace_back([&, t] {
                    Arg b = a;
                    void* args[] = {&b};
                    for (int i = 0; i < per; ++i)
                        (void)hipModuleLaunchKernel(fn, 1, 1, 1, 256, 1, 1, 0, st[t], args, nullptr);
                });
            for (auto& x : th) x.join();
            CHECK(hipDeviceSynchronize());
            const double t1 = now_us();
            printf("module launch, %d host threads x 1 stream each: %.2f us/launch overall\n", T, (t1 - t0) / (per * T));
            fflush(stdout);
        }
    } else {
        printf("module launch: tools/_bin/empty.co not loadable\n");
    }
    // device-side cost of a dependent kernel: a hipGraph of 64 empty kernels in a chain
    // (the host launches once), timed with events; 1 and 4 graphs on 4 streams at once
    for (int grid : {1, 2048}) {
        hipGraph_t g;
        hipGraphExec_t ge;
        CHECK(hipStreamBeginCapture(st[0], hipStreamCaptureModeGlobal));
        for (int i = 0; i < 64; ++i) hipLaunchKernelGGL(k_empty, dim3(grid), dim3(256), 0, st[0], a);
        CHECK(hipStreamEndCapture(st[0], &g));
        CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        for (int i = 0; i < 3; ++i) CHECK(hipGraphLaunch(ge, st[0]));
        CHECK(hipDeviceSynchronize());
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        for (int S : {1, 4}) {
            CHECK(hipEventRecord(e0, st[0]));
            for (int s = 1; s < S; ++s) CHECK(hipStreamWaitEvent(st[s], e0, 0));
            const int reps = 10;
            for (int r = 0; r < reps; ++r)
                for (int s = 0; s < S; ++s) CHECK(hipGraphLaunch(ge, st[s]));
            for (int s = 1; s < S; ++s) {
                hipEvent_t es;
                (void)hipEventCreate(&es);
                CHECK(hipEventRecord(es, st[s]));
                CHECK(hipStreamWaitEvent(st[0], es, 0));
            }
            CHECK(hipEventRecord(e1, st[0]));
            CHECK(hipEventSynchronize(e1));
            float ms = 0;
            (void)hipEventElapsedTime(&ms, e0, e1);
            printf("graph of 64 dependent empty kernels, grid %d, %d streams at once: %.2f us per kernel per stream, "
                   "%.2f us per kernel overall\n", grid, S, ms * 1e3 / (reps * 64), ms * 1e3 / (reps * 64 * S));
            fflush(stdout);
        }
        (void)hipGraphExecDestroy(ge);
        (void)hipGraphDestroy(g);
    }
    // dependent-launch latency: one stream, launch + sync each time
    {
        const int R = 2000;
        const double t0 = now_us();
        for (int i = 0; i < R; ++i) {
            hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st[0], a);
            (void)hipStreamSynchronize(st[0]);
        }
        const double t1 = now_us();
        printf("launch + stream sync round trip: %.2f us\n", (t1 - t0) / R);
    }
    for (auto& s : st) (void)hipStreamDestroy(s);
    return 0;
}

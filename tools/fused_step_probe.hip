// The per-step floor of a C4 1/8 rank share: today's chain of 4 dependent
// kernels per polygonization against ONE persistent kernel whose 4 phases are separated by
// grid barriers, both with no work in them, E engines (streams) taking the steps in turn.
//
//   chain  k_precheck 216 blocks | k_mpu 256 | k_vertex 4096 (16 / CU, persistent) |
//          k_finish 2048 (8 / CU): the 1/8 share's grids, empty bodies;
//   fused  one launch of B blocks (1 or 2 per CU, all resident: a grid barrier needs that),
//          3 grid barriers: XCD-hierarchical (MI355X_MICROARCH.md "barrier-xcd": a counter per
//          group of blocks b mod 8 -- one XCD each under round-robin dispatch -- the group's
//          last arriver bumps the top counter, every block polls the top counter with s_sleep;
//          release fence before arriving, acquire fence after), every spin bounded (a block that
//          gives up sets an error word and leaves; the run then reports it).
// Kernel arguments are 336 bytes, as psgpu::Params.  No scalar-cache stores anywhere.
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/_bin/fused_step_probe tools/fused_step_probe.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

struct Arg {
    unsigned int w[84];  // 336 B
};

__global__ void __launch_bounds__(256) k_empty(Arg a) {
    if (a.w[0] == 0xdeadbeefu && threadIdx.x == 1234567) a.w[1] = 0;  // never true
}

struct Bar {
    unsigned int* group;  // 8 counters, 32 words (128 B) apart
    unsigned int* top;    // the top counter
    unsigned int* err;    // set by a block whose spin gave up
    unsigned int perGroup, groups, spinMax;
};

__device__ __forceinline__ bool grid_barrier(const Bar& b, unsigned int phase) {
    __syncthreads();
    bool ok = true;
    if (threadIdx.x == 0) {
        const unsigned int g = blockIdx.x & 7u;
        __atomic_thread_fence(__ATOMIC_RELEASE);  // this block's phase writes before the arrival
        const unsigned int arrived = __hip_atomic_fetch_add(b.group + 32 * g, 1u, __ATOMIC_RELAXED,
                                                            __HIP_MEMORY_SCOPE_AGENT);
        if (arrived + 1u == b.perGroup * (phase + 1u))  // the group's last block
            __hip_atomic_fetch_add(b.top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned int want = b.groups * (phase + 1u);
        unsigned int spins = 0;
        while (__hip_atomic_load(b.top, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want) {
            __builtin_amdgcn_s_sleep(1);
            if (++spins > b.spinMax) {
                __hip_atomic_store(b.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                ok = false;
                break;
            }
        }
        __atomic_thread_fence(__ATOMIC_ACQUIRE);
    }
    __shared__ int sOk;
    if (threadIdx.x == 0) sOk = ok ? 1 : 0;
    __syncthreads();
    return sOk != 0;
}

// launch n of an engine: its barriers are phases nbar n .. nbar n + nbar - 1 of monotonic
// counters (no reset between launches, so no memset joins the step)
__global__ void __launch_bounds__(256) k_fused(Arg a, Bar b, unsigned int n, unsigned int nbar) {
    if (a.w[0] == 0xdeadbeefu && threadIdx.x == 1234567) a.w[1] = 0;
    for (unsigned int ph = 0; ph < nbar; ++ph)
        if (!grid_barrier(b, nbar * n + ph)) return;  // every block leaves: the error word says why
}

#define CHECK(x)                                                     \
    do {                                                             \
        hipError_t e_ = (x);                                         \
        if (e_ != hipSuccess) {                                      \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); \
            return 1;                                                \
        }                                                            \
    } while (0)

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
    const int steps = argc > 1 ? atoi(argv[1]) : 2000;
    Arg a{};
    CHECK(hipFree(nullptr));
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    std::vector<hipStream_t> st(4);
    for (auto& s : st) CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    // one barrier state per engine (a step's barriers count up; reset between measurements)
    const size_t words = 8 * 32 + 32 + 32;
    std::vector<unsigned int*> mem(4);
    for (auto& m : mem) CHECK(hipMalloc(&m, words * 4));
    for (int i = 0; i < 200; ++i) hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st[0], a);
    CHECK(hipDeviceSynchronize());
    const unsigned int chain[4] = {216, 256, (unsigned)(16 * cus), (unsigned)(8 * cus)};
    for (int E : {1, 4}) {
        // chain of 4 empty kernels per step
        {
            const double t0 = now_us();
            for (int s = 0; s < steps; ++s)
                for (int l = 0; l < 4; ++l) hipLaunchKernelGGL(k_empty, dim3(chain[l]), dim3(256), 0, st[s % E], a);
            CHECK(hipDeviceSynchronize());
            const double t1 = now_us();
            printf("engines %d chain  (216 | 256 | %u | %u blocks): %.2f us/step\n", E, chain[2], chain[3],
                   (t1 - t0) / steps);
            fflush(stdout);
        }
        {  // two kernels per step (k_precheck + k_mpu and k_vertex + k_finish each fused)
            const double t0 = now_us();
            for (int s = 0; s < steps; ++s) {
                hipLaunchKernelGGL(k_empty, dim3(256), dim3(256), 0, st[s % E], a);
                hipLaunchKernelGGL(k_empty, dim3(chain[2]), dim3(256), 0, st[s % E], a);
            }
            CHECK(hipDeviceSynchronize());
            const double t1 = now_us();
            printf("engines %d chain2 (256 | %u blocks): %.2f us/step\n", E, chain[2], (t1 - t0) / steps);
            fflush(stdout);
        }
        for (int cfg = 0; cfg < 4; ++cfg) {
            const int perCu = cfg == 3 ? 2 : 1;
            const unsigned int nbar = cfg == 0 ? 0u : (cfg == 1 ? 1u : 3u);
            const unsigned int B = (unsigned)(perCu * cus);
            for (auto& m : mem) CHECK(hipMemset(m, 0, words * 4));
            unsigned int err = 0;
            const double t0 = now_us();
            for (int s = 0; s < steps; ++s) {
                const int e = s % E;
                Bar b{mem[e], mem[e] + 8 * 32, mem[e] + 8 * 32 + 32, B / 8u, 8u, 1u << 22};
                hipLaunchKernelGGL(k_fused, dim3(B), dim3(256), 0, st[e], a, b, (unsigned)(s / E), nbar);
            }
            CHECK(hipDeviceSynchronize());
            const double t1 = now_us();
            for (int e = 0; e < E; ++e) {
                unsigned int x = 0;
                CHECK(hipMemcpy(&x, mem[e] + 8 * 32 + 32, 4, hipMemcpyDeviceToHost));
                err |= x;
            }
            printf("engines %d fused  (%u blocks, %u grid barriers): %.2f us/step%s\n", E, B, nbar, (t1 - t0) / steps,
                   err ? "  [a barrier spin gave up]" : "");
            fflush(stdout);
        }
    }
    for (auto& m : mem) (void)hipFree(m);
    return 0;
}

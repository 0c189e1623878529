// psgpu_kernels.hip — static CDNA4 (gfx950) kernels of the BlobTree polygonizer.
//
// Pipeline for one polygonization of MPUs [begin, begin+count) (the reference's
// Polygonize + CMPUProcessor, PS_Polygonizer.cpp:315-385, 441-829):
//
//   k_precheck  8 lanes per MPU, 2 quads: S1 corner test F>0          (:483-540), and the
//               ordered list of the MPUs that passed (single-pass look-back compaction)
//   k_mpu       one wavefront per passing MPU: S2 8^3 field cache in LDS (quads of 4
//               z-consecutive corners), S3 configs, vertex ownership + wave prefix
//               sums for the reference's discovery order, triangle records
//   k_scan      one block: per-MPU vertex/triangle offsets (compact mesh)
//   k_vertex    one quad per vertex: S4 4-sample root bracket, S5 colour + normals
//   k_finish    vertex colours (64 per wave) + triangle records -> global vertex ids
//
// The tree-evaluating kernels (precheck, mpu, vertex, probe) exist twice: here with
// the generic walk-program interpreter (InterpEval), and specialised per model
// structure at run time by psgpu_jit.cpp (hiprtc), which the host prefers.  Both
// instantiate the same bodies from psgpu_device.h.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "psgpu_device.h"

namespace psgpu {

__global__ void __launch_bounds__(256) k_precheck(Params p) {
    extern __shared__ float lds[];
    precheck_body<InterpEval>(p, lds);
}

__global__ void __launch_bounds__(256) k_mpu(Params p) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    mpu_body<InterpEval>(p, smem);
}

__global__ void __launch_bounds__(256) k_vertex(Params p) {
    extern __shared__ __attribute__((aligned(16))) float vlds[];
    vertex_body<InterpEval>(p, vlds);
}

__global__ void __launch_bounds__(256) k_probe(Params p, const float* __restrict__ xyz, float* __restrict__ out,
                                               float* __restrict__ colOut, uint32_t n, int mode) {
    extern __shared__ __attribute__((aligned(16))) float plds[];
    probe_body<InterpEval>(p, plds, xyz, out, colOut, n, mode);
}

__global__ void __launch_bounds__(256) k_finish(Params p) {
    extern __shared__ __attribute__((aligned(16))) float flds[];
    finish_body<InterpEval>(p, flds);
}

// Exclusive offsets of the per-MPU (V | T << 32) counts of the range, in MPU order (the
// reference's PolyMPUs order): offs[0] = 0, offs[w + 1] = inclusive sum.  Single pass:
// each 1024-thread block owns chunks of kScanItems counts (8 consecutive per thread,
// 64-B vector loads), publishes its aggregate, looks back over up to 64 predecessors at
// once (decoupled look-back), then scans.  V and T halves are scanned as two u32 DPP
// scans (their totals stay below 2^31).  Status words (state << 62 | T << 31 | V) start
// at zero: the previous run's k_finish cleared them.  All blocks are resident.
namespace {
__device__ __forceinline__ uint64_t scan_word(uint32_t state, uint32_t v, uint32_t t) {
    return ((uint64_t)state << 62) | ((uint64_t)(t & 0x7fffffffu) << 31) | (uint64_t)(v & 0x7fffffffu);
}

struct Chunk8 {
    uint64_t c[8];
    __device__ void load(const uint64_t* counts, uint32_t e, uint32_t hi) {
        if (e + 8 <= hi) {
            const uint4* src = reinterpret_cast<const uint4*>(counts + e);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint4 q = src[i];
                c[2 * i] = (uint64_t)q.x | ((uint64_t)q.y << 32);
                c[2 * i + 1] = (uint64_t)q.z | ((uint64_t)q.w << 32);
            }
        } else {
#pragma unroll
            for (int i = 0; i < 8; ++i) c[i] = e + i < hi ? counts[e + i] : 0ull;
        }
    }
    __device__ void sum(uint32_t& v, uint32_t& t) const {
        v = 0u;
        t = 0u;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            v += (uint32_t)c[i];
            t += (uint32_t)(c[i] >> 32);
        }
    }
};
}  // namespace

__global__ void __launch_bounds__(1024) k_scan(Params p) {
    __shared__ uint32_t sWave[2][16];
    __shared__ uint32_t sPrefix[2];
    const uint32_t n = p.mpuCount;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const uint32_t b = blockIdx.x;
    const uint32_t lo = b * p.scanChunks * kScanItems;
    const uint32_t hi = min(n, lo + p.scanChunks * kScanItems);
    // pass 1: the block's aggregate (the first chunk stays in registers)
    Chunk8 ch;
    ch.load(p.counts, lo + (uint32_t)t * 8u, hi);
    uint32_t sv, st;
    ch.sum(sv, st);
    for (uint32_t c = 1; c < p.scanChunks; ++c) {
        Chunk8 more;
        more.load(p.counts, lo + c * kScanItems + (uint32_t)t * 8u, hi);
        uint32_t a, bb;
        more.sum(a, bb);
        sv += a;
        st += bb;
    }
    const uint32_t wv_v = lane_value(wave_incl_scan(sv), 63), wv_t = lane_value(wave_incl_scan(st), 63);
    if (lane == 0) {
        sWave[0][wv] = wv_v;
        sWave[1][wv] = wv_t;
    }
    __syncthreads();
    if (wv == 0) {
        uint32_t aggV = 0u, aggT = 0u;
#pragma unroll
        for (int w = 0; w < 16; ++w) {
            aggV += sWave[0][w];
            aggT += sWave[1][w];
        }
        uint32_t exV = 0u, exT = 0u;
        if (b == 0) {
            if (lane == 0) __hip_atomic_store(&p.scanStatus[0], scan_word(2, aggV, aggT), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            if (lane == 0) __hip_atomic_store(&p.scanStatus[b], scan_word(1, aggV, aggT), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            int64_t j = (int64_t)b - 1;
            for (;;) {
                const int64_t idx = j - lane;
                uint32_t state = 2, v = 0u, tt = 0u;
                if (idx >= 0) {
                    uint64_t w = 0ull;
                    uint32_t spins = 0;  // bounded: a broken protocol ends the kernel, flagged
                    do {
                        w = __hip_atomic_load(&p.scanStatus[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    } while ((w >> 62) == 0ull && ++spins < (1u << 20));
                    if ((w >> 62) == 0ull) {
                        atomicOr(&p.ctr->error, 1u);
                        w = scan_word(2, 0u, 0u);
                    }
                    state = (uint32_t)(w >> 62);
                    v = (uint32_t)(w & 0x7fffffffull);
                    tt = (uint32_t)((w >> 31) & 0x7fffffffull);
                }
                const uint64_t inc = ballot(state == 2);
                const bool stop = inc != 0ull;
                const int k = stop ? __builtin_ctzll(inc) : 63;  // newest predecessor with an inclusive prefix
                exV += lane_value(wave_incl_scan(lane <= k ? v : 0u), 63);
                exT += lane_value(wave_incl_scan(lane <= k ? tt : 0u), 63);
                if (stop) break;
                j -= 64;
            }
            if (lane == 0)
                __hip_atomic_store(&p.scanStatus[b], scan_word(2, exV + aggV, exT + aggT), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
        if (lane == 0) {
            sPrefix[0] = exV;
            sPrefix[1] = exT;
        }
    }
    if (b == 0 && t == 0) p.offs[0] = 0ull;
    __syncthreads();
    // pass 2: per thread 8 consecutive counts; one block-wide scan per chunk
    uint32_t carryV = sPrefix[0], carryT = sPrefix[1];
    for (uint32_t c = 0; c < p.scanChunks; ++c) {
        const uint32_t e0 = lo + c * kScanItems + (uint32_t)t * 8u;
        if (c > 0) {
            ch.load(p.counts, e0, hi);
            ch.sum(sv, st);
            __syncthreads();  // sWave reuse
        }
        const uint32_t iv = wave_incl_scan(sv), it = wave_incl_scan(st);
        if (lane == 63) {
            sWave[0][wv] = iv;
            sWave[1][wv] = it;
        }
        __syncthreads();
        uint32_t runV = carryV + iv - sv, runT = carryT + it - st;
        uint32_t totV = 0u, totT = 0u;
#pragma unroll
        for (int w = 0; w < 16; ++w) {
            const uint32_t a = sWave[0][w], bb = sWave[1][w];
            runV += w < wv ? a : 0u;
            runT += w < wv ? bb : 0u;
            totV += a;
            totT += bb;
        }
        uint64_t out[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            runV += (uint32_t)ch.c[i];
            runT += (uint32_t)(ch.c[i] >> 32);
            out[i] = (uint64_t)runV | ((uint64_t)runT << 32);
        }
#pragma unroll
        for (int i = 0; i < 8; ++i)
            if (e0 + i < hi) p.offs[e0 + i + 1] = out[i];
        carryV += totV;
        carryT += totT;
    }
}

// ---------------------------------------------------------------------------
// Host-side launch helpers (psgpu_launch.h).
size_t mpu_lds_bytes(uint32_t slots) { return kLdsTables + 4 * (kLdsSlots + (size_t)slots * 64 * 4); }
size_t walk_lds_bytes(uint32_t slots) { return 4 * ((size_t)slots * 4 * 64 * 4); }
size_t precheck_lds_bytes(uint32_t slots) { return 4 * ((size_t)slots * 64 * 4); }

hipError_t launch_precheck(const Params& p, hipStream_t s) {
    hipLaunchKernelGGL(k_precheck, dim3(p.preBlocks), dim3(256), precheck_lds_bytes(p.slotsPerLane), s, p);
    return hipGetLastError();
}
hipError_t launch_scan(const Params& p, hipStream_t s) {
    hipLaunchKernelGGL(k_scan, dim3(p.scanBlocks), dim3(1024), 0, s, p);
    return hipGetLastError();
}
hipError_t launch_mpu(const Params& p, hipStream_t s) {
    const uint32_t blocks = kShards * ((p.pShardCap + 3) / 4);
    hipLaunchKernelGGL(k_mpu, dim3(blocks), dim3(256), mpu_lds_bytes(p.slotsPerLane), s, p);
    return hipGetLastError();
}
hipError_t launch_vertex(const Params& p, hipStream_t s, uint32_t blocks) {
    hipLaunchKernelGGL(k_vertex, dim3(blocks), dim3(256), walk_lds_bytes(p.slotsPerLane), s, p);
    return hipGetLastError();
}
hipError_t launch_finish(const Params& p, hipStream_t s, uint32_t blocks) {
    hipLaunchKernelGGL(k_finish, dim3(blocks), dim3(256), walk_lds_bytes(p.slotsPerLane), s, p);
    return hipGetLastError();
}
hipError_t launch_probe(const Params& p, hipStream_t s, const float* xyz, float* out, float* col, uint32_t n,
                        int mode) {
    const uint32_t blocks = (n + 255) / 256;
    hipLaunchKernelGGL(k_probe, dim3(blocks ? blocks : 1), dim3(256), walk_lds_bytes(p.slotsPerLane), s, p, xyz,
                       out, col, n, mode);
    return hipGetLastError();
}

}  // namespace psgpu

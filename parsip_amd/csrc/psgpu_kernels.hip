// psgpu_kernels.hip — static CDNA4 (gfx950) kernels of the BlobTree polygonizer.
//
// Pipeline for one polygonization of MPUs [begin, begin+count) (the reference's
// Polygonize + CMPUProcessor, PS_Polygonizer.cpp:315-385, 441-829):
//
//   k_precheck  8 lanes per MPU, 2 quads: S1 corner test F>0          (:483-540); field
//               bounds per octant prove surface-free survivors; the rest are queued
//   k_mpu       one wavefront per queued survivor: S2 inside bits of the 8^3 corners
//               (quads of 4 z-consecutive corners), S3 configs, vertex ownership + wave
//               prefix sums for the reference's discovery order, vertex / triangle records
//   k_vertex    its first blocks scan the per-MPU counts into mesh offsets; then one
//               quad per vertex: S4 4-sample root bracket and linear root
//   k_finish    one lane per vertex: S5 value + colour + 3 normal samples as one 4-point
//               walk, the compact mesh; triangle records -> global vertex ids
//
// The tree-evaluating kernels (precheck, mpu, vertex, finish, probe) exist twice: here with
// the generic walk-program interpreter (InterpEval), and specialised per model
// structure at run time by psgpu_jit.cpp (hiprtc), which the host prefers.  Both
// instantiate the same bodies from psgpu_device.h.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "psgpu_device.h"
#include "psgpu_launch.h"

namespace psgpu {

__global__ void __launch_bounds__(256) k_precheck(Params p) {
    extern __shared__ float lds[];
    PSGPU_STAMPED(0, item_, precheck_body<InterpEval>(p, lds));
}

__global__ void __launch_bounds__(256) k_mpu(Params p) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    PSGPU_STAMPED(1, item_, mpu_body<InterpEval>(p, smem, &item_));
}

__global__ void __launch_bounds__(256) k_vertex(Params p) {
    extern __shared__ __attribute__((aligned(16))) float vlds[];
    PSGPU_STAMPED(2, item_, vertex_body<InterpEval>(p, vlds));
}

__global__ void __launch_bounds__(256) k_probe(Params p, const float* __restrict__ xyz, float* __restrict__ out,
                                               float* __restrict__ colOut, uint32_t n, int mode) {
    extern __shared__ __attribute__((aligned(16))) float plds[];
    probe_body<InterpEval>(p, plds, xyz, out, colOut, n, mode);
}

__global__ void __launch_bounds__(256) k_finish(Params p) {
    extern __shared__ __attribute__((aligned(16))) float flds[];
    PSGPU_STAMPED(3, item_, (finish_body<InterpEval, 64>(p, flds)));
}
__global__ void __launch_bounds__(256) k_finish_q(Params p) {
    extern __shared__ __attribute__((aligned(16))) float flds[];
    PSGPU_STAMPED(3, item_, (finish_body<InterpEval, 16>(p, flds)));
}
__global__ void __launch_bounds__(256) k_finish_p(Params p) {
    extern __shared__ __attribute__((aligned(16))) float flds[];
    PSGPU_STAMPED(3, item_, (finish_body<InterpEval, 32>(p, flds)));
}

// Gathered parts of one grid (psgpu_group_gather): a part's triangles get its vertex
// base added to their ids and its MPU offsets (V | T << 32) its (vertex, triangle)
// bases, so the concatenation is the single-device mesh.  One u32 / u64 per lane,
// 4 per thread, grid-stride.
__global__ void __launch_bounds__(256) k_rebase(uint32_t* __restrict__ tris, uint64_t nTri, uint32_t vBase,
                                                uint64_t* __restrict__ offs, uint64_t nOff, uint64_t offBase) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nTri; i += stride) tris[i] += vBase;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nOff; i += stride) offs[i] += offBase;
}

// The totals of a rank's parts (one device, several streams) as one rank's 8 words for
// the RCCL exchange: counts add, the first overflowing MPU is the minimum, errors OR.
__global__ void __launch_bounds__(64) k_sum_totals(TotalsParts tp, uint32_t* __restrict__ out) {
    const int i = threadIdx.x;
    if (i >= 8) return;
    uint32_t v = i == 6 ? 0x7fffffffu : 0u;
    for (int k = 0; k < tp.n; ++k) {
        const uint32_t x = tp.p[k][i];
        if (i == 6) v = x < v ? x : v;
        else if (i == 7) v |= x;
        else v += x;
    }
    out[i] = v;
}

// The blocking export's packing (psgpu_launch.h PackSrc), written straight into the pinned host
// staging over PCIe -- no copy-engine transfers (each cost ~13 us of setup, r04) and one launch:
// every block walks the pieces in order, writes its share of one, then raises its flag for it
// (flags[(piece * gridDim.x + block) * kExportFlagStride] = epoch, a system-scope release), so the host scatters
// piece k while piece k + 1 is still on the link.
__global__ void __launch_bounds__(256) k_export_pack(PackSrc src, uint32_t* __restrict__ dst) {
    uint64_t base = 0;  // the piece's first word
    for (uint32_t k = 0; k < src.pieces; ++k) {
        const uint32_t m0 = (uint32_t)((uint64_t)src.n * k / src.pieces);
        const uint32_t m1 = (uint32_t)((uint64_t)src.n * (k + 1) / src.pieces);
        const uint64_t a = src.offs[m0], b = src.offs[m1];
        const uint32_t v0 = (uint32_t)a, v1 = (uint32_t)b, t0 = (uint32_t)(a >> 32), t1 = (uint32_t)(b >> 32);
        const uint64_t nv = 3ull * (v1 - v0);  // words per vertex array
        const uint64_t ne = 3ull * (t1 - t0);  // triangle corners, two 16-bit local indices a word
        const uint32_t* pos = reinterpret_cast<const uint32_t*>(src.pos) + 3ull * v0;
        const uint32_t* nrm = reinterpret_cast<const uint32_t*>(src.nrm) + 3ull * v0;
        const uint32_t* col = reinterpret_cast<const uint32_t*>(src.col) + 3ull * v0;
        const uint32_t* tri = src.tris + 3ull * t0;
        const uint64_t total = 3 * nv + (ne + 1) / 2;
        // a corner's index relative to its MPU's first vertex (PolyMPUs' uint16 triangles,
        // Polygonize :368): the MPU from a binary search of the piece's triangle offsets
        auto local = [&](uint64_t e) -> uint32_t {
            const uint32_t t = t0 + (uint32_t)(e / 3);
            uint32_t lo = m0, hi = m1;  // offs_t[lo] <= t < offs_t[hi]
            while (hi - lo > 1) {
                const uint32_t mid = (lo + hi) >> 1;
                if ((uint32_t)(src.offs[mid] >> 32) <= t) lo = mid;
                else hi = mid;
            }
            return (tri[e] - (uint32_t)src.offs[lo]) & 0xffffu;
        };
        uint32_t* out = dst + base;
        if (blockIdx.x == src.delayBlock) {  // test hook: a straggling block (its share lands last)
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            while (__builtin_amdgcn_s_memrealtime() - t0 < src.delayTicks) __builtin_amdgcn_s_sleep(32);
        }
        for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (uint64_t)gridDim.x * blockDim.x) {
            uint32_t w;
            if (i < nv) w = pos[i];
            else if (i < 2 * nv) w = nrm[i - nv];
            else if (i < 3 * nv) w = col[i - 2 * nv];
            else {
                const uint64_t e = 2 * (i - 3 * nv);
                w = local(e) | (e + 1 < ne ? local(e + 1) << 16 : 0u);
            }
            out[i] = w;
        }
        base += pack_words(v1 - v0, t1 - t0);
        // every wave's stores acknowledged, then one system-scope release per block (its L2
        // write-back covers the block's words) before the flag: one fence a block, not a wave
        __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0)
        __syncthreads();
        if (threadIdx.x == 0)
            __hip_atomic_store(src.flags + ((uint64_t)k * gridDim.x + blockIdx.x) * kExportFlagStride, src.epoch,
                               __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// ---------------------------------------------------------------------------
// Host-side launch helpers (psgpu_launch.h).
size_t mpu_lds_bytes(uint32_t slots) { return kLdsWaveSlots + 4 * ((size_t)slots * 64 * 4); }
size_t walk_lds_bytes(uint32_t slots) { return 4 * ((size_t)slots * 4 * 64 * 4); }
size_t precheck_lds_bytes(uint32_t slots) { return 4 * ((size_t)slots * 64 * 4); }

hipError_t launch_precheck(const Params& p, hipStream_t s) {
    hipLaunchKernelGGL(k_precheck, dim3(p.preBlocks), dim3(256), precheck_lds_bytes(p.slotsPerLane), s, p);
    return hipGetLastError();
}
hipError_t launch_mpu(const Params& p, hipStream_t s) {
    hipLaunchKernelGGL(k_mpu, dim3(p.mpuBlocks), dim3(256), mpu_lds_bytes(p.slotsPerLane), s, p);
    return hipGetLastError();
}
hipError_t launch_vertex(const Params& p, hipStream_t s, uint32_t blocks) {
    hipLaunchKernelGGL(k_vertex, dim3(blocks), dim3(256), walk_lds_bytes(p.slotsPerLane), s, p);
    return hipGetLastError();
}
hipError_t launch_finish(const Params& p, hipStream_t s, uint32_t blocks, int vpw) {
    if (vpw == 16) hipLaunchKernelGGL(k_finish_q, dim3(blocks), dim3(256), walk_lds_bytes(p.slotsPerLane), s, p);
    else if (vpw == 32) hipLaunchKernelGGL(k_finish_p, dim3(blocks), dim3(256), walk_lds_bytes(p.slotsPerLane), s, p);
    else hipLaunchKernelGGL(k_finish, dim3(blocks), dim3(256), walk_lds_bytes(p.slotsPerLane), s, p);
    return hipGetLastError();
}
hipError_t launch_probe(const Params& p, hipStream_t s, const float* xyz, float* out, float* col, uint32_t n,
                        int mode) {
    const uint32_t blocks = (n + 255) / 256;
    hipLaunchKernelGGL(k_probe, dim3(blocks ? blocks : 1), dim3(256), walk_lds_bytes(p.slotsPerLane), s, p, xyz,
                       out, col, n, mode);
    return hipGetLastError();
}

hipError_t launch_rebase(uint32_t* tris, uint64_t nTri, uint32_t vBase, uint64_t* offs, uint64_t nOff,
                         uint64_t offBase, hipStream_t s) {
    const uint64_t n = nTri > nOff ? nTri : nOff;
    if (n == 0) return hipSuccess;
    uint64_t blocks = (n + 1023) / 1024;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(k_rebase, dim3((uint32_t)blocks), dim3(256), 0, s, tris, nTri, vBase, offs, nOff, offBase);
    return hipGetLastError();
}

hipError_t launch_export_pack(const PackSrc& src, uint32_t* dst, hipStream_t s) {
    hipLaunchKernelGGL(k_export_pack, dim3(src.blocks), dim3(256), 0, s, src, dst);
    return hipGetLastError();
}

// The export's metadata (offsets, S1 flags, per-MPU counts) into the pinned host staging.
__global__ void __launch_bounds__(256) k_export_meta(MetaSrc src, unsigned char* __restrict__ dst) {
    const uint64_t nOff = src.offs ? 2ull * (src.n + 1) : 0, nCnt = src.counts ? 2ull * src.n : 0;
    const uint32_t* offs = reinterpret_cast<const uint32_t*>(src.offs);
    const uint32_t* cnt = reinterpret_cast<const uint32_t*>(src.counts);
    uint32_t* dOff = reinterpret_cast<uint32_t*>(dst + src.oOffs);
    uint32_t* dCnt = reinterpret_cast<uint32_t*>(dst + src.oCnt);
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nOff; i += stride) dOff[i] = offs[i];
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nCnt; i += stride) dCnt[i] = cnt[i];
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < src.n; i += stride)
        dst[src.oPass + i] = src.passed[i];
}
hipError_t launch_export_meta(const MetaSrc& src, unsigned char* dst, hipStream_t s) {
    hipLaunchKernelGGL(k_export_meta, dim3(128), dim3(256), 0, s, src, dst);
    return hipGetLastError();
}

// One reading of the device clock the kernels stamp with (s_memrealtime), stored into mapped
// host memory: the host brackets it with its own clock to map device ticks to host time
// (MPUSTATS, psgpu_download_process_stats).
__global__ void __launch_bounds__(64) k_clock_probe(uint64_t* out) {
    const uint64_t t = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) __hip_atomic_store(out, t, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
hipError_t launch_clock_probe(uint64_t* out, hipStream_t s) {
    hipLaunchKernelGGL(k_clock_probe, dim3(1), dim3(64), 0, s, out);
    return hipGetLastError();
}

hipError_t launch_sum_totals(const TotalsParts& tp, uint32_t* out, hipStream_t s) {
    hipLaunchKernelGGL(k_sum_totals, dim3(1), dim3(64), 0, s, tp, out);
    return hipGetLastError();
}

}  // namespace psgpu

// psgpu_kernels.hip — static CDNA4 (gfx950) kernels of the BlobTree polygonizer.
//
// Pipeline for one polygonization of MPUs [begin, begin+count) (the reference's
// Polygonize + CMPUProcessor, PS_Polygonizer.cpp:315-385, 441-829):
//
//   k_precheck  8 lanes per MPU, 2 quads: S1 corner test F>0          (:483-540)
//   k_compact   one workgroup: ordered list of MPUs that passed S1
//   k_mpu       one wavefront per passing MPU: S2 8^3 field cache in LDS (quads of 4
//               z-consecutive corners), S3 configs, vertex ownership + wave prefix
//               sums for the reference's discovery order, triangle records
//   k_scan      one workgroup: per-MPU vertex/triangle offsets (compact mesh)
//   k_vertex    one quad per vertex: S4 4-sample root bracket, S5 colour + normals
//   k_tris      triangle records -> global vertex ids
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
    __shared__ uint32_t waveMask[4];
    precheck_body<InterpEval>(p, lds, waveMask);
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

// Ordered compaction of the S1 survivors (single workgroup of 1024 threads).
__global__ void __launch_bounds__(1024) k_compact(Params p) {
    __shared__ uint32_t part[1024];
    const uint32_t nWords = (p.mpuCount + 31) / 32;
    const uint32_t per = (nWords + 1023) / 1024;
    const uint32_t w0 = threadIdx.x * per;
    uint32_t cnt = 0;
    for (uint32_t w = w0; w < w0 + per && w < nWords; ++w) cnt += __popc(p.passMask[w]);
    part[threadIdx.x] = cnt;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
        uint32_t v = threadIdx.x >= (uint32_t)off ? part[threadIdx.x - off] : 0u;
        __syncthreads();
        part[threadIdx.x] += v;
        __syncthreads();
    }
    uint32_t base = part[threadIdx.x] - cnt;
    for (uint32_t w = w0; w < w0 + per && w < nWords; ++w) {
        uint32_t mk = p.passMask[w];
        while (mk) {
            int b = __ffs(mk) - 1;
            mk &= mk - 1;
            p.passList[base++] = p.mpuBegin + w * 32 + (uint32_t)b;
        }
    }
    if (threadIdx.x == 1023) p.ctr->passCount = part[1023];
}

// Exclusive scan of per-MPU (V,T) into mesh offsets (single workgroup).
__global__ void __launch_bounds__(1024) k_scan(Params p) {
    __shared__ uint32_t sv[1024], st[1024], surf[1024];
    const uint32_t n = p.ctr->passCount;
    const uint32_t per = (n + 1023) / 1024;
    const uint32_t s0 = threadIdx.x * per;
    uint32_t a = 0, b = 0, sc = 0;
    int firstOv = 0x7fffffff;
    for (uint32_t w = s0; w < s0 + per && w < n; ++w) {
        const uint2 c = p.counts[w];
        a += c.x;
        b += c.y;
        sc += c.y > 0 ? 1u : 0u;
        if ((c.x > 512u || c.y > 512u) && firstOv == 0x7fffffff) firstOv = (int)p.passList[w];
    }
    if (firstOv != 0x7fffffff) atomicMin(&p.ctr->firstOverflow, firstOv);
    sv[threadIdx.x] = a;
    st[threadIdx.x] = b;
    surf[threadIdx.x] = sc;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
        uint32_t x = threadIdx.x >= (uint32_t)off ? sv[threadIdx.x - off] : 0u;
        uint32_t y = threadIdx.x >= (uint32_t)off ? st[threadIdx.x - off] : 0u;
        uint32_t z = threadIdx.x >= (uint32_t)off ? surf[threadIdx.x - off] : 0u;
        __syncthreads();
        sv[threadIdx.x] += x;
        st[threadIdx.x] += y;
        surf[threadIdx.x] += z;
        __syncthreads();
    }
    uint32_t va = sv[threadIdx.x] - a, ta = st[threadIdx.x] - b;
    for (uint32_t w = s0; w < s0 + per && w < n; ++w) {
        const uint2 c = p.counts[w];
        p.voff[w] = va;
        p.toff[w] = ta;
        va += c.x;
        ta += c.y;
    }
    if (threadIdx.x == 1023) {
        p.voff[n] = sv[1023];
        p.toff[n] = st[1023];
        p.ctr->surfaceCount = surf[1023];
    }
}

__global__ void __launch_bounds__(256) k_tris(Params p) {
    const uint32_t nT = min(p.ctr->tCount, p.tcap);
    for (uint32_t t = blockIdx.x * 256 + threadIdx.x; t < nT; t += gridDim.x * 256) {
        const TriRec R = p.tq[t];
        const uint32_t g = p.toff[R.w] + R.tlocal;
        const uint32_t b = p.voff[R.w];
        p.tris[g * 3 + 0] = b + (R.v01 & 0xffffu);
        p.tris[g * 3 + 1] = b + (R.v01 >> 16);
        p.tris[g * 3 + 2] = b + R.v2;
    }
}

// ---------------------------------------------------------------------------
// Host-side launch helpers (psgpu_launch.h).
size_t mpu_lds_bytes(uint32_t slots) { return 4 * (kLdsSlots + (size_t)slots * 64 * 4); }
size_t walk_lds_bytes(uint32_t slots) { return 4 * ((size_t)slots * 4 * 64 * 4); }
size_t precheck_lds_bytes(uint32_t slots) { return 4 * ((size_t)slots * 64 * 4); }

hipError_t launch_precheck(const Params& p, hipStream_t s) {
    const uint32_t blocks = (p.mpuCount + 31) / 32;
    hipLaunchKernelGGL(k_precheck, dim3(blocks), dim3(256), precheck_lds_bytes(p.slotsPerLane), s, p);
    return hipGetLastError();
}
hipError_t launch_compact(const Params& p, hipStream_t s) {
    hipLaunchKernelGGL(k_compact, dim3(1), dim3(1024), 0, s, p);
    return hipGetLastError();
}
hipError_t launch_mpu(const Params& p, hipStream_t s) {
    const uint32_t blocks = (p.mpuCount + 3) / 4;
    hipLaunchKernelGGL(k_mpu, dim3(blocks), dim3(256), mpu_lds_bytes(p.slotsPerLane), s, p);
    return hipGetLastError();
}
hipError_t launch_scan(const Params& p, hipStream_t s) {
    hipLaunchKernelGGL(k_scan, dim3(1), dim3(1024), 0, s, p);
    return hipGetLastError();
}
hipError_t launch_vertex(const Params& p, hipStream_t s, uint32_t blocks) {
    hipLaunchKernelGGL(k_vertex, dim3(blocks), dim3(256), walk_lds_bytes(p.slotsPerLane), s, p);
    return hipGetLastError();
}
hipError_t launch_tris(const Params& p, hipStream_t s, uint32_t blocks) {
    hipLaunchKernelGGL(k_tris, dim3(blocks), dim3(256), 0, s, p);
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

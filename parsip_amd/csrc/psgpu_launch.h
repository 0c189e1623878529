// psgpu_launch.h — host entry points of the kernels in psgpu_kernels.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "psgpu_model.h"

namespace psgpu {

size_t mpu_lds_bytes(uint32_t slots);
size_t walk_lds_bytes(uint32_t slots);
size_t precheck_lds_bytes(uint32_t slots);
hipError_t launch_precheck(const Params& p, hipStream_t s);
hipError_t launch_mpu(const Params& p, hipStream_t s);
hipError_t launch_vertex(const Params& p, hipStream_t s, uint32_t blocks);
hipError_t launch_finish(const Params& p, hipStream_t s, uint32_t blocks, int vpw);  // 64, 32 or 16 vertices per wave
hipError_t launch_probe(const Params& p, hipStream_t s, const float* xyz, float* out, float* col, uint32_t n,
                        int mode);
// tris[0..nTri) += vBase; offs[0..nOff) += offBase (gathered parts, psgpu_group.cpp)
struct TotalsParts {  // the k_finish totals (8 words) of up to 16 parts on one device
    const uint32_t* p[16];
    int n;
};
hipError_t launch_sum_totals(const TotalsParts& tp, uint32_t* out, hipStream_t s);
hipError_t launch_rebase(uint32_t* tris, uint64_t nTri, uint32_t vBase, uint64_t* offs, uint64_t nOff,
                         uint64_t offBase, hipStream_t s);

}  // namespace psgpu

// psgpu_scan.hip — device-wide compaction and scan of the per-MPU results, on rocPRIM's
// single-pass (decoupled look-back) primitives.
//
//   select: ordered list of the MPUs that passed the S1 precheck (the reference keeps
//           MPUs in x-major order, PS_Polygonizer.cpp:360-371; the compact mesh keeps it)
//   scan:   per-MPU (vertices | triangles << 32) counts -> mesh offsets; offs[0] = 0,
//           offs[w+1] = inclusive sum, so offs[n] is the total
#include <hip/hip_runtime.h>

#include <cstring>

#include <rocprim/device/device_scan.hpp>
#include <rocprim/device/device_select.hpp>
#include <rocprim/iterator/counting_iterator.hpp>

#include "psgpu_launch.h"

namespace psgpu {

hipError_t select_passing(void* temp, size_t& bytes, const uint8_t* flags, uint32_t begin, uint32_t* out,
                          uint32_t* count, uint32_t n, hipStream_t s) {
    return rocprim::select(temp, bytes, rocprim::counting_iterator<uint32_t>(begin), flags, out, count, (size_t)n, s);
}

hipError_t scan_counts(void* temp, size_t& bytes, const uint64_t* counts, uint64_t* offs, uint32_t n, hipStream_t s) {
    return rocprim::inclusive_scan(temp, bytes, counts, offs + 1, (size_t)n, rocprim::plus<uint64_t>(), s);
}

}  // namespace psgpu

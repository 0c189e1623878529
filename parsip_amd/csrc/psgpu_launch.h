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
// The compact mesh of `pieces` MPU ranges [N k / pieces, N (k+1) / pieces), packed piece by
// piece as pos | nrm | col (float words) | triangle corners as 16-bit indices relative to their
// MPU's first vertex, two a word (PolyMPUs' triangles): one contiguous buffer the blocking
// export's staging receives piece by piece.  A piece of nv vertices, nt triangles takes
// pack_words(nv, nt) words.
inline __host__ __device__ uint64_t pack_words(uint64_t nv, uint64_t nt) {
    return (9 * nv + (3 * nt + 1) / 2 + 3) & ~(uint64_t)3;  // padded to 16 bytes
}
struct PackSrc {
    const uint64_t* offs;
    const float *pos, *nrm, *col;
    const uint32_t* tris;
    uint32_t n, pieces;
    uint32_t* flags;  // [pieces][blocks] x kExportFlagStride words, set to epoch as each block finishes a piece
    uint32_t epoch, blocks;
    uint32_t delayBlock;  // test hook (PSGPU_OPT_DEBUG bit 24): this block waits delayTicks of the
    uint32_t delayTicks;  // 100 MHz device clock before each piece's share (0xffffffff: none)
};
constexpr uint32_t kExportPackBlocks = 256;
// every block's flag on a 64-B line of its own: the host's poller, re-reading the line of the
// first flag still down, then shares it with no other block's flag write (16 flags a line made
// some calls' whole transfer ~5x slower: DESIGN.md §4 "Blocking", profiles/r06_blocking_tail.txt)
constexpr uint32_t kExportFlagStride = 16;
hipError_t launch_export_pack(const PackSrc& src, uint32_t* dst, hipStream_t s);
struct MetaSrc {  // offs / counts null when not exported
    const uint64_t* offs;
    const uint8_t* passed;
    const uint64_t* counts;
    uint32_t n;
    size_t oOffs, oPass, oCnt;  // byte offsets in dst
};
hipError_t launch_export_meta(const MetaSrc& src, unsigned char* dst, hipStream_t s);
// *out (mapped host memory, device address) = the device clock (s_memrealtime) at one instant
hipError_t launch_clock_probe(uint64_t* out, hipStream_t s);

}  // namespace psgpu

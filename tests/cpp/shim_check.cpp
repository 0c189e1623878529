// Compiles parsip_gpu.hpp against reference-shaped caller types (the caller's own
// SoA structs, here plain aliases of the C-ABI ones plus a PolyMPUs of capacity 8) and
// exercises the host-only entry points; Polygonize must fail loudly without a device.
#include <cstdio>
#include <cstring>

#include "parsip_gpu.hpp"

struct svec3f { float x, y, z; };
struct PolyMPUs8 { PsMPU vMPUs[8]; uint32_t ctMPUs; };
// a caller's MPUSTATS (PS_Polygonizer.h:201-207) with TBB-like opaque members
class Tid { unsigned long id_ = 0; };
class Tick { long long count_ = 0; };
struct MPUSTATS { int idxThread; int bIntersected; Tid threadID; Tick tickStart; Tick tickEnd; };

int main() {
    svec3f lo{-4, -4, -4}, hi{4, 4, 4};
    const uint32_t n = psgpu::CountMPUNeeded(8.0f / 256, lo, hi);
    if (n != 37u * 37u * 37u) { std::printf("count %u\n", n); return 1; }
    static PsSoaBlobPrims prims;
    static PsSoaBlobOps ops;
    static PsSoaPrimMatrices mats;
    static PsSoaBoxMatrices boxes;
    std::memset(&prims, 0, sizeof prims);
    std::memset(&ops, 0, sizeof ops);
    std::memset(&mats, 0, sizeof mats);
    std::memset(&boxes, 0, sizeof boxes);
    prims.ctPrims = 1;
    prims.skeletType[0] = PSGPU_PRIM_POINT;
    if (psgpu::PrepareBBoxes(0.05f, prims, boxes, ops) != PSGPU_RET_SUCCESS) return 2;
    const float iso = PSGPU_ISO_DIST + 5.0f * PSGPU_MIN_CELL_SIZE;
    if (prims.vPrimBoxHiX[0] != iso || prims.bboxLo.x != -iso) return 3;
    static PolyMPUs8 out;
    const int rc = psgpu::Polygonize(0.05f, prims, mats, ops, out);
    const bool haveDevice = psgpu_device_count() > 0;
    std::printf("rc %d device %d\n", rc, (int)haveDevice);
    if (!haveDevice && rc != PSGPU_RET_DEVICE_ERROR) return 4;
    if (haveDevice && rc != PSGPU_RET_MPU_OVERFLOW) return 5;  // 2x2x2 lattice fits? see test
    // the reference's optional lpProcessStats: NULL, nullptr and a caller MPUSTATS* all compile
    static MPUSTATS stats[8];
    const int r1 = psgpu::Polygonize(0.05f, prims, mats, ops, out, NULL);
    const int r2 = psgpu::Polygonize(0.05f, prims, mats, ops, out, nullptr);
    const int r3 = psgpu::Polygonize(0.05f, prims, mats, ops, out, stats);
    if (r1 != rc || r2 != rc || r3 != rc) return 6;
    return 0;
}

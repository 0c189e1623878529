/*
 * parsip_gpu.hpp — header-only C++ face of parsip_gpu.h for Parsip's C++ callers.
 *
 * Mirrors the reference's PS_SimdPoly interface (Parsip100/PS_SimdPoly/include/
 * PS_Polygonizer.h:384-393) and the SimdPoly adapter (Parsip100/ParsipHaptics/include/
 * PS_HighPerformanceRender.h:15-33), so a caller swaps
 *
 *     #include "PS_SimdPoly/include/PS_Polygonizer.h"
 *     PS::SIMDPOLY::Polygonize(cs, prims, mats, ops, polyMPUs);
 * for
 *     #include "parsip_gpu.hpp"
 *     psgpu::Polygonize(cs, prims, mats, ops, polyMPUs);
 *
 * The templates take the reference's own struct types (SOABlobPrims, SOABlobOps,
 * SOABlobPrimMatrices, SOABlobBoxMatrices, PolyMPUs, MPUSTATS) without including the
 * reference headers: the layouts are checked byte for byte at compile time and the
 * bytes are handed to the C-ABI unchanged.  Return codes are the reference's
 * (1 success, -1 parameter error) plus -3..-6 (parsip_gpu.h).
 */
#ifndef PARSIP_GPU_HPP
#define PARSIP_GPU_HPP

#include <cstddef>
#include <cstdint>
#include <memory>
#include <type_traits>

#include "parsip_gpu.h"

namespace psgpu {

namespace detail {
template <class T, class C>
inline const C* as_c(const T& v) {
    static_assert(sizeof(T) == sizeof(C), "struct size differs from the PS_SimdPoly layout");
    static_assert(std::is_trivially_copyable<T>::value, "SoA structs are plain data");
    return reinterpret_cast<const C*>(&v);
}
template <class T, class C>
inline C* as_c_mut(T& v) {
    static_assert(sizeof(T) == sizeof(C), "struct size differs from the PS_SimdPoly layout");
    return reinterpret_cast<C*>(&v);
}
struct CtxDeleter {
    void operator()(psgpu_ctx* c) const { psgpu_destroy(c); }
};
}  // namespace detail

/* One device context (device-resident model and mesh buffers). */
class Context {
public:
    explicit Context(int device = 0) {
        psgpu_ctx* c = nullptr;
        status_ = psgpu_create(device, &c);
        ctx_.reset(c);
    }
    bool ok() const { return ctx_ != nullptr && status_ == PSGPU_RET_SUCCESS; }
    int status() const { return status_; }
    psgpu_ctx* get() const { return ctx_.get(); }

private:
    std::unique_ptr<psgpu_ctx, detail::CtxDeleter> ctx_;
    int status_ = PSGPU_RET_DEVICE_ERROR;
};

/* The calling thread's default context on device 0 (the reference's Polygonize is a
 * free function with process-global state, PS_Polygonizer.cpp:18-19). */
inline Context& default_context() {
    static thread_local Context ctx(0);
    return ctx;
}

/* CountMPUNeeded (PS_Polygonizer.h:384). */
template <class Vec3>
inline uint32_t CountMPUNeeded(float cellsize, const Vec3& lo, const Vec3& hi) {
    const float l[3] = {lo.x, lo.y, lo.z}, h[3] = {hi.x, hi.y, hi.z};
    return psgpu_count_mpus(cellsize, l, h);
}

/* PrepareBBoxes (PS_Polygonizer.h:385). */
template <class Prims, class BoxMats, class Ops>
inline int PrepareBBoxes(float cellsize, Prims& prims, BoxMats& boxMatrices, Ops& ops) {
    return psgpu_prepare_bboxes(cellsize, detail::as_c_mut<Prims, PsSoaBlobPrims>(prims),
                                detail::as_c_mut<BoxMats, PsSoaBoxMatrices>(boxMatrices),
                                detail::as_c_mut<Ops, PsSoaBlobOps>(ops));
}

/* Polygonize (PS_Polygonizer.h:386-391): fills polyMPUs.vMPUs[0..ctMPUs) and ctMPUs.
 * PolyMPUs is {MPU vMPUs[MAX_MPU_COUNT]; U32 ctMPUs;} (PS_Polygonizer.h:196-198);
 * MPUs that fail S1 get zero counts (the reference leaves them stale). */
template <class Prims, class Mats, class Ops, class PolyMPUsT>
inline int Polygonize(float cellsize, const Prims& prims, const Mats& mats, const Ops& ops, PolyMPUsT& polyMPUs,
                      void* lpProcessStats = nullptr, Context* ctx = nullptr) {
    static_assert(sizeof(polyMPUs.vMPUs[0]) == sizeof(PsMPU), "MPU layout");
    (void)lpProcessStats;  // MPUSTATS is filled by the reference only under a compile flag
    Context& c = ctx ? *ctx : default_context();
    if (!c.ok()) return c.status();
    const uint32_t capacity = (uint32_t)(sizeof(polyMPUs.vMPUs) / sizeof(polyMPUs.vMPUs[0]));
    uint32_t ct = 0;
    const int rc = psgpu_polygonize_mpus(c.get(), cellsize, detail::as_c<Prims, PsSoaBlobPrims>(prims),
                                         detail::as_c<Mats, PsSoaPrimMatrices>(mats),
                                         detail::as_c<Ops, PsSoaBlobOps>(ops),
                                         reinterpret_cast<PsMPU*>(&polyMPUs.vMPUs[0]), capacity, &ct, nullptr);
    // on failure nothing was exported: report no MPUs (SimdPoly::draw walks ctMPUs,
    // PS_HighPerformanceRender.cpp:378-426, and must not draw stale ones)
    polyMPUs.ctMPUs = rc == PSGPU_RET_SUCCESS ? ct : 0u;
    return rc;
}

/* SimdPoly-shaped adapter (PS_HighPerformanceRender.h:15-33) over a device-resident
 * compact mesh: setModel once per edit, run() per frame, mesh() for GL / export. */
template <class Prims, class Mats, class Ops>
class SimdPolyGpu {
public:
    explicit SimdPolyGpu(int device = 0) : ctx_(device) {}
    int setModel(const Prims& prims, const Mats& mats, const Ops& ops) {
        if (!ctx_.ok()) return ctx_.status();
        return psgpu_set_model(ctx_.get(), detail::as_c<Prims, PsSoaBlobPrims>(prims),
                               detail::as_c<Mats, PsSoaPrimMatrices>(mats), detail::as_c<Ops, PsSoaBlobOps>(ops));
    }
    /* SimdPoly::run(cellsize) (PS_HighPerformanceRender.cpp:373-376), asynchronous
     * on `stream` (a hipStream_t, NULL = the context's stream) until finish(). */
    int run(float cellsize, void* stream = nullptr) {
        if (!ctx_.ok()) return ctx_.status();
        return psgpu_polygonize(ctx_.get(), cellsize, 0, 0xffffffffu, stream);
    }
    int finish(PsMeshInfo* info) { return psgpu_finish(ctx_.get(), info); }
    int mesh(PsMeshDevice* out) { return psgpu_mesh_device(ctx_.get(), out); }
    Context& context() { return ctx_; }

private:
    Context ctx_;
};

}  // namespace psgpu

#endif /* PARSIP_GPU_HPP */

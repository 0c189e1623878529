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
#include <cstring>
#include <memory>
#include <type_traits>
#include <vector>

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
struct GroupDeleter {
    void operator()(psgpu_group* g) const { psgpu_group_destroy(g); }
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

/* `parts` contexts on one device, each polygonizing a cost-balanced MPU range on a stream of
 * its own (psgpu_group over {device, ..., device}): one polygonization's kernels finish
 * sooner as 2 parts, whose kernel chains fill each other's tails (C3: 0.106 vs 0.114 ms,
 * DESIGN.md §4) -- what SimdPolyT::run waits for; the parts' meshes concatenate in range
 * order to the one-context mesh.  The split comes from a planning run of the lattice
 * (PSGPU_GROUP_BALANCE_PLAN), made once per cell size and scene box. */
/* A part's smallest range: a lattice of fewer than 2 x this many MPUs runs as one chain
 * (C2, 6,859 MPUs: one context 0.048 ms vs 2 parts 0.058 for the kernels; C3, 50,653: 0.114
 * vs 0.106 -- tools/blocking_breakdown.py). */
constexpr uint32_t kBlockingMinPartMpus = 16384;

class Group {
public:
    explicit Group(int device = 0, int parts = 2, uint32_t minPartMpus = kBlockingMinPartMpus) {
        std::vector<int> devs((size_t)(parts > 0 ? parts : 1), device);
        psgpu_group* g = nullptr;
        status_ = psgpu_group_create(devs.data(), (int)devs.size(), &g);
        g_.reset(g);
        if (ok()) status_ = psgpu_group_set_option(g, PSGPU_GROUP_OPT_BALANCE, PSGPU_GROUP_BALANCE_PLAN);
        if (ok()) status_ = psgpu_group_set_option(g, PSGPU_GROUP_OPT_MIN_PART_MPUS, minPartMpus);
    }
    bool ok() const { return g_ != nullptr && status_ == PSGPU_RET_SUCCESS; }
    int status() const { return status_; }
    psgpu_group* get() const { return g_.get(); }

private:
    std::unique_ptr<psgpu_group, detail::GroupDeleter> g_;
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

namespace detail {
template <class Prims, class Mats, class Ops, class PolyMPUsT>
inline int polygonize(float cellsize, const Prims& prims, const Mats& mats, const Ops& ops, PolyMPUsT& polyMPUs,
                      PsMpuProcessStats* processStats, Context* ctx) {
    static_assert(sizeof(polyMPUs.vMPUs[0]) == sizeof(PsMPU), "MPU layout");
    const uint32_t capacity = (uint32_t)(sizeof(polyMPUs.vMPUs) / sizeof(polyMPUs.vMPUs[0]));
    uint32_t ct = 0;
    Context& c = ctx ? *ctx : default_context();
    if (!c.ok()) return c.status();
    const int rc = psgpu_polygonize_mpus_ex(c.get(), cellsize, as_c<Prims, PsSoaBlobPrims>(prims),
                                            as_c<Mats, PsSoaPrimMatrices>(mats), as_c<Ops, PsSoaBlobOps>(ops),
                                            reinterpret_cast<PsMPU*>(&polyMPUs.vMPUs[0]), capacity, &ct, nullptr,
                                            processStats);
    // on failure nothing was exported: report no MPUs (SimdPoly::draw walks ctMPUs,
    // PS_HighPerformanceRender.cpp:378-426, and must not draw stale ones)
    polyMPUs.ctMPUs = rc == PSGPU_RET_SUCCESS ? ct : 0u;
    return rc;
}
}  // namespace detail

/* Polygonize (PS_Polygonizer.h:386-391): fills polyMPUs.vMPUs[0..ctMPUs) and ctMPUs.
 * PolyMPUs is {MPU vMPUs[MAX_MPU_COUNT]; U32 ctMPUs;} (PS_Polygonizer.h:196-198);
 * MPUs that fail S1 get zero counts (the reference leaves them stale).  Runs on `ctx`, or
 * on the calling thread's default context of device 0 (DESIGN.md §4 "Blocking").
 * Without lpProcessStats (omitted, NULL or nullptr) no ticks are recorded. */
template <class Prims, class Mats, class Ops, class PolyMPUsT>
inline int Polygonize(float cellsize, const Prims& prims, const Mats& mats, const Ops& ops, PolyMPUsT& polyMPUs,
                      std::nullptr_t lpProcessStats = nullptr, Context* ctx = nullptr) {
    (void)lpProcessStats;
    return detail::polygonize(cellsize, prims, mats, ops, polyMPUs, nullptr, ctx);
}
/* With the reference's MPUSTATS* lpProcessStats (PS_Polygonizer.h:201-207; handed to
 * CMPUProcessor, .cpp:379, which writes threadID / tickStart / tickEnd of every MPU,
 * .cpp:449-461): lpProcessStats[0..ctMPUs) receives them as parsip_gpu.h's
 * PsMpuProcessStats describes (ticks in tbb::tick_count's CLOCK_REALTIME nanoseconds, the
 * device wave's hardware slot as the thread id; idxThread / bIntersected untouched).  The
 * caller's struct is checked against that layout member by member at compile time. */
template <class Prims, class Mats, class Ops, class PolyMPUsT, class MpuStatsT>
inline int Polygonize(float cellsize, const Prims& prims, const Mats& mats, const Ops& ops, PolyMPUsT& polyMPUs,
                      MpuStatsT* lpProcessStats, Context* ctx = nullptr) {
    static_assert(!std::is_void<MpuStatsT>::value, "pass an MPUSTATS* (PS_Polygonizer.h:201-207), not a void*");
    static_assert(sizeof(MpuStatsT) == sizeof(PsMpuProcessStats), "MPUSTATS size differs from the LP64 layout");
    static_assert(offsetof(MpuStatsT, idxThread) == 0 && offsetof(MpuStatsT, bIntersected) == 4 &&
                      offsetof(MpuStatsT, threadID) == 8 && offsetof(MpuStatsT, tickStart) == 16 &&
                      offsetof(MpuStatsT, tickEnd) == 24,
                  "MPUSTATS member offsets");
    static_assert(sizeof(lpProcessStats->threadID) == 8 && sizeof(lpProcessStats->tickStart) == 8 &&
                      sizeof(lpProcessStats->tickEnd) == 8,
                  "MPUSTATS: 8-byte thread id and ticks (pthread_t, tick_count)");
    return detail::polygonize(cellsize, prims, mats, ops, polyMPUs,
                              reinterpret_cast<PsMpuProcessStats*>(lpProcessStats), ctx);
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

/* ---- BlobTree -> SoA linearizer + SimdPoly-shaped driver ---------------------------
 * SimdPoly (Parsip100/ParsipHaptics/include/PS_HighPerformanceRender.h:15-33, bodies
 * .cpp:42-426) on the device.  `Api` names the caller's BlobTree classes (the
 * ParsipHaptics library: see parsip_gpu_blobtree.hpp; tests: a mock with the same methods):
 *   Api::Node               CBlobNode: isOperator(), getNodeType() (_constSettings.h
 *                           codes), countChildren(), getChild(i), getOctree().lower/.upper,
 *                           getMaterial().diffused, getTransform().getBackwardMatrix()
 *                           (isIdentity(), getRow(float*, int))
 *   Api::SkeletonPrimitive  getSkeleton(); Api::SkeletonPoint/Line/Ring/Disc/Cylinder/Cube/
 *                           Triangle with the reference getters
 *   Api::Pcm, RicciBlend, WarpTwist, WarpTaper, WarpBend, WarpShear  operator parameters
 * linearizeBlobTree follows the reference walk exactly: pre-order ids (an operator takes
 * its id before its children; root op 0), opChildKind = isOpLeft * 2 + isOpRight, boxes
 * from getOctree(), a non-identity backward matrix into the next 12-float row slot
 * (rows 0-2), identity -> idxMatrix 0, Ricci resY = 1/n, -1/-2/-3 on prim / op overflow
 * or a non-binary operator.  Two documented differences: node types are translated to
 * the PS_Polygonizer.h enum the hot path switches on (translateTypes = false writes the
 * raw BlobTree codes as the reference does, SURVEY.md §8(b) "Enum"), and a child's error
 * code is returned instead of being stored as a child id; triangleCompat = true keeps the
 * reference's Triangle packing bug (p2.z written into resX, .cpp:342-344). */
namespace bt {  // _constSettings.h:26-38 (the caller-side BlobTree codes)
enum : int {
    PrimPoint = 0, PrimLine = 1, PrimCylinder = 2, PrimDisc = 3, PrimRing = 4, PrimPolygon = 5, PrimCube = 6,
    PrimTriangle = 7, PrimNull = 12, OpUnion = 14, OpRicciBlend = 19, OpPcm = 22, OpWarpTwist = 24,
    OpWarpTaper = 25, OpWarpBend = 26, OpWarpShear = 27
};
}  // namespace bt

template <class Api>
class SimdPolyT {
public:
    using Node = typename Api::Node;
    static constexpr int kErrPrimOverflow = -1;      // PS_ERROR_PRIM_OVERFLOW (.cpp:10)
    static constexpr int kErrOperatorOverflow = -2;  // PS_ERROR_OPERATOR_OVERFLOW
    static constexpr int kErrNonBinaryOp = -3;       // PS_ERROR_NON_BINARY_OP

    /* `parts`: the polygonization runs as that many cost-balanced MPU ranges on streams of
     * the device (Group; 2 by default: run() waits for one polygonization, and 2 parts
     * finish it sooner than one context) */
    explicit SimdPolyT(int device = 0, bool translateTypes = true, bool triangleCompat = false, int parts = 2)
        : grp_(device, parts), translate_(translateTypes), triangleCompat_(triangleCompat) {
        reset();
    }

    /* SimdPoly::reset (.cpp:31-38): empty SoA (zero-filled, so repeated linearizations
     * give identical bytes). */
    void reset() {
        std::memset(&prims_, 0, sizeof(prims_));
        std::memset(&ops_, 0, sizeof(ops_));
        std::memset(&primMats_, 0, sizeof(primMats_));
        std::memset(&boxMats_, 0, sizeof(boxMats_));
        info_ = PsMeshInfo{};
        haveMesh_ = false;
    }

    /* SimdPoly::linearizeBlobTree (.cpp:366-371): the root's id (0) or -1/-2/-3. */
    int linearizeBlobTree(Node* root) {
        reset();
        int isOperator = 0;
        return linearize(root, -1, isOperator);
    }

    /* SimdPoly::run (.cpp:373-376): upload the SoA and polygonize on the device (blocking;
     * the compact mesh stays in HBM until draw / exportPolyMPUs / mesh). */
    int run(float cellsize) {
        if (!grp_.ok()) return grp_.status();
        if (prims_.ctPrims == 0) return PSGPU_RET_PARAM_ERROR;  // Polygonize :322-323
        int rc = psgpu_group_set_model(grp_.get(), &prims_, &primMats_, &ops_);
        if (rc == PSGPU_RET_SUCCESS) rc = psgpu_group_polygonize(grp_.get(), cellsize);
        if (rc == PSGPU_RET_SUCCESS) rc = psgpu_group_finish(grp_.get(), &info_, nullptr);
        haveMesh_ = false;
        return rc;
    }

    /* SimdPoly::draw (.cpp:378-426) without GL: visits every MPU with triangles, in
     * PolyMPUs order, as the arrays draw() hands to glColorPointer / glNormalPointer /
     * glVertexPointer / glDrawElements: f(pos, nrm, col, ctVertices, tris (MPU-local
     * U16 ids), ctTriangles). */
    template <class F>
    int draw(F&& perMpu) {
        int rc = download();
        if (rc != PSGPU_RET_SUCCESS) return rc;
        std::vector<uint16_t> local;
        for (uint32_t m = 0; m < info_.ctMPUs; ++m) {
            const uint32_t v0 = (uint32_t)offs_[m], v1 = (uint32_t)offs_[m + 1];
            const uint32_t t0 = (uint32_t)(offs_[m] >> 32), t1 = (uint32_t)(offs_[m + 1] >> 32);
            if (t1 == t0) continue;
            local.resize((size_t)(t1 - t0) * 3);
            for (size_t i = 0; i < local.size(); ++i) local[i] = (uint16_t)(tris_[(size_t)t0 * 3 + i] - v0);
            perMpu(&pos_[(size_t)v0 * 3], &nrm_[(size_t)v0 * 3], &col_[(size_t)v0 * 3], v1 - v0, local.data(), t1 - t0);
        }
        return PSGPU_RET_SUCCESS;
    }

    /* The PolyMPUs layout (vMPUs[0..ctMPUs)), for callers that keep the reference's arrays. */
    template <class PolyMPUsT>
    int exportPolyMPUs(PolyMPUsT& polyMPUs) {
        static_assert(sizeof(polyMPUs.vMPUs[0]) == sizeof(PsMPU), "MPU layout");
        const uint32_t capacity = (uint32_t)(sizeof(polyMPUs.vMPUs) / sizeof(polyMPUs.vMPUs[0]));
        uint32_t ct = 0;
        const int rc =
            psgpu_group_export_polympus(grp_.get(), reinterpret_cast<PsMPU*>(&polyMPUs.vMPUs[0]), capacity, &ct);
        polyMPUs.ctMPUs = rc == PSGPU_RET_SUCCESS ? ct : 0u;
        return rc;
    }

    /* the whole mesh in HBM of the device (the parts gathered, vertex ids rebased) */
    int mesh(PsMeshDevice* out) { return psgpu_group_gather(grp_.get(), 0, out); }
    const PsMeshInfo& info() const { return info_; }
    const PsSoaBlobPrims& prims() const { return prims_; }
    const PsSoaBlobOps& ops() const { return ops_; }
    const PsSoaPrimMatrices& primMatrices() const { return primMats_; }
    const PsSoaBoxMatrices& boxMatrices() const { return boxMats_; }
    Group& group() { return grp_; }

private:
    template <class V>
    static void put3(float* x, float* y, float* z, int i, const V& v) {
        x[i] = v.x;
        y[i] = v.y;
        z[i] = v.z;
    }
    uint8_t code(int blobTreeType) const {
        if (!translate_) return (uint8_t)blobTreeType;
        const int t = psgpu_translate_blobtree_type(blobTreeType);
        return (uint8_t)(t < 0 ? blobTreeType : t);
    }

    int linearize(Node* root, int parentID, int& outIsOperator) {
        if (parentID == -1) {  // .cpp:45-64: scene box from the root's octree, identity matrix slot 0
            prims_.bboxLo = PsVec3f{root->getOctree().lower.x, root->getOctree().lower.y, root->getOctree().lower.z};
            prims_.bboxHi = PsVec3f{root->getOctree().upper.x, root->getOctree().upper.y, root->getOctree().upper.z};
            const float identity[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
            primMats_.count = 1;
            boxMats_.count = 1;
            for (int i = 0; i < PSGPU_PRIM_MATRIX_STRIDE; ++i) primMats_.matrix[i] = identity[i];
            for (int i = 0; i < PSGPU_BOX_MATRIX_STRIDE; ++i) boxMats_.matrix[i] = identity[i];
        }
        outIsOperator = root->isOperator() ? 1 : 0;
        const int type = (int)root->getNodeType();
        if (outIsOperator) {  // .cpp:67-161
            if (ops_.ctOps >= PSGPU_MAX_TREE_NODES) return kErrOperatorOverflow;
            const int cur = (int)ops_.ctOps++;
            ops_.opType[cur] = code(type);
            if (root->countChildren() != 2) return kErrNonBinaryOp;
            int isOp[2] = {0, 0}, kid[2] = {0, 0};
            for (int c = 0; c < 2; ++c) {
                kid[c] = linearize(root->getChild(c), cur, isOp[c]);
                if (kid[c] < 0) return kid[c];
            }
            ops_.opLeftChild[cur] = (uint8_t)kid[0];
            ops_.opRightChild[cur] = (uint8_t)kid[1];
            ops_.opChildKind[cur] = (uint8_t)(isOp[0] * 2 + isOp[1]);
            put3(ops_.vBoxLoX, ops_.vBoxLoY, ops_.vBoxLoZ, cur, root->getOctree().lower);
            put3(ops_.vBoxHiX, ops_.vBoxHiY, ops_.vBoxHiZ, cur, root->getOctree().upper);
            switch (type) {
            case bt::OpPcm: {
                auto* n = reinterpret_cast<typename Api::Pcm*>(root);
                ops_.resX[cur] = n->getPropagateLeft();
                ops_.resY[cur] = n->getPropagateRight();
                ops_.resZ[cur] = n->getAlphaLeft();
                ops_.resW[cur] = n->getAlphaRight();
            } break;
            case bt::OpRicciBlend: {
                const float nn = reinterpret_cast<typename Api::RicciBlend*>(root)->getN();
                ops_.resX[cur] = nn;
                if (nn != 0.0f) ops_.resY[cur] = 1.0f / nn;
            } break;
            case bt::OpWarpTwist: {
                auto* n = reinterpret_cast<typename Api::WarpTwist*>(root);
                ops_.resX[cur] = n->getWarpFactor();
                ops_.resY[cur] = static_cast<float>(n->getMajorAxis());
            } break;
            case bt::OpWarpTaper: {
                auto* n = reinterpret_cast<typename Api::WarpTaper*>(root);
                ops_.resX[cur] = n->getWarpFactor();
                ops_.resY[cur] = static_cast<float>(n->getAxisAlong());
                ops_.resZ[cur] = static_cast<float>(n->getAxisTaper());
            } break;
            case bt::OpWarpBend: {
                auto* n = reinterpret_cast<typename Api::WarpBend*>(root);
                ops_.resX[cur] = n->getBendRate();
                ops_.resY[cur] = n->getBendCenter();
                ops_.resZ[cur] = n->getBendRegion().left;
                ops_.resW[cur] = n->getBendRegion().right;
            } break;
            case bt::OpWarpShear: {
                auto* n = reinterpret_cast<typename Api::WarpShear*>(root);
                ops_.resX[cur] = n->getWarpFactor();
                ops_.resY[cur] = static_cast<float>(n->getAxisAlong());
                ops_.resZ[cur] = static_cast<float>(n->getAxisDependent());
            } break;
            default: break;
            }
            return cur;
        }
        // primitive (.cpp:162-363)
        if (prims_.ctPrims >= PSGPU_MAX_TREE_NODES) return kErrPrimOverflow;
        const int cur = (int)prims_.ctPrims++;
        const auto d = root->getMaterial().diffused;
        prims_.colorX[cur] = d.x;
        prims_.colorY[cur] = d.y;
        prims_.colorZ[cur] = d.z;
        put3(prims_.vPrimBoxLoX, prims_.vPrimBoxLoY, prims_.vPrimBoxLoZ, cur, root->getOctree().lower);
        put3(prims_.vPrimBoxHiX, prims_.vPrimBoxHiY, prims_.vPrimBoxHiZ, cur, root->getOctree().upper);
        const auto back = root->getTransform().getBackwardMatrix();
        if (back.isIdentity()) {
            prims_.idxMatrix[cur] = 0;
        } else {
            // 128 slots with slot 0 the identity: a 128th transformed primitive has no slot
            // (the reference adapter would write past SOABlobPrimMatrices::matrix)
            if (primMats_.count >= PSGPU_MAX_TREE_NODES) return kErrPrimOverflow;
            const uint32_t k = primMats_.count;
            prims_.idxMatrix[cur] = (uint8_t)k;
            float row[16];
            for (int r = 0; r < 4; ++r) back.getRow(&row[4 * r], r);
            for (int i = 0; i < PSGPU_PRIM_MATRIX_STRIDE; ++i) primMats_.matrix[k * PSGPU_PRIM_MATRIX_STRIDE + i] = row[i];
            primMats_.count++;
        }
        prims_.skeletType[cur] = code(type);
        auto* sp = reinterpret_cast<typename Api::SkeletonPrimitive*>(root);
        switch (type) {
        case bt::PrimPoint: {
            auto* s = reinterpret_cast<typename Api::SkeletonPoint*>(sp->getSkeleton());
            put3(prims_.posX, prims_.posY, prims_.posZ, cur, s->getPosition());
        } break;
        case bt::PrimLine: {
            auto* s = reinterpret_cast<typename Api::SkeletonLine*>(sp->getSkeleton());
            put3(prims_.posX, prims_.posY, prims_.posZ, cur, s->getStartPosition());
            put3(prims_.dirX, prims_.dirY, prims_.dirZ, cur, s->getEndPosition());
        } break;
        case bt::PrimRing:
        case bt::PrimDisc: {
            float r;
            if (type == bt::PrimRing) {
                auto* s = reinterpret_cast<typename Api::SkeletonRing*>(sp->getSkeleton());
                put3(prims_.posX, prims_.posY, prims_.posZ, cur, s->getPosition());
                put3(prims_.dirX, prims_.dirY, prims_.dirZ, cur, s->getDirection());
                r = s->getRadius();
            } else {
                auto* s = reinterpret_cast<typename Api::SkeletonDisc*>(sp->getSkeleton());
                put3(prims_.posX, prims_.posY, prims_.posZ, cur, s->getPosition());
                put3(prims_.dirX, prims_.dirY, prims_.dirZ, cur, s->getDirection());
                r = s->getRadius();
            }
            prims_.resX[cur] = r;
            prims_.resY[cur] = r * r;
        } break;
        case bt::PrimCylinder: {
            auto* s = reinterpret_cast<typename Api::SkeletonCylinder*>(sp->getSkeleton());
            put3(prims_.posX, prims_.posY, prims_.posZ, cur, s->getPosition());
            put3(prims_.dirX, prims_.dirY, prims_.dirZ, cur, s->getDirection());
            prims_.resX[cur] = s->getRadius();
            prims_.resY[cur] = s->getHeight();
        } break;
        case bt::PrimCube: {
            auto* s = reinterpret_cast<typename Api::SkeletonCube*>(sp->getSkeleton());
            put3(prims_.posX, prims_.posY, prims_.posZ, cur, s->getPosition());
            prims_.resX[cur] = s->getSide();
        } break;
        case bt::PrimTriangle: {
            auto* s = reinterpret_cast<typename Api::SkeletonTriangle*>(sp->getSkeleton());
            const auto p0 = s->getTriangleCorner(0), p1 = s->getTriangleCorner(1), p2 = s->getTriangleCorner(2);
            put3(prims_.posX, prims_.posY, prims_.posZ, cur, p0);
            put3(prims_.dirX, prims_.dirY, prims_.dirZ, cur, p1);
            prims_.resX[cur] = p2.x;
            prims_.resY[cur] = p2.y;
            if (triangleCompat_) prims_.resX[cur] = p2.z;  // the reference adapter's bug
            else prims_.resZ[cur] = p2.z;
        } break;
        case bt::PrimNull:
            prims_.posX[cur] = prims_.posY[cur] = prims_.posZ[cur] = 0.0f;
            break;
        default:  // "has not been implemented in compact mode yet" (.cpp:353-359): parameters stay 0
            break;
        }
        return cur;
    }

    int download() {
        if (haveMesh_) return PSGPU_RET_SUCCESS;
        PsMeshInfo I;
        int rc = psgpu_group_finish(grp_.get(), &I, nullptr);
        if (rc != PSGPU_RET_SUCCESS) return rc;
        info_ = I;
        pos_.resize((size_t)I.ctVertices * 3);
        nrm_.resize(pos_.size());
        col_.resize(pos_.size());
        tris_.resize((size_t)I.ctTriangles * 3);
        offs_.resize((size_t)I.ctMPUs + 1);
        rc = psgpu_group_download_mesh(grp_.get(), pos_.data(), nrm_.data(), col_.data(), tris_.data(), offs_.data());
        haveMesh_ = rc == PSGPU_RET_SUCCESS;
        return rc;
    }

    Group grp_;
    bool translate_, triangleCompat_;
    PsSoaBlobPrims prims_;
    PsSoaBlobOps ops_;
    PsSoaPrimMatrices primMats_;
    PsSoaBoxMatrices boxMats_;
    PsMeshInfo info_{};
    bool haveMesh_ = false;
    std::vector<float> pos_, nrm_, col_;
    std::vector<uint32_t> tris_;
    std::vector<uint64_t> offs_;
};

}  // namespace psgpu

/* The reference's own names for the drop-in: a host that includes this header instead
 * of PS_SimdPoly/include/PS_Polygonizer.h keeps calling PS::SIMDPOLY::Polygonize etc.
 * (PS_Polygonizer.h:384-393) on its PS::SIMDPOLY SoA types.  Define PSGPU_NO_PS_NAMES
 * when both headers must coexist. */
#ifndef PSGPU_NO_PS_NAMES
namespace PS {
namespace SIMDPOLY {
typedef PsSoaBlobPrims SOABlobPrims;
typedef PsSoaBlobOps SOABlobOps;
typedef PsSoaPrimMatrices SOABlobPrimMatrices;
typedef PsSoaBoxMatrices SOABlobBoxMatrices;
typedef PsMPU MPU;
typedef PsMpuProcessStats MPUSTATS;  /* PS_Polygonizer.h:201-207, LP64 layout (parsip_gpu.h) */
struct PolyMPUs {  /* PS_Polygonizer.h:196-198 */
    MPU vMPUs[PSGPU_MAX_MPU_COUNT];
    uint32_t ctMPUs;
};
using psgpu::CountMPUNeeded;
using psgpu::Polygonize;
using psgpu::PrepareBBoxes;
/* PrintThreadResults (PS_Polygonizer.h:393, .cpp:414-428): one entry per device context
 * that ran a Polygonize since the last call (the library's worker; psgpu_print_thread_results
 * in parsip_gpu.h).  As the reference, the arrays must hold one U32 per entry:
 * psgpu_thread_result_count() says how many. */
inline void PrintThreadResults(int ctAttempts, uint32_t* lpThreadProcessed = NULL, uint32_t* lpThreadCrossed = NULL) {
    psgpu_print_thread_results(ctAttempts, lpThreadProcessed, lpThreadCrossed, 0xffffffffu, 1);
}
}  // namespace SIMDPOLY
}  // namespace PS
#endif

#endif /* PARSIP_GPU_HPP */

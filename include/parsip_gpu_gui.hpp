/*
 * parsip_gpu_gui.hpp — header-only C++ face of the compat mode (include/parsip_gpu_gui.h):
 * ParsipHaptics' own polygonizer, CParsipOptimized over a COMPACTBLOBTREE
 * (Parsip100/ParsipHaptics/include/CPolyParsipOptimized.{h,cpp}, CompactBlobTree.{h,cpp}),
 * on the MI355X.
 *
 *   psgpu::CompactTreeT<Api>      COMPACTBLOBTREE::convert (CompactBlobTree.cpp:25-408) over
 *                                 the caller's BlobTree classes: pre-order operator ids, DFS
 *                                 primitive ids, a matrix slot per non-identity backward
 *                                 matrix, the operator parameters of :159-240 and primitive
 *                                 fields of :287-400, the same error codes.
 *   psgpu::ParsipOptimizedT<Api>  CParsipOptimized (CPolyParsipOptimized.h:226-305): setup,
 *                                 run, countMPUs and the stats* accessors, drawMesh (per-MPU
 *                                 arrays to a visitor), exportMesh (one mesh).
 *   psgpu::Run_Polygonizer        Run_Polygonizer (:615-628).
 *
 * `Api` names the caller's classes as for SimdPolyT (parsip_gpu.hpp), plus
 *   Api::Node::getID(), the material's diffuse alpha (diffused.w),
 *   Api::QuadricPoint with getPosition(), getFieldRadius(), getFieldScale(), and
 *   Api::Instance with getOriginalNode().
 * The PCM contact state: ParsipOptimizedT::pcmState / setPcmState (parsip_gpu_gui.h).
 * parsip_gpu_blobtree.hpp binds it to ParsipHaptics' PS::BLOBTREE classes.
 */
#ifndef PARSIP_GPU_GUI_HPP
#define PARSIP_GPU_GUI_HPP

#include <cstring>
#include <memory>
#include <vector>

#include "parsip_gpu.hpp"
#include "parsip_gpu_gui.h"

namespace psgpu {

template <class Api>
class CompactTreeT {
public:
    using Node = typename Api::Node;
    static constexpr int kErrOpsOverflow = -1;        // ERR_OPS_OVERFLOW (CompactBlobTree.cpp:8)
    static constexpr int kErrPrimsOverflow = -2;      // ERR_PRIMS_OVERFLOW
    static constexpr int kErrKidsOverflow = -3;       // ERR_KIDS_OVERFLOW
    static constexpr int kErrParamError = -4;         // ERR_PARAM_ERROR
    static constexpr int kErrNodeNotRecognized = -5;  // ERR_NODE_NOT_RECOGNIZED
    static constexpr int kMaxKids = 1024;             // MAX_COMPACT_KIDS_COUNT (CompactBlobTree.h:14)

    /* COMPACTBLOBTREE::convert: the root's id (0) or a negative ERR_* code. */
    int convert(Node* root) {
        prims.clear();
        ops.clear();
        kids.clear();
        mtx.assign(1, PsGuiMatrix{{{1, 0, 0, 0}, {0, 1, 0, 0}, {0, 0, 1, 0}, {0, 0, 0, 1}}});
        converted_.clear();
        if (!root) return kErrParamError;
        int isOp = 0;
        const int res = rec(root, isOp);
        // updateInstanceNodes (:410-431): an Instance's origin by its node id
        for (PsGuiPrim& p : prims)
            if (p.type == PSGUI_PRIM_INSTANCE && (int)p.res1[0] == -1)
                for (const auto& c : converted_)
                    if (c.first == (int)p.res1[1]) {
                        p.res1[0] = (float)c.second;
                        break;
                    }
        return res;
    }

    std::vector<PsGuiPrim> prims;
    std::vector<PsGuiOp> ops;
    std::vector<uint32_t> kids;
    std::vector<PsGuiMatrix> mtx;

private:
    std::vector<std::pair<int, int>> converted_;  // m_lstConvertedIds: (node id, compact id)

    template <class V>
    static void set4(float* d, const V& v, float w = 0.0f) {
        d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = w;
    }
    static void splat(float* d, float v) { d[0] = d[1] = d[2] = d[3] = v; }

    template <class N>
    uint32_t matrix_index(N* n) {  // :118-135 / :266-283
        const auto back = n->getTransform().getBackwardMatrix();
        if (back.isIdentity()) return 0;
        PsGuiMatrix m;
        for (int r = 0; r < 4; ++r) back.getRow(m.r[r], r);
        mtx.push_back(m);
        return (uint32_t)(mtx.size() - 1);
    }

    int rec(Node* n, int& isOp) {
        const int type = (int)n->getNodeType();
        isOp = n->isOperator() ? 1 : 0;
        if (isOp) {  // :96-241
            const int cur = (int)ops.size();
            ops.push_back(PsGuiOp{});
            PsGuiOp o{};
            o.type = type;
            o.orgID = n->getID();
            set4(o.octLo, n->getOctree().lower);
            set4(o.octHi, n->getOctree().upper);
            o.idxMtx = matrix_index(n);
            if ((int)n->countChildren() > kMaxKids) { ops[cur] = o; return kErrKidsOverflow; }
            o.ctKids = (int)n->countChildren();
            o.kidStart = (uint32_t)kids.size();
            kids.resize(kids.size() + (size_t)o.ctKids, 0u);
            ops[cur] = o;
            for (int i = 0; i < o.ctKids; ++i) {
                int kidIsOp = 0;
                const int kid = rec(n->getChild((size_t)i), kidIsOp);
                if (kid < 0) return kid;
                kids[o.kidStart + (uint32_t)i] = (uint32_t)kid | ((uint32_t)kidIsOp << 16);
            }
            float* prm = ops[cur].params;
            switch (type) {
            case PSGUI_OP_UNION: case PSGUI_OP_BLEND: case PSGUI_OP_DIF: case PSGUI_OP_SMOOTHDIF:
            case PSGUI_OP_INTERSECT:
                break;
            case PSGUI_OP_PCM: {
                auto* p = reinterpret_cast<typename Api::Pcm*>(n);
                prm[0] = p->getPropagateLeft(); prm[1] = p->getPropagateRight();
                prm[2] = p->getAlphaLeft(); prm[3] = p->getAlphaRight();
            } break;
            case PSGUI_OP_RICCIBLEND: {
                const float nn = reinterpret_cast<typename Api::RicciBlend*>(n)->getN();
                prm[0] = nn;
                if (nn != 0.0f) prm[1] = 1.0f / nn;
            } break;
            case PSGUI_OP_WARPTWIST: {
                auto* w = reinterpret_cast<typename Api::WarpTwist*>(n);
                prm[0] = w->getWarpFactor(); prm[1] = static_cast<float>(w->getMajorAxis());
            } break;
            case PSGUI_OP_WARPTAPER: {
                auto* w = reinterpret_cast<typename Api::WarpTaper*>(n);
                prm[0] = w->getWarpFactor(); prm[1] = static_cast<float>(w->getAxisAlong());
                prm[2] = static_cast<float>(w->getAxisTaper());
            } break;
            case PSGUI_OP_WARPBEND: {
                auto* w = reinterpret_cast<typename Api::WarpBend*>(n);
                prm[0] = w->getBendRate(); prm[1] = w->getBendCenter();
                prm[2] = w->getBendRegion().left; prm[3] = w->getBendRegion().right;
            } break;
            case PSGUI_OP_WARPSHEAR: {
                auto* w = reinterpret_cast<typename Api::WarpShear*>(n);
                prm[0] = w->getWarpFactor(); prm[1] = static_cast<float>(w->getAxisAlong());
                prm[2] = static_cast<float>(w->getAxisDependent());
            } break;
            default:
                return kErrNodeNotRecognized;
            }
            converted_.push_back({n->getID(), cur});
            return cur;
        }
        const int cur = (int)prims.size();  // :242-401
        PsGuiPrim p{};
        p.type = type;
        p.orgID = n->getID();
        const auto d = n->getMaterial().diffused;
        p.color[0] = d.x; p.color[1] = d.y; p.color[2] = d.z; p.color[3] = d.w;
        set4(p.octLo, n->getOctree().lower);
        set4(p.octHi, n->getOctree().upper);
        p.idxMtx = matrix_index(n);
        switch (type) {
        case PSGUI_PRIM_POINT: {
            auto* s = reinterpret_cast<typename Api::SkeletonPoint*>(
                reinterpret_cast<typename Api::SkeletonPrimitive*>(n)->getSkeleton());
            set4(p.pos, s->getPosition());
        } break;
        case PSGUI_PRIM_LINE: {
            auto* s = reinterpret_cast<typename Api::SkeletonLine*>(
                reinterpret_cast<typename Api::SkeletonPrimitive*>(n)->getSkeleton());
            set4(p.res1, s->getStartPosition());
            set4(p.res2, s->getEndPosition());
        } break;
        case PSGUI_PRIM_RING: {
            auto* s = reinterpret_cast<typename Api::SkeletonRing*>(
                reinterpret_cast<typename Api::SkeletonPrimitive*>(n)->getSkeleton());
            set4(p.pos, s->getPosition());
            set4(p.dir, s->getDirection());
            const float r = s->getRadius();
            splat(p.res1, r);
            splat(p.res2, r * r);
        } break;
        case PSGUI_PRIM_DISC: {
            auto* s = reinterpret_cast<typename Api::SkeletonDisc*>(
                reinterpret_cast<typename Api::SkeletonPrimitive*>(n)->getSkeleton());
            set4(p.pos, s->getPosition());
            set4(p.dir, s->getDirection());
            const float r = s->getRadius();
            splat(p.res1, r);
            splat(p.res2, r * r);
        } break;
        case PSGUI_PRIM_CYLINDER: {
            auto* s = reinterpret_cast<typename Api::SkeletonCylinder*>(
                reinterpret_cast<typename Api::SkeletonPrimitive*>(n)->getSkeleton());
            set4(p.pos, s->getPosition());
            set4(p.dir, s->getDirection());
            splat(p.res1, s->getRadius());
            splat(p.res2, s->getHeight());
        } break;
        case PSGUI_PRIM_CUBE: {
            auto* s = reinterpret_cast<typename Api::SkeletonCube*>(
                reinterpret_cast<typename Api::SkeletonPrimitive*>(n)->getSkeleton());
            set4(p.pos, s->getPosition());
            splat(p.res1, s->getSide());
        } break;
        case PSGUI_PRIM_TRIANGLE: {
            auto* s = reinterpret_cast<typename Api::SkeletonTriangle*>(
                reinterpret_cast<typename Api::SkeletonPrimitive*>(n)->getSkeleton());
            set4(p.pos, s->getTriangleCorner(0));
            set4(p.res1, s->getTriangleCorner(1));
            set4(p.res2, s->getTriangleCorner(2));
        } break;
        case PSGUI_PRIM_QUADRICPOINT: {
            auto* q = reinterpret_cast<typename Api::QuadricPoint*>(n);
            set4(p.pos, q->getPosition());
            splat(p.res1, q->getFieldRadius());
            splat(p.res2, q->getFieldScale());
        } break;
        case PSGUI_PRIM_NULL:
            break;
        case PSGUI_PRIM_INSTANCE: {  // :383-391, resolved after the walk
            Node* o = reinterpret_cast<typename Api::Instance*>(n)->getOriginalNode();
            if (!o) {
                prims.push_back(p);
                return kErrParamError;
            }
            p.res1[0] = -1.0f;
            p.res1[1] = (float)o->getID();
            p.res1[2] = o->isOperator() ? 1.0f : 0.0f;
            p.res1[3] = (float)(int)o->getNodeType();
        } break;
        default:
            prims.push_back(p);
            return kErrNodeNotRecognized;
        }
        prims.push_back(p);
        converted_.push_back({n->getID(), cur});
        return cur;
    }
};

template <class Api>
class ParsipOptimizedT {
public:
    using Node = typename Api::Node;

    explicit ParsipOptimizedT(int device = 0) { status_ = psgpu_gui_create(device, &g_); }
    ~ParsipOptimizedT() { psgpu_gui_destroy(g_); }
    ParsipOptimizedT(const ParsipOptimizedT&) = delete;
    ParsipOptimizedT& operator=(const ParsipOptimizedT&) = delete;
    bool ok() const { return g_ != nullptr && status_ == PSGPU_RET_SUCCESS; }
    int status() const { return status_; }

    /* setup (:330-390) from the caller's tree: convert (COMPACTBLOBTREE) + upload; the
     * lattice over `lower, upper` (the root's octree in Run_Polygonizer).  Returns the
     * conversion's negative code, a PSGPU_RET_* / PSGUI_RET_* code, or PSGPU_RET_SUCCESS. */
    template <class V3>
    int setup(Node* root, const V3& lower, const V3& upper, int id, float cellsize, float isovalue = 0.5f) {
        if (!ok()) return status_;
        const int code = tree_.convert(root);
        if (code < 0) return code;
        id_ = id;
        lo_[0] = lower.x; lo_[1] = lower.y; lo_[2] = lower.z;
        hi_[0] = upper.x; hi_[1] = upper.y; hi_[2] = upper.z;
        cs_ = cellsize;
        iso_ = isovalue;
        haveMesh_ = false;
        return psgpu_gui_set_tree(g_, tree_.prims.data(), (uint32_t)tree_.prims.size(), tree_.ops.data(),
                                  (uint32_t)tree_.ops.size(), tree_.kids.data(), (uint32_t)tree_.kids.size(),
                                  tree_.mtx.data(), (uint32_t)tree_.mtx.size());
    }

    /* run (:392-410): blocking, statistics ready afterwards. */
    int run() {
        if (!ok()) return status_;
        haveMesh_ = false;
        int rc = psgpu_gui_polygonize(g_, lo_, hi_, cs_, iso_);
        if (rc == PSGPU_RET_SUCCESS) rc = psgpu_gui_finish(g_, &info_);
        return rc;
    }

    // statistics (:487-527, .h:278-302)
    size_t countMPUs() const { return info_.ctMPUs; }
    size_t statsIntersectedMPUs() const { return info_.ctIntersectedMPUs; }
    void statsMeshInfo(size_t& ctVertices, size_t& ctFaces) const {
        ctVertices = info_.ctVertices;
        ctFaces = info_.ctTriangles;
    }
    size_t statsTotalFieldEvals() const { return (size_t)info_.ctFieldEvals; }
    size_t statsIntersectedCellsCount() const { return info_.ctIntersectedCells; }
    size_t statsTotalCellInAllMPUs() const { return (size_t)(PSGUI_GRID_DIM - 1) * (PSGUI_GRID_DIM - 1) * (PSGUI_GRID_DIM - 1) * countMPUs(); }
    size_t statsTotalCellsInIntersectedMPUs() const { return (size_t)info_.ctCellsInIntersectedMPUs; }
    const PsGuiInfo& info() const { return info_; }
    /* the PCM contact state (maxCompressionLeft, Right) the next run reads */
    int pcmState(float state[2]) { return ok() ? psgpu_gui_get_pcm_state(g_, state) : status_; }
    int setPcmState(const float state[2]) { return ok() ? psgpu_gui_set_pcm_state(g_, state) : status_; }
    int id() const { return id_; }
    const CompactTreeT<Api>& compactTree() const { return tree_; }

    /* drawMesh (:425-434) without GL: every MPU with faces, lattice order:
     * f(pos, nrm, rgba, ctVertices, tris (MPU-local ids), ctTriangles). */
    template <class F>
    int drawMesh(F&& perMpu) {
        const int rc = download();
        if (rc != PSGPU_RET_SUCCESS) return rc;
        std::vector<uint32_t> local;
        for (uint32_t m = 0; m < info_.ctLatticeMPUs; ++m) {
            const uint32_t v0 = (uint32_t)offs_[m], v1 = (uint32_t)offs_[m + 1];
            const uint32_t t0 = (uint32_t)(offs_[m] >> 32), t1 = (uint32_t)(offs_[m + 1] >> 32);
            if (t1 == t0) continue;
            local.resize((size_t)(t1 - t0) * 3);
            for (size_t i = 0; i < local.size(); ++i) local[i] = tris_[(size_t)t0 * 3 + i] - v0;
            perMpu(&pos_[(size_t)v0 * 3], &nrm_[(size_t)v0 * 3], &col_[(size_t)v0 * 4], v1 - v0, local.data(), t1 - t0);
        }
        return PSGPU_RET_SUCCESS;
    }

    /* exportMesh (:594-613): one mesh (mesh-wide triangle ids). */
    int exportMesh(std::vector<float>& pos, std::vector<float>& nrm, std::vector<float>& rgba,
                   std::vector<uint32_t>& tris) {
        const int rc = download();
        if (rc != PSGPU_RET_SUCCESS) return rc;
        pos = pos_;
        nrm = nrm_;
        rgba = col_;
        tris = tris_;
        return info_.ctTriangles > 0 ? PSGPU_RET_SUCCESS : PSGPU_RET_PARAM_ERROR;
    }

private:
    int download() {
        if (haveMesh_) return PSGPU_RET_SUCCESS;
        pos_.resize((size_t)info_.ctVertices * 3);
        nrm_.resize(pos_.size());
        col_.resize((size_t)info_.ctVertices * 4);
        tris_.resize((size_t)info_.ctTriangles * 3);
        offs_.resize((size_t)info_.ctLatticeMPUs + 1);
        const int rc = psgpu_gui_download(g_, pos_.data(), nrm_.data(), col_.data(), tris_.data(), offs_.data(),
                                          nullptr);
        haveMesh_ = rc == PSGPU_RET_SUCCESS;
        return rc;
    }

    psgpu_gui* g_ = nullptr;
    int status_ = PSGPU_RET_DEVICE_ERROR;
    CompactTreeT<Api> tree_;
    float lo_[3] = {0, 0, 0}, hi_[3] = {0, 0, 0};
    float cs_ = 0.25f, iso_ = 0.5f;
    int id_ = 0;
    PsGuiInfo info_{};
    bool haveMesh_ = false;
    std::vector<float> pos_, nrm_, col_;
    std::vector<uint32_t> tris_;
    std::vector<uint64_t> offs_;
};

/* Run_Polygonizer (:615-628): convert, setup over the root's octree, run; nullptr on a
 * conversion or device error. */
template <class Api>
std::unique_ptr<ParsipOptimizedT<Api>> Run_Polygonizer(typename Api::Node* input, float cellSize = 0.25f,
                                                       float isovalue = 0.5f, int device = 0) {
    if (!input) return nullptr;
    std::unique_ptr<ParsipOptimizedT<Api>> p(new ParsipOptimizedT<Api>(device));
    const auto oct = input->getOctree();
    if (p->setup(input, oct.lower, oct.upper, input->getID(), cellSize, isovalue) != PSGPU_RET_SUCCESS) return nullptr;
    if (p->run() != PSGPU_RET_SUCCESS) return nullptr;
    return p;
}

}  // namespace psgpu

#endif /* PARSIP_GPU_GUI_HPP */

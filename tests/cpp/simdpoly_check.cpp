// The C++ drop-in faces compiled as a ParsipHaptics host would use them:
//
//   tree <tree.txt> <soa.bin> [translate compat]
//        SimdPoly (include/parsip_gpu_blobtree.hpp) over the mock BlobTree: linearizeBlobTree
//        of the pre-order tree file written by tests/test_cpp_simdpoly.py; writes the return
//        code and the SoA bytes (prims | prim matrices | ops | box matrices).
//   run <tree.txt> <cellsize> <mesh.bin>
//        the same, then SimdPoly::run on device 0 and SimdPoly::draw's per-MPU arrays
//        (ctV, ctT, pos, nrm, col, U16 triangles per drawn MPU) into mesh.bin.
//   gui-tree <tree.txt> <compact.bin>
//        COMPACTBLOBTREE::convert (parsip_gpu_gui.hpp, CompactTreeT) of the same tree file:
//        code, counts, then the prim / op / kid / matrix arrays.
//   gui-run <tree.txt> <cellsize> <mesh.bin>
//        PS::CParsipOptimizedGpu: setup over the root's octree + run on device 0, statistics
//        and exportMesh (V, T, pos, nrm, rgba, mesh-wide triangle ids) into mesh.bin.
//   soa <soa.bin> <cellsize> <polympus.bin>
//        PS::SIMDPOLY::Polygonize on a PS::SIMDPOLY::PolyMPUs (24,000 MPUs, the reference's
//        capacity); writes rc, ctMPUs and the MPUs.
//   soa-stats <soa.bin> <cellsize> <stats.bin>
//        the same with the reference's MPUSTATS* lpProcessStats: a caller-side MPUSTATS whose
//        thread id and ticks are classes with private members, as legacy TBB's tbb_thread::id
//        and tbb::tick_count; writes rc, ctMPUs, the host clock (CLOCK_REALTIME ns) before and
//        after the call, then the ctMPUs 32-byte records.
//   soa-mt <soa.bin> <cellsize> <out.bin>
//        4 host threads call PS::SIMDPOLY::Polygonize 3 times each, each into its own PolyMPUs
//        (each thread runs on its own default context); writes every call's rc, ctMPUs and a
//        hash of the filled records, PrintThreadResults(3, ...)'s entries, then thread 0's MPUs.
#include <time.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <memory>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "mock_blobtree.hpp"
#include "parsip_gpu_blobtree.hpp"

using namespace PS::BLOBTREE;

namespace {

// One node per line, pre-order: type nKids lo3 hi3 diffuse3 identity back16 params12 alpha id
// (params: a3 b3 c3 r h and res0..3 for operators, as the writer documents).
CBlobNode* read_node(std::istream& in, std::vector<std::unique_ptr<CBlobNode>>& own) {
    int type, nk;
    in >> type >> nk;
    if (!in) return nullptr;
    float v[3 + 3 + 3 + 1 + 16 + 12 + 2];
    for (float& f : v) in >> f;
    CBlobNode* n;
    if (type == 10) {  // QuadricPoint: position, radius, scale in the skeleton slots
        CQuadricPoint* q = new CQuadricPoint();
        q->pos = vec3f{v[26], v[27], v[28]};
        q->radius = v[35];
        q->scale = v[36];
        n = q;
    } else if (type == 13) {  // Instance: the origin's node id in the first skeleton slot
        n = new CInstance();
    } else if (type >= 14) {
        switch (type) {
        case 19: n = new CRicciBlend(); break;
        case 22: n = new CPcm(); break;
        case 24: n = new CWarpTwist(); break;
        case 25: n = new CWarpTaper(); break;
        case 26: n = new CWarpBend(); break;
        case 27: n = new CWarpShear(); break;
        default: n = new CBlobNode(); break;
        }
    } else {
        CSkeletonPrimitive* sp = new CSkeletonPrimitive();
        CSkeleton* s;
        switch (type) {
        case 0: s = new CSkeletonPoint(); break;
        case 1: s = new CSkeletonLine(); break;
        case 2: s = new CSkeletonCylinder(); break;
        case 3: s = new CSkeletonDisc(); break;
        case 4: s = new CSkeletonRing(); break;
        case 6: s = new CSkeletonCube(); break;
        case 7: s = new CSkeletonTriangle(); break;
        default: s = new CSkeleton(); break;
        }
        const float* q = v + 26;
        s->a = vec3f{q[0], q[1], q[2]};
        s->b = vec3f{q[3], q[4], q[5]};
        s->c = vec3f{q[6], q[7], q[8]};
        s->r = q[9];
        s->h = q[10];
        sp->skeleton = s;
        n = sp;
    }
    own.emplace_back(n);
    n->type = type;
    n->octree.lower = vec3f{v[0], v[1], v[2]};
    n->octree.upper = vec3f{v[3], v[4], v[5]};
    n->material.diffused = vec4f{v[6], v[7], v[8], v[38]};
    n->id = (int)v[39];
    n->transform.back.identity = v[9] != 0.0f;
    std::memcpy(n->transform.back.e, v + 10, 64);
    for (int k = 0; k < 4; ++k) n->res[k] = v[26 + k];
    for (int c = 0; c < nk; ++c) n->kids.push_back(read_node(in, own));
    return n;
}

// Instances name their origin by node id (OriginalNodeIndex, findNodeByID)
void resolve_instances(std::vector<std::unique_ptr<CBlobNode>>& own) {
    for (auto& n : own)
        if (n->type == 13)
            for (auto& m : own)
                if (m->id == (int)n->res[0]) {
                    static_cast<CInstance*>(n.get())->origin = m.get();
                    break;
                }
}

// The reference's MPUSTATS (PS_Polygonizer.h:201-207) over stand-ins with legacy TBB's
// representations (tbb_thread::id: a pthread_t; tick_count: one long long).
class ThreadIdLike {
    unsigned long my_id = 0;
};
class TickCountLike {
    long long my_count = 0;
};
struct MPUSTATS {
    int idxThread;
    int bIntersected;
    ThreadIdLike threadID;
    TickCountLike tickStart;
    TickCountLike tickEnd;
};

long long now_ns() {
    timespec ts;
    clock_gettime(CLOCK_REALTIME, &ts);
    return (long long)ts.tv_sec * 1000000000ll + ts.tv_nsec;
}

template <class T>
void put(std::ofstream& o, const T& x) { o.write(reinterpret_cast<const char*>(&x), sizeof(T)); }

}  // namespace

int main(int argc, char** argv) {
    if (argc < 4) return 64;
    const std::string mode = argv[1];
    if (mode == "tree" || mode == "run") {
        std::ifstream in(argv[2]);
        std::vector<std::unique_ptr<CBlobNode>> own;
        CBlobNode* root = read_node(in, own);
        if (!root) return 65;
        const bool translate = argc > 4 && mode == "tree" ? std::atoi(argv[4]) != 0 : true;
        const bool compat = argc > 5 && mode == "tree" ? std::atoi(argv[5]) != 0 : false;
        std::unique_ptr<SimdPoly> poly(new SimdPoly(0, translate, compat));
        const int code = poly->linearizeBlobTree(root);
        if (mode == "tree") {
            std::ofstream o(argv[3], std::ios::binary);
            put(o, code);
            put(o, poly->prims());
            put(o, poly->primMatrices());
            put(o, poly->ops());
            put(o, poly->boxMatrices());
            return 0;
        }
        if (code < 0) return 66;
        const float cs = (float)std::atof(argv[3]);
        std::fprintf(stderr, "linearized %d prims\n", (int)poly->prims().ctPrims);
        const int rc = poly->run(cs);
        std::fprintf(stderr, "ran %d\n", rc);
        std::printf("run rc %d V %u T %u\n", rc, poly->info().ctVertices, poly->info().ctTriangles);
        if (rc != PSGPU_RET_SUCCESS) return 67;
        std::ofstream o(argv[4], std::ios::binary);
        uint32_t drawn = 0;
        const int dr = poly->draw([&](const float* pos, const float* nrm, const float* col, uint32_t nv,
                                      const uint16_t* tris, uint32_t nt) {
            put(o, nv);
            put(o, nt);
            o.write(reinterpret_cast<const char*>(pos), (std::streamsize)nv * 12);
            o.write(reinterpret_cast<const char*>(nrm), (std::streamsize)nv * 12);
            o.write(reinterpret_cast<const char*>(col), (std::streamsize)nv * 12);
            o.write(reinterpret_cast<const char*>(tris), (std::streamsize)nt * 6);
            ++drawn;
        });
        std::fprintf(stderr, "drawn %u\n", drawn);
        o.close();
        poly.reset();
        std::fprintf(stderr, "destroyed\n");
        return dr == PSGPU_RET_SUCCESS ? 0 : 68;
    }
    if (mode == "gui-tree" || mode == "gui-run") {
        std::ifstream in(argv[2]);
        std::vector<std::unique_ptr<CBlobNode>> own;
        CBlobNode* root = read_node(in, own);
        if (!root) return 65;
        resolve_instances(own);
        if (mode == "gui-tree") {
            PS::COMPACTBLOBTREEGpu tree;
            const int code = tree.convert(root);
            std::ofstream o(argv[3], std::ios::binary);
            put(o, code);
            const uint32_t n[4] = {(uint32_t)tree.prims.size(), (uint32_t)tree.ops.size(), (uint32_t)tree.kids.size(),
                                   (uint32_t)tree.mtx.size()};
            o.write(reinterpret_cast<const char*>(n), sizeof n);
            o.write(reinterpret_cast<const char*>(tree.prims.data()), (std::streamsize)(n[0] * sizeof(PsGuiPrim)));
            o.write(reinterpret_cast<const char*>(tree.ops.data()), (std::streamsize)(n[1] * sizeof(PsGuiOp)));
            o.write(reinterpret_cast<const char*>(tree.kids.data()), (std::streamsize)(n[2] * 4));
            o.write(reinterpret_cast<const char*>(tree.mtx.data()), (std::streamsize)(n[3] * sizeof(PsGuiMatrix)));
            return 0;
        }
        if (argc < 5) return 64;
        PS::CParsipOptimizedGpu p(0);
        const int rs = p.setup(root, root->getOctree().lower, root->getOctree().upper, root->getID(),
                               (float)std::atof(argv[3]));
        const int rc = rs == PSGPU_RET_SUCCESS ? p.run() : rs;
        std::printf("gui rc %d MPUs %zu V %u T %u evals %zu\n", rc, p.countMPUs(), p.info().ctVertices,
                    p.info().ctTriangles, p.statsTotalFieldEvals());
        if (rc != PSGPU_RET_SUCCESS) return 67;
        std::vector<float> pos, nrm, col;
        std::vector<uint32_t> tris;
        const int re = p.exportMesh(pos, nrm, col, tris);
        size_t drawnT = 0;
        p.drawMesh([&](const float*, const float*, const float*, uint32_t, const uint32_t*, uint32_t nt) { drawnT += nt; });
        if (drawnT != tris.size() / 3) return 69;
        std::ofstream o(argv[4], std::ios::binary);
        const uint32_t vt[2] = {(uint32_t)(pos.size() / 3), (uint32_t)(tris.size() / 3)};
        o.write(reinterpret_cast<const char*>(vt), sizeof vt);
        o.write(reinterpret_cast<const char*>(pos.data()), (std::streamsize)(pos.size() * 4));
        o.write(reinterpret_cast<const char*>(nrm.data()), (std::streamsize)(nrm.size() * 4));
        o.write(reinterpret_cast<const char*>(col.data()), (std::streamsize)(col.size() * 4));
        o.write(reinterpret_cast<const char*>(tris.data()), (std::streamsize)(tris.size() * 4));
        return re == PSGPU_RET_SUCCESS ? 0 : 68;
    }
    if ((mode == "soa" || mode == "soa-stats" || mode == "soa-threads" || mode == "soa-mt") && argc >= 5) {
        static PS::SIMDPOLY::SOABlobPrims prims;
        static PS::SIMDPOLY::SOABlobPrimMatrices mats;
        static PS::SIMDPOLY::SOABlobOps ops;
        static PS::SIMDPOLY::SOABlobBoxMatrices boxes;
        std::ifstream in(argv[2], std::ios::binary);
        in.read(reinterpret_cast<char*>(&prims), sizeof prims);
        in.read(reinterpret_cast<char*>(&mats), sizeof mats);
        in.read(reinterpret_cast<char*>(&ops), sizeof ops);
        in.read(reinterpret_cast<char*>(&boxes), sizeof boxes);
        if (!in) return 65;
        std::unique_ptr<PS::SIMDPOLY::PolyMPUs> poly(new PS::SIMDPOLY::PolyMPUs());
        poly->ctMPUs = 12345;  // must be overwritten (0 on failure)
        const float cs = (float)std::atof(argv[3]);
        if (mode == "soa-stats") {
            std::vector<MPUSTATS> stats(PSGPU_MAX_MPU_COUNT);
            for (size_t i = 0; i < stats.size(); ++i) {  // fields the reference leaves alone
                stats[i].idxThread = -7;
                stats[i].bIntersected = (int)i;
            }
            const long long t0 = now_ns();
            const int rc = PS::SIMDPOLY::Polygonize(cs, prims, mats, ops, *poly, stats.data());
            const long long t1 = now_ns();
            std::printf("Polygonize rc %d ctMPUs %u\n", rc, poly->ctMPUs);
            std::ofstream o(argv[4], std::ios::binary);
            put(o, rc);
            put(o, poly->ctMPUs);
            put(o, t0);
            put(o, t1);
            o.write(reinterpret_cast<const char*>(stats.data()), (std::streamsize)poly->ctMPUs * sizeof(MPUSTATS));
            return 0;
        }
        if (mode == "soa-threads") {  // Polygonize twice, then PrintThreadResults(2, ...) twice
            const int rc1 = PS::SIMDPOLY::Polygonize(cs, prims, mats, ops, *poly, NULL);
            const int rc2 = PS::SIMDPOLY::Polygonize(cs, prims, mats, ops, *poly);
            const int n = psgpu_thread_result_count();
            std::vector<uint32_t> pr(n > 0 ? n : 1, 0xdeadbeefu), cr(n > 0 ? n : 1, 0xdeadbeefu);
            PS::SIMDPOLY::PrintThreadResults(2, pr.data(), cr.data());
            const int after = psgpu_thread_result_count();
            std::vector<uint32_t> pr2(4, 0xdeadbeefu);
            PS::SIMDPOLY::PrintThreadResults(2, pr2.data());  // nothing accumulated since: no entry
            std::ofstream o(argv[4], std::ios::binary);
            put(o, rc1);
            put(o, rc2);
            put(o, n);
            put(o, after);
            o.write(reinterpret_cast<const char*>(pr.data()), (std::streamsize)n * 4);
            o.write(reinterpret_cast<const char*>(cr.data()), (std::streamsize)n * 4);
            o.write(reinterpret_cast<const char*>(pr2.data()), 16);
            o.write(reinterpret_cast<const char*>(poly->vMPUs), (std::streamsize)poly->ctMPUs * sizeof(PsMPU));
            return 0;
        }
        if (mode == "soa-mt") {  // kThreads host threads, kCalls Polygonize each into its own PolyMPUs
            constexpr int kThreads = 4, kCalls = 3;
            std::vector<std::unique_ptr<PS::SIMDPOLY::PolyMPUs>> outs;
            outs.push_back(std::move(poly));
            for (int t = 1; t < kThreads; ++t) outs.emplace_back(new PS::SIMDPOLY::PolyMPUs());
            std::vector<int> rcs(kThreads * kCalls, -100);
            std::vector<uint32_t> cts(kThreads * kCalls, 0u);
            std::vector<uint64_t> sums(kThreads * kCalls, 0ull);
            std::vector<std::thread> ts;
            for (int t = 0; t < kThreads; ++t) {
                ts.emplace_back([&, t] {
                    for (int k = 0; k < kCalls; ++k) {
                        const int i = t * kCalls + k;
                        rcs[i] = PS::SIMDPOLY::Polygonize(cs, prims, mats, ops, *outs[t]);
                        cts[i] = outs[t]->ctMPUs;
                        // FNV-1a over the filled records' words (the rest of each record is the
                        // zero of the value-initialised PolyMPUs in every thread)
                        const uint64_t* w = reinterpret_cast<const uint64_t*>(outs[t]->vMPUs);
                        uint64_t h = 1469598103934665603ull;
                        for (size_t j = 0, n = (size_t)cts[i] * sizeof(PsMPU) / 8; j < n; ++j)
                            h = (h ^ w[j]) * 1099511628211ull;
                        sums[i] = h;
                    }
                });
            }
            for (std::thread& t : ts) t.join();
            const int n = psgpu_thread_result_count();
            std::vector<uint32_t> pr(n > 0 ? n : 1, 0xdeadbeefu), cr(n > 0 ? n : 1, 0xdeadbeefu);
            PS::SIMDPOLY::PrintThreadResults(kCalls, pr.data(), cr.data());
            std::ofstream o(argv[4], std::ios::binary);
            put(o, kThreads * kCalls);
            o.write(reinterpret_cast<const char*>(rcs.data()), (std::streamsize)rcs.size() * 4);
            o.write(reinterpret_cast<const char*>(cts.data()), (std::streamsize)cts.size() * 4);
            o.write(reinterpret_cast<const char*>(sums.data()), (std::streamsize)sums.size() * 8);
            put(o, n);
            o.write(reinterpret_cast<const char*>(pr.data()), (std::streamsize)n * 4);
            o.write(reinterpret_cast<const char*>(cr.data()), (std::streamsize)n * 4);
            o.write(reinterpret_cast<const char*>(outs[0]->vMPUs), (std::streamsize)outs[0]->ctMPUs * sizeof(PsMPU));
            return 0;
        }
        const int rc = PS::SIMDPOLY::Polygonize(cs, prims, mats, ops, *poly, NULL);  // the reference's default
        std::printf("Polygonize rc %d ctMPUs %u\n", rc, poly->ctMPUs);
        std::ofstream o(argv[4], std::ios::binary);
        put(o, rc);
        put(o, poly->ctMPUs);
        o.write(reinterpret_cast<const char*>(poly->vMPUs), (std::streamsize)poly->ctMPUs * sizeof(PsMPU));
        return 0;
    }
    return 64;
}

// psgpu_host.cpp — C-ABI of the MI355X polygonizer (include/parsip_gpu.h).
//
// Host side of PS::SIMDPOLY::Polygonize (PS_Polygonizer.cpp:315-385): MPU lattice,
// model upload (the reference's per-thread FieldComputer copy, :22-50, becomes one
// 28 KB device image read through the scalar cache), kernel sequencing on one HIP
// stream, and the exports back to the reference PolyMPUs layout.
#include <hip/hip_runtime.h>

#include <atomic>
#include <algorithm>
#include <numeric>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <functional>
#include <limits>
#include <memory>
#include <chrono>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/parsip_gpu.h"
#include "psgpu_internal.h"
#include "psgpu_launch.h"


using namespace psgpu;

namespace {

// ---------------------------------------------------------------------------
// Marching-cubes table.  Generated, not transcribed: Bloomenthal's cube-table
// construction ("An Implicit Surface Polygonizer", Graphics Gems IV, 1994) walks
// each sign-changing edge clockwise around the cube faces to build polygons; the
// reference's g_triTableCache (_CellConfigTable.h:60-317) keeps polygons in
// discovery order with each polygon's edges in reverse walk order and fans
// triangles about the last edge.  Corner c: bit2 = x, bit1 = y, bit0 = z.
struct CubeTables {
    int8_t tri[256][16];
    uint8_t ntri[256];
    uint8_t corner1[12], corner2[12], axis[12];
};

const CubeTables& cube_tables() {
    static CubeTables T;
    static std::once_flag once;
    std::call_once(once, [] {
        // edges LB LT LN LF RB RT RN RF BN BF TN TF; faces L R B T N F
        static const uint8_t c1[12] = {0, 2, 0, 1, 4, 6, 4, 5, 0, 1, 2, 3};
        static const uint8_t c2[12] = {1, 3, 2, 3, 5, 7, 6, 7, 4, 5, 6, 7};
        static const uint8_t ax[12] = {2, 2, 1, 1, 2, 2, 1, 1, 0, 0, 0, 0};
        static const uint8_t lface[12] = {2, 0, 0, 5, 1, 3, 4, 1, 4, 2, 3, 5};
        static const uint8_t rface[12] = {0, 3, 4, 0, 2, 1, 1, 5, 2, 5, 4, 3};
        // next clockwise edge around `face` after `edge`: {face of the edge's first
        // listed face, next-if-that-face, next-otherwise}
        static const uint8_t ccwFace[12] = {0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 3, 3};
        static const uint8_t nextOn[12] = {3, 2, 0, 1, 6, 7, 5, 4, 4, 0, 1, 5};
        static const uint8_t nextOff[12] = {8, 11, 10, 9, 9, 10, 8, 11, 2, 7, 6, 3};
        memcpy(T.corner1, c1, 12);
        memcpy(T.corner2, c2, 12);
        memcpy(T.axis, ax, 12);
        for (int cfg = 0; cfg < 256; ++cfg) {
            auto in = [cfg](int c) { return (cfg >> c) & 1; };
            bool done[12] = {};
            std::vector<int> rows;
            for (int e = 0; e < 12; ++e) {
                if (done[e] || in(c1[e]) == in(c2[e])) continue;
                std::vector<int> poly;
                int edge = e, face = in(c1[e]) ? rface[e] : lface[e];
                for (;;) {
                    edge = (face == ccwFace[edge]) ? nextOn[edge] : nextOff[edge];
                    done[edge] = true;
                    if (in(c1[edge]) != in(c2[edge])) {
                        poly.insert(poly.begin(), edge);
                        if (edge == e) break;
                        face = (face == lface[edge]) ? rface[edge] : lface[edge];
                    }
                }
                const int np = (int)poly.size();
                for (int t = np - 3; t >= 0; --t) {
                    rows.push_back(poly[t]);
                    rows.push_back(poly[t + 1]);
                    rows.push_back(poly[np - 1]);
                }
            }
            for (int i = 0; i < 16; ++i) T.tri[cfg][i] = i < (int)rows.size() ? (int8_t)rows[i] : (int8_t)-1;
            T.ntri[cfg] = (uint8_t)(rows.size() / 3);
        }
    });
    return T;
}

// Packed device tables (psgpu_model.h CubeTablesDev).
void fill_device_tables(const CubeTables& T, CubeTablesDev& D) {
    memset(&D, 0, sizeof(D));
    for (int c = 0; c < 256; ++c) {
        uint64_t row = 0, order = 0;
        uint32_t seen = 0;
        int nd = 0;
        for (int e = 0; e < 16 && T.tri[c][e] >= 0; ++e) {
            const int ed = T.tri[c][e];
            row |= (uint64_t)ed << (4 * e);
            if (!((seen >> ed) & 1u)) {
                seen |= 1u << ed;
                order |= (uint64_t)ed << (4 * nd++);
            }
        }
        uint32_t cross = 0;
        for (int e = 0; e < 12; ++e)
            if (((c >> T.corner1[e]) & 1) != ((c >> T.corner2[e]) & 1)) cross |= 1u << e;
        D.row[c] = row;
        D.order[c] = order;
        D.cross[c] = (uint16_t)cross;
        D.ntri[c] = T.ntri[c];
        D.crossNtri[c] = cross | ((uint32_t)T.ntri[c] << 16);
    }
    // ownership: the first cell in (i,j,k) order containing an edge owns it; an edge
    // starting at cell corner (cx,cy,cz) on axis a is owned by this cell iff every
    // non-axis corner bit is 1 or the cell sits on that axis' low boundary
    for (int b = 0; b < 8; ++b) {
        const bool i0 = b & 4, j0 = b & 2, k0 = b & 1;
        uint32_t m = 0;
        for (int e = 0; e < 12; ++e) {
            const int c1 = T.corner1[e], ax = T.axis[e];
            const bool bx = (c1 >> 2) & 1, by = (c1 >> 1) & 1, bz = c1 & 1;
            const bool okx = ax == 0 || bx || i0, oky = ax == 1 || by || j0, okz = ax == 2 || bz || k0;
            if (okx && oky && okz) m |= 1u << e;
        }
        D.own[b] = (uint16_t)m;
    }
    uint64_t edge = 0;
    for (int e = 0; e < 12; ++e) edge |= (uint64_t)(T.corner1[e] | (T.axis[e] << 3)) << (5 * e);
    D.edge = edge;
}

// ---------------------------------------------------------------------------
// Walk program: the reference's processing order of fieldValue's explicit stack.
bool op_needs_left(int t) { return (t >= 14 && t <= 19) || (t >= 22 && t <= 25); }
bool op_needs_right(int t) { return t >= 14 && t <= 19; }

struct ProgramBuilder {
    const PsSoaBlobOps& O;
    std::vector<Instr> prog;
    std::vector<uint8_t> seen;
    int maxSlot = 0;
    bool ok = true;

    explicit ProgramBuilder(const PsSoaBlobOps& ops) : O(ops), seen(128, 0) {}

    void emit(int op, int depth, int h) {
        if (!ok) return;
        if (op < 0 || op >= (int)O.ctOps || seen[op] || depth > 127 || h + 3 >= kMaxSlots) {
            ok = false;
            return;
        }
        seen[op] = 1;
        const int kind = O.opChildKind[op];
        const int L = O.opLeftChild[op], R = O.opRightChild[op];
        const int type = O.opType[op];
        size_t enterAt = 0;
        if (depth > 3) {
            Instr e{};
            e.kind = kEnter;
            e.idx = (uint16_t)op;
            e.out = (uint8_t)h;
            enterAt = prog.size();
            prog.push_back(e);
        }
        int next = h, lslot = 0, rslot = 0;
        if (kind & 1) {  // right op subtree first (pushed last, popped first)
            emit(R, depth + 1, h);
            rslot = h;
            next = h + 1;
        }
        if (kind & 2) {
            emit(L, depth + 1, next);
            lslot = next;
            next = next + 1;
        }
        if (!ok) return;
        int freeSlot = next;
        if (!(kind & 2) && op_needs_left(type)) {
            if (L >= 128) { ok = false; return; }
            Instr p{};
            p.kind = kPrim;
            p.idx = (uint16_t)L;
            p.out = (uint8_t)freeSlot;
            prog.push_back(p);
            lslot = freeSlot++;
        }
        if (!(kind & 1) && op_needs_right(type)) {
            if (R >= 128) { ok = false; return; }
            Instr p{};
            p.kind = kPrim;
            p.idx = (uint16_t)R;
            p.out = (uint8_t)freeSlot;
            prog.push_back(p);
            rslot = freeSlot++;
        }
        maxSlot = std::max(maxSlot, freeSlot);
        Instr c{};
        c.kind = kOp;
        c.type = (uint8_t)type;
        c.out = (uint8_t)h;
        c.lslot = (uint8_t)lslot;
        c.rslot = (uint8_t)rslot;
        c.childKind = (uint8_t)kind;
        c.L = (uint8_t)L;
        c.R = (uint8_t)R;
        c.idx = (uint16_t)op;
        prog.push_back(c);
        if (depth > 3) prog[enterAt].skipTo = (uint16_t)prog.size();
        if (prog.size() > (size_t)kMaxInstr) ok = false;
    }
};

bool finite3(const float* v) { return std::isfinite(v[0]) && std::isfinite(v[1]) && std::isfinite(v[2]); }

int build_device_model(const PsSoaBlobPrims& P, const PsSoaPrimMatrices& Mx, const PsSoaBlobOps& O, DevModel& D) {
    memset(&D, 0, sizeof(D));
    if (P.ctPrims == 0 || P.ctPrims > 128 || O.ctOps > 128) return PSGPU_RET_PARAM_ERROR;
    D.ctPrims = P.ctPrims;
    D.ctOps = O.ctOps;
    if (O.ctOps == 0) {
        for (uint32_t i = 0; i < P.ctPrims; ++i) {
            Instr s{};
            s.kind = kSumPrim;
            s.idx = (uint16_t)i;
            D.instr[i] = s;
        }
        D.nInstr = P.ctPrims;
        D.nSlots = 1;
    } else {
        ProgramBuilder b(O);
        b.emit(0, 0, 0);
        if (!b.ok) return PSGPU_RET_INVALID_BVH;
        D.nInstr = (uint32_t)b.prog.size();
        std::copy(b.prog.begin(), b.prog.end(), D.instr);
        D.nSlots = (uint32_t)std::max(1, b.maxSlot);
    }
    for (uint32_t i = 0; i < 128; ++i) {
        DevOp& d = D.ops[i];
        d.lo[0] = O.vBoxLoX[i]; d.lo[1] = O.vBoxLoY[i]; d.lo[2] = O.vBoxLoZ[i];
        d.hi[0] = O.vBoxHiX[i]; d.hi[1] = O.vBoxHiY[i]; d.hi[2] = O.vBoxHiZ[i];
        d.resY = O.resY[i];
        d.type = O.opType[i];
    }
    // Colour of each op whose subtree is all +0 fields (culled primitives, or pruned: the
    // reference's colour pass then reads zeroed arrays, :1472-1522): a constant of the tree
    // and the primitive colours, computed in fp32 exactly as op_colour_weights + the
    // weighted sum on the device.  Children first (post-order over the tree the program
    // builder validated: every child op id < ctOps, every prim id < 128, no cycles), so any
    // op numbering works, not only pre-order; unreachable ops keep zero.
    const float* pc[3] = {P.colorX, P.colorY, P.colorZ};
    std::function<void(int)> zero_col = [&](int op) {
        const uint32_t t = O.opType[op], kind = O.opChildKind[op];
        const uint32_t L = O.opLeftChild[op], R = O.opRightChild[op];
        if (kind & 2) zero_col((int)L);
        if (kind & 1) zero_col((int)R);
        float cl[3], cr[3];
        for (int k = 0; k < 3; ++k) {
            cl[k] = (kind & 2) ? D.zeroCol[L][k] : pc[k][L];
            cr[k] = (kind & 1) ? D.zeroCol[R][k] : pc[k][R];
        }
        const float lf = 0.0f, rf = 0.0f;
        float v = 0.0f, wl = 0.0f, wr = 0.0f;
        bool weighted = true;
        switch (t) {
        case PSGPU_OP_BLEND: v = lf + rf; wl = 2.0f * (0.5f + lf) - 1.0f; wr = 2.0f * (0.5f + rf) - 1.0f; break;
        case PSGPU_OP_UNION: v = lf > rf ? lf : rf; wl = (v - lf) == 0.0f ? 1.0f : 0.0f; wr = (v - rf) == 0.0f ? 1.0f : 0.0f; break;
        case PSGPU_OP_INTERSECT: v = lf < rf ? lf : rf; wl = (v - lf) == 0.0f ? 1.0f : 0.0f; wr = (v - rf) == 0.0f ? 1.0f : 0.0f; break;
        case PSGPU_OP_DIF: { const float q = 1.0f - rf; v = lf < q ? lf : q; wl = lf == v ? 1.0f : 0.0f; wr = (1.0f - rf) == v ? 1.0f : 0.0f; } break;
        case PSGPU_OP_SMOOTHDIF: v = lf * (1.0f - rf); wl = lf == v ? 1.0f : 0.0f; wr = (1.0f - rf) == v ? 1.0f : 0.0f; break;
        default: weighted = false; break;
        }
        for (int k = 0; k < 3; ++k) {
            if (weighted) D.zeroCol[op][k] = wl * cl[k] + wr * cr[k];
            else if (t >= PSGPU_OP_WARPTWIST && t <= PSGPU_OP_WARPSHEAR) D.zeroCol[op][k] = cl[k];
            else D.zeroCol[op][k] = 0.0f;  // not used: zero subtrees contain only the types above
        }
    };
    if (O.ctOps > 0) zero_col(0);
    // every one of the 128 prim slots is uploaded: the reference evaluates whatever
    // index an op names, even past ctPrims (SOABlobPrims keeps all 128 entries)
    for (uint32_t i = 0; i < 128; ++i) {
        DevPrim& d = D.prims[i];
        d.pos[0] = P.posX[i]; d.pos[1] = P.posY[i]; d.pos[2] = P.posZ[i];
        d.dir[0] = P.dirX[i]; d.dir[1] = P.dirY[i]; d.dir[2] = P.dirZ[i];
        d.res[0] = P.resX[i]; d.res[1] = P.resY[i]; d.res[2] = P.resZ[i];
        d.col[0] = P.colorX[i]; d.col[1] = P.colorY[i]; d.col[2] = P.colorZ[i];
        d.type = P.skeletType[i];
        const uint32_t im = P.idxMatrix[i];
        d.hasMatrix = im != 0;
        if (im != 0) {
            if (im >= 128) return PSGPU_RET_PARAM_ERROR;
            memcpy(d.mat, &Mx.matrix[im * PSGPU_PRIM_MATRIX_STRIDE], 12 * sizeof(float));
        }
        // exact-culling eligibility (see make_cull_mask in psgpu_kernels.hip)
        bool c = !d.hasMatrix && finite3(d.pos);
        switch (d.type) {
        case PSGPU_PRIM_POINT: break;
        case PSGPU_PRIM_LINE: {
            const double ux = (double)d.dir[0] - d.pos[0], uy = (double)d.dir[1] - d.pos[1],
                         uz = (double)d.dir[2] - d.pos[2];
            c = c && finite3(d.dir) && (ux * ux + uy * uy + uz * uz) > 1e-6;
        } break;
        case PSGPU_PRIM_CUBE: c = c && std::isfinite(d.res[0]) && d.res[0] >= 0.0f; break;
        case PSGPU_PRIM_CYLINDER: {
            const double n2 = (double)d.dir[0] * d.dir[0] + (double)d.dir[1] * d.dir[1] + (double)d.dir[2] * d.dir[2];
            c = c && finite3(d.dir) && std::fabs(n2 - 1.0) < 1e-4 && d.res[0] >= 0.0f && d.res[1] >= 0.0f &&
                std::isfinite(d.res[0]) && std::isfinite(d.res[1]);
        } break;
        default: c = false; break;
        }
        // culling skeleton (CullSeg, psgpu_model.h): a lower bound of the distance
        CullSeg& cs = D.cull[i];
        memset(&cs, 0, sizeof(cs));
        const float inf = std::numeric_limits<float>::infinity();
        cs.radius = inf;  // never culled unless eligible below
        cs.tmin = 0.0f;
        cs.tmax = 1.0f;
        cs.axisClear = -inf;
        uint32_t flags = c ? 1u : 0u;
        if (c) {
            for (int a = 0; a < 3; ++a) cs.a[a] = d.pos[a];
            cs.radius = 0.0f;
            double uu = 0.0;
            if (d.type == PSGPU_PRIM_LINE) {
                for (int a = 0; a < 3; ++a) cs.u[a] = d.dir[a] - d.pos[a];
                cs.tmin = -inf;
                cs.tmax = inf;
                flags |= 2u;
            } else if (d.type == PSGPU_PRIM_CYLINDER) {
                for (int a = 0; a < 3; ++a) cs.u[a] = d.res[1] * d.dir[a];  // axis segment, length h
                cs.radius = d.res[0];
                cs.axisClear = 0.05f;
                flags |= 4u;
            } else if (d.type == PSGPU_PRIM_CUBE) {
                cs.radius = (float)(d.res[0] * 1.7320508075688772 * (1.0 + 1e-6));
            }
            for (int a = 0; a < 3; ++a) uu += (double)cs.u[a] * cs.u[a];
            cs.invUU = uu > 0.0 ? (float)(1.0 / uu) : 0.0f;
            if (d.type == PSGPU_PRIM_CYLINDER && uu == 0.0) {  // h = 0: no axis direction
                flags &= ~1u;
                cs.radius = inf;
            }
        } else if (d.type == PSGPU_PRIM_TRIANGLE) {
            cs.radius = -inf;  // field exactly 0 everywhere (dist2 = FLT_MAX)
        }
        if (i >= P.ctPrims) cs.radius = inf;  // (the culling masks only cover ctPrims)
        d.cullable = flags;
    }
    // field bounds (k_precheck, prim_bound in psgpu_device.h) need every primitive the
    // walk evaluates to have a true-distance bound with sane parameters (the culling
    // eligibility above) or be a Triangle (field 0), and every op a monotone map
    bool bnd = D.nInstr > 0;
    for (uint32_t k = 0; k < D.nInstr; ++k) {
        const Instr& I = D.instr[k];
        if (I.kind == kOp && !((I.type >= 14 && I.type <= 18) || (I.type >= 22 && I.type <= 25))) bnd = false;
        if (I.kind == kPrim || I.kind == kSumPrim) {
            const DevPrim& q = D.prims[I.idx];
            if (!(q.type == PSGPU_PRIM_TRIANGLE || (q.cullable & 1u))) bnd = false;
        }
    }
    D.boundable = bnd ? 1u : 0u;
    return PSGPU_RET_SUCCESS;
}

void lattice_dims(float cs, const PsVec3f& lo, const PsVec3f& hi, uint32_t d[3]) {
    const float ext[3] = {hi.x - lo.x, hi.y - lo.y, hi.z - lo.z};
    for (int a = 0; a < 3; ++a) {
        const float q = ext[a] / cs;
        const int cells = (int)std::ceil(q);
        int n = cells / PSGPU_CELLS_PER_MPU;
        if (cells % PSGPU_CELLS_PER_MPU != 0) ++n;
        d[a] = n > 0 ? (uint32_t)n : 0u;
    }
}

template <typename T>
hipError_t grow(T*& ptr, size_t& cap, size_t need) {
    if (need <= cap && ptr) return hipSuccess;
    if (ptr) (void)hipFree(ptr);
    ptr = nullptr;
    size_t n = std::max<size_t>(need, cap + cap / 2);
    hipError_t e = hipMalloc(&ptr, std::max<size_t>(n, 1) * sizeof(T));
    cap = e == hipSuccess ? n : 0;
    return e;
}

const char* kKernelNames[kNumKernels] = {"k_precheck", "k_mpu", "k_vertex", "k_finish"};

}  // namespace

namespace psgpu {
int hip_fail(hipError_t e, const char* what) {
    if (e == hipSuccess) return PSGPU_RET_SUCCESS;
    fprintf(stderr, "psgpu: %s failed: %s\n", what, hipGetErrorString(e));
    return e == hipErrorOutOfMemory ? PSGPU_RET_NOT_ENOUGH_MEM : PSGPU_RET_DEVICE_ERROR;
}

int set_device(psgpu_ctx* c) { return hip_fail(hipSetDevice(c->device), "hipSetDevice"); }
}  // namespace psgpu

namespace {

// k_precheck covers the MPU range with 2x2x2 bricks of MPUs (one per wavefront: a
// compact box for its culling test), whole brick rows along x.
void brick_layout(const psgpu_ctx* c, uint32_t* i0, uint32_t bd[3]) {
    const uint32_t nyz = c->dims[1] * c->dims[2];
    const uint32_t first = nyz ? c->mpuBegin / nyz : 0;
    const uint32_t last = (nyz && c->mpuCount) ? (c->mpuBegin + c->mpuCount - 1) / nyz : first;
    *i0 = first / 2;
    bd[0] = c->mpuCount ? last / 2 - first / 2 + 1 : 0;
    bd[1] = (c->dims[1] + 1) / 2;
    bd[2] = (c->dims[2] + 1) / 2;
}
// The brick permutation of k_precheck: stride 1 keeps the lattice order; otherwise a
// stride near n / golden ratio, coprime with n, so consecutive wave slots (one block, one
// CU) take bricks far apart and the bricks crossed by the surface spread over the chip.
uint32_t brick_stride(uint32_t n, bool spread) {
    if (!spread || n < 3) return 1u;
    for (uint32_t s = (uint32_t)(n * 0.6180339887) | 1u; s > 1; --s)
        if (std::gcd(s, n) == 1u) return s;
    return 1u;
}
size_t brick_count(const psgpu_ctx* c) {
    uint32_t i0, bd[3];
    brick_layout(c, &i0, bd);
    return (size_t)bd[0] * bd[1] * bd[2];
}

// The S2-by-octants experiment (PSGPU_S2_OCT, off by default, measured slower: DESIGN.md §4)
// is compiled in only through PSGPU_JIT_FLAGS; its per-entry proof words exist only then.
bool s2_oct_enabled() {
    static const bool on = [] {
        const char* f = getenv("PSGPU_JIT_FLAGS");
        const char* d = f ? strstr(f, "PSGPU_S2_OCT=") : nullptr;
        return d != nullptr && d[13] != '\0' && d[13] != '0';
    }();
    return on;
}

// k_front sub-queue capacity for a k_precheck grid of `blocks` blocks of `mpb` bricks: every
// 8th block's bricks x 8 MPUs; front_cap(bricks) bounds it for both grids (2 and 4 bricks per block)
uint32_t front_sub_cap(uint32_t blocks, uint32_t mpb) { return 8u * mpb * ((blocks + 7u) / 8u); }
uint32_t front_cap(size_t bricks) {
    const uint32_t b = (uint32_t)bricks;
    return std::max(front_sub_cap((b + 1u) / 2u, 2u), front_sub_cap((b + 3u) / 4u, 4u));
}

int ensure_buffers(psgpu_ctx* c, uint32_t mpuCount) {
    const size_t n = std::max<uint32_t>(mpuCount, 1);
    c->pShardCap = 8u * (uint32_t)((brick_count(c) + kShards - 1) / kShards);
    // k_front's 8 sub-queues: a block's bricks x 8 MPUs for every 8th k_precheck block
    const size_t fq = 8 * front_cap(brick_count(c));
    const size_t nq = std::max<size_t>((size_t)c->pShardCap * kShards, fq);
    PSGPU_CHECK(grow(c->pq, c->capList, nq));
    PSGPU_CHECK(grow(c->pqMask, c->capPqMask, nq * 2));
    if (fq > c->capFq) {  // ready words start at 0: no run's tag
        PSGPU_CHECK(grow(c->fqReady, c->capFq, fq));
        PSGPU_CHECK(hipMemset(c->fqReady, 0, c->capFq * sizeof(uint32_t)));
    }
    if (s2_oct_enabled()) PSGPU_CHECK(grow(c->pqOct, c->capPqOct, (size_t)c->pShardCap * kShards));
    PSGPU_CHECK(grow(c->counts, c->capCounts, n));
    PSGPU_CHECK(grow(c->passed, c->capPassed, n));
    PSGPU_CHECK(grow(c->mpuMasks, c->capMasks, 2 * n));
    PSGPU_CHECK(grow(c->offs, c->capOff, n + 1));
    PSGPU_CHECK(grow(c->vk, c->capVk, (size_t)c->vShardCap * kShards));
    PSGPU_CHECK(grow(c->vp, c->capVp, (size_t)c->vShardCap * kShards));
    PSGPU_CHECK(grow(c->tq, c->capTq, (size_t)c->tShardCap * kShards));
    size_t capV2 = c->capV, capV3 = c->capV;
    PSGPU_CHECK(grow(c->pos, c->capV, (size_t)c->vcap * 3));
    PSGPU_CHECK(grow(c->nrm, capV2, (size_t)c->vcap * 3));
    PSGPU_CHECK(grow(c->col, capV3, (size_t)c->vcap * 3));
    PSGPU_CHECK(grow(c->tris, c->capT, (size_t)c->tcap * 3));
    if (c->mpuTicksOpt) PSGPU_CHECK(grow(c->mpuTicks, c->capTicks, 4 * n));
    return PSGPU_RET_SUCCESS;
}

// k_precheck / k_mpu with the walk split at the root (two waves per brick / MPU)
// (2: when the last finished run of this range queued at most splitMaxQueued MPUs for S2 --
// a launch too small to fill the device, whose span is its heaviest items' walks)
bool use_split(const psgpu_ctx* c) {
    if (!c->jit || !c->jit->precheckS || !c->splittable) return false;
    return c->treeSplit == 1 || (c->treeSplit == 2 && c->haveQueued && c->lastQueued <= c->splitMaxQueued);
}

// k_precheck + k_mpu as one launch (k_front) for the next run: 1 forces it, 2 (default) when
// the k_precheck grid is at most 8 blocks per CU -- C3 and its rank shares, whose step the
// boundary and the S1 tail weigh on (the driver's C3 window -7 %, one engine -2.4 %), not C5's
// 512^3 frame (13 k S1 blocks: +4.6 %, the fused kernel's registers cost its S1 waves a slot;
// profiles/r06_front_ab.txt).  Never with per-MPU ticks (MPUSTATS: S1 and S2 would write an
// MPU's tick words from two XCDs in one launch), on a crowded device, or while finish re-runs a
// run whose in-kernel wait gave up (surfaceOff).
bool use_front(const psgpu_ctx* c) {
    if (!c->jit || c->front == 0 || c->surfaceOff || c->crowded || c->mpuTicksOpt) return false;
    const bool split = use_split(c);
    if (!(split ? c->jit->frontS : c->jit->front)) return false;
    if (c->front == 1) return true;
    const size_t mpb = split ? 2u : (size_t)kMpusPerBlock;
    return (brick_count(c) + mpb - 1) / mpb <= 8u * (size_t)c->numCUs;
}

Params make_params(psgpu_ctx* c) {
    Params p;
    memset(&p, 0, sizeof(p));  // padding too: graph replay compares parameter bytes
    p.model = c->dModel;
    p.tables = c->dTables;
    p.cs = c->cs;
    p.side = c->cs * (float)PSGPU_CELLS_PER_MPU;
    p.lo[0] = c->primsHost.bboxLo.x;
    p.lo[1] = c->primsHost.bboxLo.y;
    p.lo[2] = c->primsHost.bboxLo.z;
    for (int a = 0; a < 3; ++a) p.dims[a] = c->dims[a];
    p.divMagic[0] = p.dims[2] ? 0xffffffffu / p.dims[2] : 0u;
    p.divMagic[1] = (p.dims[2] * p.dims[1]) ? 0xffffffffu / (p.dims[2] * p.dims[1]) : 0u;
    p.mpuBegin = c->mpuBegin;
    p.mpuCount = c->mpuCount;
    p.cull = (uint32_t)c->cull;
    brick_layout(c, &p.brickI0, p.brickDims);
    const bool split = use_split(c);
    const uint32_t mpb = split ? 2u : (uint32_t)kMpusPerBlock;  // MPUs (bricks) per block
    p.preBlocks = (uint32_t)((brick_count(c) + mpb - 1) / mpb);
    p.brickStride = brick_stride((uint32_t)brick_count(c), (c->debug & 16384) != 0);
    p.pq = c->pq;
    p.pqMask = c->pqMask;
    p.pqOct = c->pqOct;
    p.pShardCap = c->pShardCap;
    // k_mpu: one wave per queued survivor, as many as the last finished run queued + 1/4
    // (a run that queues more is re-run by finish(): the grid then fits exactly)
    const uint32_t maxBlocks = (c->mpuCount + mpb - 1) / mpb;
    const uint32_t margin = c->lastQueued / c->mpuMarginDiv + (c->mpuMarginDiv > 4 ? 64u : 256u);
    const uint32_t want = c->haveQueued ? (c->lastQueued + margin + mpb - 1) / mpb : maxBlocks;
    p.mpuBlocks = std::max(1u, std::min(maxBlocks, want));
    p.fqReady = c->fqReady;
    p.fqCap = front_sub_cap(p.preBlocks, mpb);
    if (use_front(c)) {
        // k_front's S2 blocks: 8 per row, a row takes mpb entries of each sub-queue; rows for the
        // last run's largest sub-queue + 1/4 (or every entry of a sub-queue without a last run)
        const uint32_t sub = !c->haveQueued ? p.fqCap
                             : (c->lastSubMax ? c->lastSubMax : (c->lastQueued + 7u) / 8u) + c->lastQueued / 32u + 32u;
        const uint32_t rows = (std::min(sub, p.fqCap) + mpb - 1u) / mpb;
        p.mpuBlocks = 8u * std::max(1u, rows);
    }
    if (c->debug & (1 << 20)) p.mpuBlocks = use_front(c) ? 8u : 1u;  // test hook: a k_mpu grid that falls short (finish re-runs)
    p.scanChunks = (c->mpuCount + kScanItems * kScanMaxBlocks - 1) / (kScanItems * kScanMaxBlocks);
    if (p.scanChunks == 0) p.scanChunks = 1;
    p.scanBlocks = (c->mpuCount + kScanItems * p.scanChunks - 1) / (kScanItems * p.scanChunks);
    p.scanStatus = c->scanStatus + (size_t)c->parity * kScanMaxBlocks;
    p.scanStatusNext = c->scanStatus + (size_t)(c->parity ^ 1u) * kScanMaxBlocks;
    p.counts = c->counts;
    p.passed = c->passed;
    p.bound = (c->bound && c->jit && c->model.boundable) ? 1u : 0u;
    p.mpuMasks = c->mpuMasks;
    p.offs = c->offs;
    p.vk = c->vk;
    p.vp = c->vp;
    p.vShardCap = c->vShardCap;
    p.tq = c->tq;
    p.tShardCap = c->tShardCap;
    p.pos = c->pos;
    p.nrm = c->nrm;
    p.col = c->col;
    p.tris = c->tris;
    p.vCap = c->vcap;
    p.tCap = c->tcap;
    p.ctr = c->ctr + c->parity;
    p.ctrNext = c->ctr + (c->parity ^ 1u);
    p.hostCtr = c->hostCtrDev;
    p.totals = c->totals;
    p.stamps = c->stamps;
    p.stampCap = c->stamps ? c->stampCap : 0u;
    p.spans = (c->spans && c->spanNext < c->spanCap)
                  ? c->spans + (size_t)c->spanNext * 2 * kNumStampKernels * kSpanLanes : nullptr;
    p.mpuTicks = c->mpuTicksOpt ? c->mpuTicks : nullptr;
    p.slotsPerLane = c->jit ? 0u : c->model.nSlots;
    p.debug = (uint32_t)c->debug;
    return p;
}

hipError_t launch_jit(hipFunction_t f, uint32_t blocks, uint32_t threads, size_t lds, hipStream_t s, Params& p) {
    void* args[] = {&p};
    return hipModuleLaunchKernel(f, blocks, 1, 1, threads, 1, 1, (unsigned)lds, s, args, nullptr);
}

// One polygonization = 5 kernels, no copies or fills: k_precheck resets the counters,
// k_finish publishes them to mapped host memory.
// The five launches of one polygonization (shared by direct launch and graph capture).
// k_finish layout for the next run (vertices per wave): a quad of lanes per vertex (16) when
// the last run's vertices, 16 per wave, fit the persistent grid's waves in one pass (each
// wave then walks a quarter of what a 64-vertex wave does), else a pair of lanes (32) when
// they do 32 per wave, otherwise one lane per vertex (64: fewest waves in total).
// A run alone on its device (c->alone) takes at most 32 per wave: the spans, not the total
// work, set its time (C3 full grid, one engine: 0.1077 vs 0.1110 ms with the quad k_vertex).
int finish_vpw(const psgpu_ctx* c) {
    if (c->finishQuad == 0) return 64;
    if (c->finishQuad == 1) return 16;
    if (c->finishQuad == 3) return 32;
    const uint64_t waves = (uint64_t)c->numCUs * (uint64_t)c->finishBlocksPerCU * 4u;
    if (c->lastV == 0) return 64;
    if ((uint64_t)c->lastV <= 16u * waves) return 16;
    if ((uint64_t)c->lastV <= 32u * waves || c->alone) return 32;
    return 64;
}

// k_vertex layout for the next run (vertices per wave): one lane per vertex (64: each lane's
// 4 edge samples as one walk, the least total work) when the last run's vertices, 16 per
// wave, would take more than one pass of the persistent grid; otherwise a quad of lanes per
// vertex (16: a quarter of the walk per wave, shorter spans).  The interpreter has the quad
// layout only.
int vertex_vpw(const psgpu_ctx* c) {
    if (!c->jit || c->vertexWide == 0) return 16;
    if (c->vertexWide == 1) return 64;
    const uint64_t waves = (uint64_t)c->numCUs * (uint64_t)c->vertexBlocksPerCU * 4u;
    return (uint64_t)c->lastV > 16u * waves && !c->alone ? 64 : 16;  // a lone run: the quad
}

// k_vertex + k_finish as one launch (k_surface) for the next run: 1 forces it, 2 (default) when
// both would take their quad layouts (a launch too small to fill the device: its step is the
// launch floor); only with the small-launch kernels (compiled with the split)
bool use_surface(const psgpu_ctx* c) {
    if (!c->jit || !c->jit->surface || c->fusedSurface == 0 || c->surfaceOff || c->crowded) return false;
    if (c->fusedSurface == 3) return c->jit->surfaceW != nullptr;  // the wide variant, every launch
    // a run alone on the device (a blocking caller, a frame-at-a-time editor) is bound by its
    // spans: the quad layouts in one launch, while their waves fill the device at most ~8 times
    // (C3 alone 0.110 vs 0.115 ms; C5's 512^3 frame, far more vertices, 0.613 vs 0.600:
    // profiles/r06_latency_ab.txt)
    const uint64_t loneMaxV = 16ull * 8ull * 24ull * (uint64_t)c->numCUs;  // 16 a wave, 24 waves a CU, 8 passes
    return c->fusedSurface == 1 ||
           (c->lastV != 0 && ((c->alone && c->lastV <= loneMaxV) || (vertex_vpw(c) == 16 && finish_vpw(c) == 16)));
}

int launch_all(psgpu_ctx* c, const Params& pin, hipStream_t s, bool timed) {
    Params p = pin;
    const uint32_t persistV = (uint32_t)(c->numCUs * c->vertexBlocksPerCU);
    const uint32_t persistF = (uint32_t)(c->numCUs * c->finishBlocksPerCU);
    const int vpw = finish_vpw(c);
    JitKernels* J = c->jit.get();
    if (timed) PSGPU_CHECK(hipEventRecord(c->ev[0], s));
    const bool split = use_split(c);
    if (use_front(c)) {  // S1 blocks, then S2 blocks taking the survivors as they are published
        PSGPU_CHECK(launch_jit(split ? J->frontS : J->front, p.preBlocks + p.mpuBlocks, 256,
                               mpu_lds_bytes(0) / (split ? 2 : 1), s, p));
        if (timed) {
            PSGPU_CHECK(hipEventRecord(c->ev[1], s));
            PSGPU_CHECK(hipEventRecord(c->ev[2], s));
        }
    } else {
    if (J) PSGPU_CHECK(launch_jit(split ? J->precheckS : J->precheck, p.preBlocks, 256, 0, s, p));
    else PSGPU_CHECK(launch_precheck(p, s));
    if (timed) PSGPU_CHECK(hipEventRecord(c->ev[1], s));
    // the split kernel's blocks hold 2 MPUs, the others 4 (mpu_lds_bytes(0): 4 MPUs' LDS)
    if (J) PSGPU_CHECK(launch_jit(split ? J->mpuS : J->mpu, p.mpuBlocks, 256, mpu_lds_bytes(0) / (split ? 2 : 1), s, p));
    else PSGPU_CHECK(launch_mpu(p, s));
    if (timed) PSGPU_CHECK(hipEventRecord(c->ev[2], s));
    }
    // k_vertex's first scanBlocks blocks also compute the mesh offsets (all co-resident)
    const int vpwV = J ? vertex_vpw(c) : 16;
    uint32_t gridV = std::max(persistV, p.scanBlocks);
    uint32_t gridF = persistF;
    if (c->gridFit && c->lastV) {
        // grids fitted to the last finished run: a wave per batch of its vertices + 1/8 (both
        // kernels stride over any rest), not the persistent grids' mostly empty waves
        const uint64_t vv = (uint64_t)c->lastV + c->lastV / 8 + 256;
        gridV = std::max(p.scanBlocks, std::min<uint32_t>(gridV, (uint32_t)((vv + 4ull * vpwV - 1) / (4ull * vpwV))));
        gridF = std::min<uint32_t>(gridF, (uint32_t)((vv + 4ull * vpw - 1) / (4ull * vpw)));
    }
    if (use_surface(c)) {  // both quad layouts in one launch: the vertex grid (16 per wave)
        const bool wide = c->fusedSurface == 3;  // or one lane per vertex: k_finish's grid (64 per wave)
        const uint32_t perBlock = wide ? 256u : 64u;
        uint32_t gridS = std::max(wide ? persistF : persistV, p.scanBlocks);
        if (c->gridFit && c->lastV) {
            const uint64_t vv = (uint64_t)c->lastV + c->lastV / 8 + 256;
            gridS = std::max(p.scanBlocks, std::min<uint32_t>(gridS, (uint32_t)((vv + perBlock - 1) / perBlock)));
        }
        PSGPU_CHECK(launch_jit(wide ? J->surfaceW : J->surface, gridS, 256, 0, s, p));
        if (timed) {
            PSGPU_CHECK(hipEventRecord(c->ev[3], s));
            PSGPU_CHECK(hipEventRecord(c->ev[4], s));
        }
        return PSGPU_RET_SUCCESS;
    }
    if (J) PSGPU_CHECK(launch_jit(vpwV == 64 ? J->vertexW : J->vertex, gridV, 256, 0, s, p));
    else PSGPU_CHECK(launch_vertex(p, s, gridV));
    if (timed) PSGPU_CHECK(hipEventRecord(c->ev[3], s));
    if (J) PSGPU_CHECK(launch_jit(vpw == 16 ? J->finishQ : (vpw == 32 ? J->finishP : J->finish), gridF, 256, 0, s, p));
    else PSGPU_CHECK(launch_finish(p, s, gridF, vpw));
    if (timed) PSGPU_CHECK(hipEventRecord(c->ev[4], s));
    return PSGPU_RET_SUCCESS;
}

void drop_graphs(psgpu_ctx* c) {
    for (auto& g : c->graphs) {
        if (g.exec) (void)hipGraphExecDestroy(g.exec);
        g = psgpu_ctx::GraphSlot{};
    }
}

// One polygonization = 5 kernels, no copies or fills: k_precheck needs nothing reset
// (k_finish of the previous run reset this run's counters) and k_finish publishes the
// counters to mapped host memory.  Replayed from a hipGraph (one per counter set) while
// the launch parameters repeat, e.g. per frame of an animation.
void reset_run_state(psgpu_ctx* c);
int enqueue(psgpu_ctx* c, hipStream_t s) {
    if (c->mpuCount == 0) {  // nothing to launch: an empty result
        c->runTicks = c->mpuTicksOpt != 0;
        memset(c->hostCtr, 0, sizeof(DevCounters));
        c->hostCtr->firstOverflow = 0x7fffffff;
        // the totals the count exchange reads (k_finish writes them on a real run): zero
        // MPUs, no overflow -- never a previous run's
        PSGPU_CHECK(hipMemcpyAsync(c->totals, c->emptyTotals, 8 * sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
        return PSGPU_RET_SUCCESS;
    }
    if (c->debug & (1 << 28)) {  // test hook: 3 runs short of the epoch's wrap
        c->debug &= ~(1 << 28);
        reset_run_state(c);
        DevCounters near;
        PSGPU_CHECK(hipMemcpy(&near, c->ctr, sizeof(DevCounters), hipMemcpyDeviceToHost));
        near.epoch = 0xfffffffcu;
        PSGPU_CHECK(hipMemcpy(c->ctr, &near, sizeof(DevCounters), hipMemcpyHostToDevice));
        c->epochRuns = near.epoch;
    }
    // a run at epoch 0xffffffff would tag k_front's entries 0, the value of ready words no run
    // has written: restart the counter sets at epoch 0 with the ready words zeroed (a stream
    // drain once in 2^32 runs)
    if (c->epochRuns >= 0xffffffffull) reset_run_state(c);
    ++c->epochRuns;
    const Params p = make_params(c);
    c->runTicks = p.mpuTicks != nullptr;
    c->debug &= ~((1 << 20) | (1 << 25) | (1 << 26) | (1 << 27));  // the short-grid / protocol test hooks apply to one run
    if (p.spans) c->spanNext++;
    c->runMpuBlocks = p.mpuBlocks;
    c->runMpb = use_split(c) ? 2u : (uint32_t)kMpusPerBlock;
    const uint32_t slot = c->parity;
    c->parity ^= 1u;  // k_finish of this run resets the other set for the next run
    const bool timed = c->timing != 0;
    c->runSurface = use_surface(c);
    c->runFront = use_front(c);
    c->runSplit = use_split(c);
    if (c->stamps)  // waves that do not run leave no stale records
        PSGPU_CHECK(hipMemsetAsync(c->stamps, 0, (size_t)kNumStampKernels * c->stampCap * 24 + (size_t)c->stampCap * 64, s));
    if (!c->useGraph || timed || s == nullptr) {
        const int rc = launch_all(c, p, s, timed);
        if (rc != PSGPU_RET_SUCCESS) reset_run_state(c);
        return rc;
    }
    psgpu_ctx::GraphSlot& g = c->graphs[slot];
    const uint32_t shape[6] = {(uint32_t)c->vertexBlocksPerCU, (uint32_t)c->finishBlocksPerCU, (uint32_t)c->numCUs,
                               (uint32_t)finish_vpw(c), (uint32_t)vertex_vpw(c),
                               (use_split(c) ? 1u : 0u) | (use_surface(c) ? 2u : 0u) | (use_front(c) ? 4u : 0u)};
    if (!(g.exec && g.jit == c->jit.get() && memcmp(&g.key, &p, sizeof(Params)) == 0 &&
          memcmp(g.shape, shape, sizeof(shape)) == 0)) {
        if (g.exec) (void)hipGraphExecDestroy(g.exec);
        g = psgpu_ctx::GraphSlot{};
        hipGraph_t graph = nullptr;
        PSGPU_CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        const int rc = launch_all(c, p, s, false);
        const hipError_t ec = hipStreamEndCapture(s, &graph);
        if (rc != PSGPU_RET_SUCCESS) {
            if (graph) (void)hipGraphDestroy(graph);
            reset_run_state(c);
            return rc;
        }
        PSGPU_CHECK(ec);
        const hipError_t ei = hipGraphInstantiate(&g.exec, graph, nullptr, nullptr, 0);
        (void)hipGraphDestroy(graph);
        PSGPU_CHECK(ei);
        g.key = p;
        g.jit = c->jit.get();
        memcpy(g.shape, shape, sizeof(shape));
    }
    PSGPU_CHECK(hipGraphLaunch(g.exec, s));
    return PSGPU_RET_SUCCESS;
}

// Contexts with a run enqueued and not yet collected (psgpu_finish), per device, over the
// process: a run enqueued while no other context has one pending on its device is alone on
// it (a blocking caller, a frame-at-a-time editor, one context queueing its frames) and takes
// the layouts with the shortest spans; runs that overlap other contexts' (contexts taking
// frames in turn) take the layouts with the least total work.
std::atomic<int> g_pendingRuns[64];
constexpr int kMaxWaitingPeers = 4;  // see psgpu_polygonize: crowded
void set_pending(psgpu_ctx* c, bool v) {
    if (c->pending == v) return;
    c->pending = v;
    g_pendingRuns[c->device & 63].fetch_add(v ? 1 : -1);
}

// PrintThreadResults' counters (PS_Polygonizer.cpp:15-18, :443-469): the reference keeps a
// (processed, crossed) pair per TBB worker that ran any MPU, over every Polygonize of the
// process, enumerated in the order the workers first ran one, and cleared by
// PrintThreadResults (.cpp:414-428).  The library's worker is a device context (one stream,
// one polygonization at a time): every finished run adds its range's MPUs and its MPUs with
// at least one triangle to its context's entry; an entry outlives its context, as a TBB
// worker's counter outlives the call that made it, until the next print clears them all.
std::atomic<uint64_t> g_ctxSerial{0};
std::mutex g_threadMu;
std::vector<std::pair<uint64_t, std::pair<uint64_t, uint64_t>>> g_threadCounts;  // serial -> (processed, crossed)
void thread_results_add(uint64_t serial, uint32_t processed, uint32_t crossed) {
    if (processed == 0) return;  // a worker that ran no MPU has no entry (never called local())
    std::lock_guard<std::mutex> lk(g_threadMu);
    for (auto& e : g_threadCounts)
        if (e.first == serial) {
            e.second.first += processed;
            e.second.second += crossed;
            return;
        }
    g_threadCounts.push_back({serial, {processed, crossed}});
}

// Adopt the model's specialised kernels once their compile has finished (wait: block for
// it).  Until then the interpreter runs; its output is bit-identical.  Call with the
// context's device current.
void jit_poll(psgpu_ctx* c, bool wait) {
    if (!c->jitPending) return;
    if (!wait && c->jitFut.wait_for(std::chrono::seconds(0)) != std::future_status::ready) return;
    std::shared_ptr<const JitCode> code = c->jitFut.get();
    c->jitPending = false;
    c->jitFut = JitFuture();
    if (c->pending) (void)hipStreamSynchronize(c->runStream);
    drop_graphs(c);
    c->jit = jit_load(*code, c->device, &c->jitError);
    if (!c->jit && code->code.size() && c->jitError.find("dropped") != std::string::npos) {
        // the cached object would not load: compile it afresh (bypassing the disk cache)
        c->jitFut = jit_request(c->model, c->useJit == 2, false, c->treeSplit != 0);
        c->jitPending = true;
        if (wait) jit_poll(c, true);
        return;
    }
    if (!c->jit) fprintf(stderr, "psgpu: JIT unavailable, using the interpreter: %s\n", c->jitError.c_str());
    c->tier = c->jit ? (c->useJit == 2 ? 2 : 1) : 0;
}

// PSGPU_OPT_JIT 3: adopt the baked kernels once their compile has finished (wait: block).
void tier_poll(psgpu_ctx* c, bool wait) {
    if (!c->tier2Pending) return;
    if (!wait && c->tier2Fut.wait_for(std::chrono::seconds(0)) != std::future_status::ready) return;
    std::shared_ptr<const JitCode> code = c->tier2Fut.get();
    c->tier2Pending = false;
    c->tier2Fut = JitFuture();
    std::string err;
    std::shared_ptr<JitKernels> k = jit_load(*code, c->device, &err);
    if (!k) {  // the structure kernels keep serving this model
        c->tier2Failed = true;
        fprintf(stderr, "psgpu: baked kernels unavailable, the structure kernels stay: %s\n", err.c_str());
        return;
    }
    if (c->pending && c->useGraph) (void)hipStreamSynchronize(c->runStream);  // no graph dies in flight
    drop_graphs(c);  // modules live as long as the process: in-flight runs keep theirs
    c->jit1 = c->jit;
    c->jit = k;
    c->tier = 2;
}

// PSGPU_OPT_JIT 3: count a run of the unchanged model on the structure kernels and start the
// baked compile at the threshold.
void tier_count(psgpu_ctx* c) {
    if (c->useJit != 3 || c->tier != 1 || c->tier2Pending || c->tier2Failed) return;
    if (++c->staticRuns < c->tierRuns) return;
    c->tier2Fut = jit_request(c->model, true, true, c->treeSplit != 0);
    c->tier2Pending = true;
}

// Start (or restart) the compile of the current model's kernels.
void jit_start(psgpu_ctx* c) {
    c->jit.reset();
    c->jit1.reset();
    // a compile still running for the previous model or options finishes in the background, and
    // psgpu_destroy waits for it: a hiprtc thread left running into process exit can outlive
    // the compiler's own lazily built statics (a core dump after a run that changed options
    // under a compile, tools/fuzz_parity.py in round 6)
    if (c->jitPending && c->jitFut.valid()) c->retired.push_back(c->jitFut);
    c->jitPending = false;
    c->jitFut = JitFuture();
    c->tier = 0;
    c->staticRuns = 0;
    c->tier2Failed = false;
    if (c->tier2Pending) c->retired.push_back(c->tier2Fut);  // finishes in the background
    c->tier2Pending = false;
    c->tier2Fut = JitFuture();
    for (size_t i = 0; i < c->retired.size();) {  // forget the finished ones
        if (c->retired[i].wait_for(std::chrono::seconds(0)) == std::future_status::ready) {
            c->retired.erase(c->retired.begin() + (long)i);
        } else {
            ++i;
        }
    }
    if (!c->useJit || !c->haveModel) return;
    c->jitFut = jit_request(c->model, c->useJit == 2, true, c->treeSplit != 0);
    c->jitPending = true;
    jit_poll(c, !c->jitAsync);
}

// Put a context whose launch sequence failed part-way back into a usable state: the
// next run's counters and look-back words were to be reset by this run's k_finish.
void reset_run_state(psgpu_ctx* c) {
    DevCounters init[2];
    memset(init, 0, sizeof(init));
    init[0].firstOverflow = init[1].firstOverflow = 0x7fffffff;
    (void)hipStreamSynchronize(c->stream);
    (void)hipMemcpy(c->ctr, init, sizeof(init), hipMemcpyHostToDevice);
    (void)hipMemset(c->scanStatus, 0, 2 * kScanMaxBlocks * sizeof(uint64_t));
    if (c->fqReady) (void)hipMemset(c->fqReady, 0, c->capFq * sizeof(uint32_t));  // the epochs restart at 0
    (void)hipDeviceSynchronize();
    c->parity = 0;
    c->epochRuns = 0;
    drop_graphs(c);
}

}  // namespace

// ===========================================================================
extern "C" {

const char* psgpu_version(void) { return "parsip_amd 0.1 (gfx950)"; }

void psgpu_tritable(int32_t out[256 * 16]) {
    const CubeTables& T = cube_tables();
    for (int c = 0; c < 256; ++c)
        for (int i = 0; i < 16; ++i) out[c * 16 + i] = T.tri[c][i];
}

uint32_t psgpu_count_mpus(float cellsize, const float lo[3], const float hi[3]) {
    if (!(cellsize > 0.0f)) return 0;
    PsVec3f l{lo[0], lo[1], lo[2]}, h{hi[0], hi[1], hi[2]};
    uint32_t d[3];
    lattice_dims(cellsize, l, h, d);
    return d[0] * d[1] * d[2];
}

int psgpu_mpu_dims(float cellsize, const PsSoaBlobPrims* prims, uint32_t dims[3]) {
    if (!prims || !(cellsize > 0.0f)) return PSGPU_RET_PARAM_ERROR;
    lattice_dims(cellsize, prims->bboxLo, prims->bboxHi, dims);
    return PSGPU_RET_SUCCESS;
}

int psgpu_translate_blobtree_type(int t) {
    // _constSettings.h:26-38 -> PS_Polygonizer.h:84-91
    static const int map[29] = {
        PSGPU_PRIM_POINT, PSGPU_PRIM_LINE, PSGPU_PRIM_CYLINDER, PSGPU_PRIM_DISC, PSGPU_PRIM_RING,
        PSGPU_PRIM_POLYGON, PSGPU_PRIM_CUBE, PSGPU_PRIM_TRIANGLE, PSGPU_PRIM_CATMULLROM, PSGPU_PRIM_SKELETON,
        PSGPU_PRIM_QUADRICPOINT, PSGPU_PRIM_HALFPLANE, PSGPU_PRIM_NULL, -1 /* Instance */,
        PSGPU_OP_UNION, PSGPU_OP_INTERSECT, PSGPU_OP_DIF, PSGPU_OP_SMOOTHDIF, PSGPU_OP_BLEND,
        PSGPU_OP_RICCIBLEND, PSGPU_OP_GRADIENTBLEND, PSGPU_PRIM_FASTQPS, PSGPU_OP_PCM, PSGPU_OP_CACHE,
        PSGPU_OP_WARPTWIST, PSGPU_OP_WARPTAPER, PSGPU_OP_WARPBEND, PSGPU_OP_WARPSHEAR, PSGPU_OP_TEXTURE};
    return (t >= 0 && t < 29) ? map[t] : -1;
}

// PrepareBBoxes (PS_Polygonizer.cpp:55-309) with iso distance ISO_DIST + 5*MIN_CELL_SIZE.
int psgpu_prepare_bboxes(float cellsize, PsSoaBlobPrims* P, PsSoaBoxMatrices* BM, PsSoaBlobOps* O) {
    (void)cellsize;
    if (!P || !O || P->ctPrims == 0 || P->ctPrims > 128) return PSGPU_RET_PARAM_ERROR;
    const float iso = PSGPU_ISO_DIST + 5.0f * PSGPU_MIN_CELL_SIZE;
    float* boxLo[3] = {P->vPrimBoxLoX, P->vPrimBoxLoY, P->vPrimBoxLoZ};
    float* boxHi[3] = {P->vPrimBoxHiX, P->vPrimBoxHiY, P->vPrimBoxHiZ};
    for (uint32_t i = 0; i < P->ctPrims; ++i) {
        const float p[3] = {P->posX[i], P->posY[i], P->posZ[i]};
        const float d[3] = {P->dirX[i], P->dirY[i], P->dirZ[i]};
        float lo[3], hi[3];
        for (int a = 0; a < 3; ++a) { lo[a] = boxLo[a][i]; hi[a] = boxHi[a][i]; }
        switch (P->skeletType[i]) {
        case PSGPU_PRIM_POINT:
            for (int a = 0; a < 3; ++a) { lo[a] = p[a] - iso; hi[a] = p[a] + iso; }
            break;
        case PSGPU_PRIM_LINE:
            for (int a = 0; a < 3; ++a) {
                const float e = iso * 1.0f + (3.0f * iso) * (d[a] - p[a]);
                lo[a] = p[a] - e; hi[a] = d[a] + e;
            }
            break;
        case PSGPU_PRIM_RING: case PSGPU_PRIM_DISC: {
            const float r = P->resX[i] + iso;
            for (int a = 0; a < 3; ++a) {
                const float e = (r + iso) * (1.0f - d[a]) + iso * d[a];
                lo[a] = p[a] - e; hi[a] = p[a] + e;
            }
        } break;
        case PSGPU_PRIM_CYLINDER: {
            const float r = P->resX[i], h = P->resY[i];
            for (int a = 0; a < 3; ++a) {
                const float s1 = p[a] + h * d[a];
                const float e = (iso + r) * 1.0f + (0.5f * iso) * d[a];
                lo[a] = p[a] - e; hi[a] = s1 + e;
            }
        } break;
        case PSGPU_PRIM_CUBE: {
            const float s = P->resX[i] + iso;
            for (int a = 0; a < 3; ++a) { lo[a] = p[a] - s; hi[a] = p[a] + s; }
        } break;
        case PSGPU_PRIM_TRIANGLE: {
            const float r[3] = {P->resX[i], P->resY[i], P->resZ[i]};
            for (int a = 0; a < 3; ++a) {
                float mn = p[a] < d[a] ? p[a] : d[a];
                mn = mn < r[a] ? mn : r[a];
                float mx = p[a] > d[a] ? p[a] : d[a];
                mx = mx > r[a] ? mx : r[a];
                lo[a] = mn - iso; hi[a] = mx + iso;
            }
        } break;
        default: break;
        }
        const uint32_t im = P->idxMatrix[i];
        if (im != 0 && BM && im < BM->count) {  // mat4Transform, PS_MATRIX4.h:199-209 (column vectors)
            const float* M = &BM->matrix[im * PSGPU_BOX_MATRIX_STRIDE];
            float tl[3], th[3];
            for (int r = 0; r < 3; ++r) {
                tl[r] = ((M[r] * lo[0] + M[4 + r] * lo[1]) + M[8 + r] * lo[2]) + M[12 + r];
                th[r] = ((M[r] * hi[0] + M[4 + r] * hi[1]) + M[8 + r] * hi[2]) + M[12 + r];
            }
            memcpy(lo, tl, sizeof(lo));
            memcpy(hi, th, sizeof(hi));
        }
        for (int a = 0; a < 3; ++a) { boxLo[a][i] = lo[a]; boxHi[a][i] = hi[a]; }
        float* bl = &P->bboxLo.x;
        float* bh = &P->bboxHi.x;
        for (int a = 0; a < 3; ++a) {
            if (i == 0) { bl[a] = lo[a]; bh[a] = hi[a]; }
            else { bl[a] = bl[a] < lo[a] ? bl[a] : lo[a]; bh[a] = bh[a] > hi[a] ? bh[a] : hi[a]; }
        }
    }
    if (O->ctOps > 0) {  // op boxes bottom-up (:238-307) as a post-order walk
        std::vector<uint8_t> done(256, 0);
        std::vector<uint32_t> st{0};
        size_t guard = 0;
        while (!st.empty()) {
            if (++guard > 100000) return PSGPU_RET_INVALID_BVH;
            const uint32_t op = st.back();
            if (op >= 128) return PSGPU_RET_INVALID_BVH;
            const uint32_t L = O->opLeftChild[op], R = O->opRightChild[op];
            const int lop = (O->opChildKind[op] & 2) >> 1, rop = O->opChildKind[op] & 1;
            if ((lop && !done[L]) || (rop && !done[R])) {
                if (lop && !done[L]) st.push_back(L);
                if (rop && !done[R]) st.push_back(R);
                continue;
            }
            st.pop_back();
            auto get = [&](int isOp, uint32_t k, float lo[3], float hi[3]) {
                if (isOp) {
                    lo[0] = O->vBoxLoX[k]; lo[1] = O->vBoxLoY[k]; lo[2] = O->vBoxLoZ[k];
                    hi[0] = O->vBoxHiX[k]; hi[1] = O->vBoxHiY[k]; hi[2] = O->vBoxHiZ[k];
                } else {
                    for (int a = 0; a < 3; ++a) { lo[a] = boxLo[a][k]; hi[a] = boxHi[a][k]; }
                }
            };
            float l0[3], h0[3], l1[3], h1[3];
            get(lop, L, l0, h0);
            get(rop, R, l1, h1);
            float* oLo[3] = {O->vBoxLoX, O->vBoxLoY, O->vBoxLoZ};
            float* oHi[3] = {O->vBoxHiX, O->vBoxHiY, O->vBoxHiZ};
            for (int a = 0; a < 3; ++a) {
                oLo[a][op] = l0[a] < l1[a] ? l0[a] : l1[a];
                oHi[a][op] = h0[a] > h1[a] ? h0[a] : h1[a];
            }
            done[op] = 1;
        }
    }
    return PSGPU_RET_SUCCESS;
}

int psgpu_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int psgpu_create(int deviceOrdinal, psgpu_ctx** out) {
    if (!out) return PSGPU_RET_PARAM_ERROR;
    *out = nullptr;
    int n = psgpu_device_count();
    if (deviceOrdinal < 0 || deviceOrdinal >= n) return PSGPU_RET_DEVICE_ERROR;
    psgpu_ctx* c = new psgpu_ctx();
    c->device = deviceOrdinal;
    c->serial = ++g_ctxSerial;
    int rc = set_device(c);
    if (rc != PSGPU_RET_SUCCESS) { delete c; return rc; }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, deviceOrdinal) == hipSuccess && prop.multiProcessorCount > 0)
        c->numCUs = prop.multiProcessorCount;
    c->splitMaxQueued = 4u * (uint32_t)c->numCUs;
    const CubeTables& T = cube_tables();
    CubeTablesDev tabHost{};
    fill_device_tables(T, tabHost);
    // the set-up copies run on the null stream BEFORE this context's stream exists: a process's
    // first stream created ahead of the null stream's first use shares its hardware queue
    // (tools/queue_probe.py: with 4 engines, the engine on that stream slowed every step ~25%)
    if (hipMalloc(&c->dTables, sizeof(CubeTablesDev)) != hipSuccess ||
        hipMemcpy(c->dTables, &tabHost, sizeof(CubeTablesDev), hipMemcpyHostToDevice) != hipSuccess ||
        hipMalloc(&c->dModel, sizeof(DevModel)) != hipSuccess ||
        hipMalloc(&c->ctr, 2 * sizeof(DevCounters)) != hipSuccess ||
        hipMalloc(&c->totals, 16 * sizeof(uint32_t)) != hipSuccess ||
        hipMalloc(&c->scanStatus, 2 * kScanMaxBlocks * sizeof(uint64_t)) != hipSuccess ||
        hipMemset(c->scanStatus, 0, 2 * kScanMaxBlocks * sizeof(uint64_t)) != hipSuccess ||
        hipHostMalloc(&c->hostCtr, sizeof(DevCounters), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
        hipHostGetDevicePointer(reinterpret_cast<void**>(&c->hostCtrDev), c->hostCtr, 0) != hipSuccess ||
        hipDeviceSynchronize() != hipSuccess ||
        hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        psgpu_destroy(c);
        return PSGPU_RET_DEVICE_ERROR;
    }
    memset(c->hostCtr, 0, sizeof(DevCounters));
    c->hostCtr->firstOverflow = 0x7fffffff;
    c->emptyTotals = c->totals + 8;  // {0, 0, 0, 0, 0, 0, no overflow, no error}
    {
        const uint32_t empty[16] = {0, 0, 0, 0, 0, 0, 0x7fffffffu, 0, 0, 0, 0, 0, 0, 0, 0x7fffffffu, 0};
        if (hipMemcpy(c->totals, empty, sizeof(empty), hipMemcpyHostToDevice) != hipSuccess) {
            psgpu_destroy(c);
            return PSGPU_RET_DEVICE_ERROR;
        }
    }
    {
        DevCounters init[2];
        memset(init, 0, sizeof(init));
        init[0].firstOverflow = init[1].firstOverflow = 0x7fffffff;
        if (hipMemcpy(c->ctr, init, sizeof(init), hipMemcpyHostToDevice) != hipSuccess) {
            psgpu_destroy(c);
            return PSGPU_RET_DEVICE_ERROR;
        }
    }
    for (int i = 0; i <= kNumKernels; ++i) (void)hipEventCreate(&c->ev[i]);
    const char* cullEnv = getenv("PSGPU_CULL");
    if (cullEnv) c->cull = atoi(cullEnv) != 0;
    const char* jitEnv = getenv("PSGPU_JIT");
    if (jitEnv) c->useJit = std::min(3, std::max(0, atoi(jitEnv)));
    const char* asyncEnv = getenv("PSGPU_JIT_ASYNC");
    if (asyncEnv) c->jitAsync = atoi(asyncEnv) != 0;
    if (const char* e = getenv("PSGPU_GRID_FIT")) c->gridFit = atoi(e) != 0;          // 0: persistent grids
    if (const char* e = getenv("PSGPU_FINISH_QUAD")) c->finishQuad = std::min(3, std::max(0, atoi(e)));
    if (const char* e = getenv("PSGPU_VERTEX_WIDE")) c->vertexWide = std::min(2, std::max(0, atoi(e)));
    if (const char* e = getenv("PSGPU_MPU_MARGIN")) c->mpuMarginDiv = std::max(1, atoi(e));
    if (const char* e = getenv("PSGPU_FUSED_SURFACE")) c->fusedSurface = std::min(3, std::max(0, atoi(e)));
    if (const char* e = getenv("PSGPU_FRONT")) c->front = std::min(2, std::max(0, atoi(e)));
    *out = c;
    return PSGPU_RET_SUCCESS;
}

void psgpu_destroy(psgpu_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    set_pending(c, false);
    drop_graphs(c);
    // an in-flight hiprtc compile must not outlive its owner: a process that exits while
    // LLVM compiles on the job thread tears LLVM's statics down under it
    if (c->jitPending && c->jitFut.valid()) c->jitFut.wait();
    if (c->tier2Pending && c->tier2Fut.valid()) c->tier2Fut.wait();
    for (JitFuture& f : c->retired)
        if (f.valid()) f.wait();
    c->jitFut = JitFuture();
    c->tier2Fut = JitFuture();
    c->jit.reset();
    c->jit1.reset();
    void* bufs[] = {c->dModel, c->dTables, c->pq, c->pqMask, c->pqOct, c->fqReady, c->scanStatus, c->counts, c->passed, c->mpuMasks, c->offs, c->vk, c->vp, c->tq,
                    c->pos, c->nrm, c->col, c->tris, c->ctr, c->totals, c->stamps, c->spans, c->mpuTicks};
    for (void* b : bufs)
        if (b) (void)hipFree(b);
    if (c->hostCtr) (void)hipHostFree(c->hostCtr);
    if (c->clockProbe) (void)hipHostFree(c->clockProbe);
    if (c->hostStage) (void)hipHostFree(c->hostStage);
    for (int i = 0; i <= kNumKernels; ++i)
        if (c->ev[i]) (void)hipEventDestroy(c->ev[i]);
    for (hipEvent_t e : c->exportEv)
        if (e) (void)hipEventDestroy(e);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

int psgpu_set_option(psgpu_ctx* c, int option, int64_t value) {
    if (!c) return PSGPU_RET_PARAM_ERROR;
    const int drc = set_device(c);  // modules load and buffers free on the context's device
    if (drc != PSGPU_RET_SUCCESS) return drc;
    if (option == PSGPU_OPT_KERNEL_TIMING) c->timing = value != 0;
    else if (option == PSGPU_OPT_CULLING) c->cull = value != 0;
    else if (option == PSGPU_OPT_DEBUG) c->debug = (int)value;
    else if (option == PSGPU_OPT_GRAPH) c->useGraph = value != 0;
    else if (option == PSGPU_OPT_BOUND) c->bound = value != 0;
    else if (option == PSGPU_OPT_CAPACITY && value >= 64 && value <= (1ll << 30)) {
        // restart the output / work-queue buffers at this vertex capacity (they grow on demand);
        // a pending result is dropped with them
        if (c->pending) (void)hipStreamSynchronize(c->runStream);
        set_pending(c, false);
        c->seenV = c->seenT = c->seenShardV = c->seenShardT = 0;
        void* bufs[] = {c->vk, c->vp, c->tq, c->pos, c->nrm, c->col, c->tris};
        for (void* b : bufs)
            if (b) (void)hipFree(b);
        c->vk = nullptr; c->vp = nullptr; c->tq = nullptr; c->pos = nullptr; c->nrm = nullptr; c->col = nullptr; c->tris = nullptr;
        c->capVk = c->capVp = c->capTq = c->capV = c->capT = 0;
        c->vcap = (uint32_t)value;
        c->tcap = (uint32_t)std::min<int64_t>(2 * value, 0xffffffffll);
        c->vShardCap = (uint32_t)std::max<int64_t>(16, value / kShards);
        c->tShardCap = 2 * c->vShardCap;
        c->haveResult = false;
    }
    else if (option == PSGPU_OPT_VERTEX_BLOCKS_PER_CU && value >= 1 && value <= 32) c->vertexBlocksPerCU = (int)value;
    else if (option == PSGPU_OPT_FINISH_BLOCKS_PER_CU && value >= 1 && value <= 32) c->finishBlocksPerCU = (int)value;
    else if (option == PSGPU_OPT_FINISH_QUAD && value >= 0 && value <= 3) c->finishQuad = (int)value;
    else if (option == PSGPU_OPT_VERTEX_WIDE && value >= 0 && value <= 2) c->vertexWide = (int)value;
    else if (option == PSGPU_OPT_TREE_SPLIT && value >= 0 && value <= 2) {
        const bool recompile = value != 0 && c->treeSplit == 0 && c->haveModel && c->splittable &&
                               !(c->jit && c->jit->precheckS);
        c->treeSplit = (int)value;
        if (recompile) {  // the loaded kernels lack the split variants: generate them
            if (c->pending) (void)hipStreamSynchronize(c->runStream);
            drop_graphs(c);
            jit_start(c);
        }
    }
    else if (option == PSGPU_OPT_SPLIT_MAX_QUEUED && value >= 0 && value <= 0xffffffffll) c->splitMaxQueued = (uint32_t)value;
    else if (option == PSGPU_OPT_FUSED_SURFACE && value >= 0 && value <= 3) c->fusedSurface = (int)value;
    else if (option == PSGPU_OPT_FRONT && value >= 0 && value <= 2) c->front = (int)value;
    else if (option == PSGPU_OPT_TIER_RUNS && value >= 1 && value <= (1 << 30)) c->tierRuns = (int)value;
    else if (option == PSGPU_OPT_JIT) {
        if (value < 0 || value > 3) return PSGPU_RET_PARAM_ERROR;
        c->useJit = (int)value;
        if (c->pending) (void)hipStreamSynchronize(c->runStream);
        drop_graphs(c);
        jit_start(c);
    }
    else if (option == PSGPU_OPT_JIT_ASYNC) c->jitAsync = value != 0;
    else if (option == PSGPU_OPT_MPU_TICKS) c->mpuTicksOpt = value != 0;  // buffers: next polygonize
    else if (option == PSGPU_OPT_SPANS && value >= 0 && value <= (1 << 20)) {
        // the next `value` runs record their kernel spans, one slot each (then none)
        if (c->pending) (void)hipStreamSynchronize(c->runStream);
        if (c->spans) (void)hipFree(c->spans);
        c->spans = nullptr;
        c->spanCap = c->spanNext = 0;
        drop_graphs(c);
        if (value > 0) {
            std::vector<uint64_t> init((size_t)value * 2 * kNumStampKernels * kSpanLanes);
            for (size_t i = 0; i < init.size(); i += 2) {
                init[i] = ~0ull;
                init[i + 1] = 0ull;
            }
            PSGPU_CHECK(hipMalloc(&c->spans, init.size() * 8));
            PSGPU_CHECK(hipMemcpy(c->spans, init.data(), init.size() * 8, hipMemcpyHostToDevice));
            c->spanCap = (uint32_t)value;
        }
    }
    else if (option == PSGPU_OPT_STAMPS && value >= 0 && value <= (1 << 24)) {
        if (c->pending) (void)hipStreamSynchronize(c->runStream);
        if (c->stamps) (void)hipFree(c->stamps);
        c->stamps = nullptr;
        c->stampCap = 0;
        drop_graphs(c);
        if (value > 0) {
            const size_t bytes = (size_t)kNumStampKernels * value * 24 + (size_t)value * 64;
            PSGPU_CHECK(hipMalloc(&c->stamps, bytes));
            PSGPU_CHECK(hipMemset(c->stamps, 0, bytes));  // a kernel a run does not launch leaves no rows
            c->stampCap = (uint32_t)value;
        }
    }
    else return PSGPU_RET_PARAM_ERROR;
    return PSGPU_RET_SUCCESS;
}

int psgpu_set_model(psgpu_ctx* c, const PsSoaBlobPrims* prims, const PsSoaPrimMatrices* mats,
                    const PsSoaBlobOps* ops) {
    if (!c || !prims || !mats || !ops) return PSGPU_RET_PARAM_ERROR;
    int rc = set_device(c);
    if (rc != PSGPU_RET_SUCCESS) return rc;
    DevModel* m = new DevModel;
    rc = build_device_model(*prims, *mats, *ops, *m);
    if (rc != PSGPU_RET_SUCCESS) { delete m; return rc; }
    if (c->pending) (void)hipStreamSynchronize(c->runStream);
    // captured graphs stay valid: specialised modules live as long as the process
    // (jit_get's cache) and the replay key compares the kernels and every parameter.
    // The same model again (build_device_model zeroes every byte first) keeps its kernels,
    // and with PSGPU_OPT_JIT 3 its tier and run count.
    const bool same = c->haveModel && memcmp(&c->model, m, sizeof(DevModel)) == 0;
    c->model = *m;
    delete m;
    c->splittable = jit_splittable(c->model);
    memcpy(&c->primsHost, prims, sizeof(PsSoaBlobPrims));
    if (!same) {  // the same bytes are already in HBM (a blocking caller re-sending its model)
        PSGPU_CHECK(hipMemcpyAsync(c->dModel, &c->model, sizeof(DevModel), hipMemcpyHostToDevice, c->stream));
        PSGPU_CHECK(hipStreamSynchronize(c->stream));
    }
    c->haveModel = true;
    if (!same || (!c->jit && !c->jitPending)) jit_start(c);
    return PSGPU_RET_SUCCESS;
}

int psgpu_polygonize(psgpu_ctx* c, float cellsize, uint32_t mpuBegin, uint32_t mpuEnd, void* stream) {
    if (!c || !c->haveModel) return PSGPU_RET_PARAM_ERROR;
    if (c->primsHost.ctPrims == 0 || !(cellsize > 0.0f)) return PSGPU_RET_PARAM_ERROR;
    int rc = set_device(c);
    if (rc != PSGPU_RET_SUCCESS) return rc;
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    if (c->pending && c->runStream != s) (void)hipStreamSynchronize(c->runStream);
    // validate into locals first: a rejected call leaves the lattice of a pending run (its
    // finish / export read c->cs and c->dims) untouched
    uint32_t dims[3];
    lattice_dims(cellsize, c->primsHost.bboxLo, c->primsHost.bboxHi, dims);
    const uint64_t total = (uint64_t)dims[0] * dims[1] * dims[2];
    if (total > 0xffffffffull) return PSGPU_RET_PARAM_ERROR;
    const uint32_t end = (uint32_t)std::min<uint64_t>(mpuEnd, total);
    const uint32_t begin = std::min(mpuBegin, end);
    if (end - begin >= kMaxRangeMpus) return PSGPU_RET_PARAM_ERROR;  // TriRec's 20-bit slot field
    c->cs = cellsize;
    memcpy(c->dims, dims, sizeof(dims));
    if (begin != c->mpuBegin || end - begin != c->mpuCount || cellsize != c->lastCs) {
        // another range or lattice: the last run's survivor count says nothing about this
        // one -- size k_mpu for the whole range (no re-run) until a run of it finishes.  A new
        // model on the same lattice (an animation frame) keeps the prediction; a frame that
        // queues more is re-run by finish(), and psgpu_comm_result agrees on that collectively.
        c->haveQueued = false;
        c->lastV = 0;
    }
    c->lastCs = cellsize;
    c->mpuBegin = begin;
    c->mpuCount = end - begin;
    jit_poll(c, false);
    tier_poll(c, false);
    tier_count(c);
    // capacity from the largest finished run + 1/4 (grows only; finish() still re-runs
    // on an overflow, so a prediction that falls short costs time, never output)
    c->vcap = std::max(c->vcap, c->seenV + c->seenV / 4);
    c->tcap = std::max(c->tcap, c->seenT + c->seenT / 4);
    c->vShardCap = std::max(c->vShardCap, c->seenShardV + c->seenShardV / 4);
    c->tShardCap = std::max(c->tShardCap, c->seenShardT + c->seenShardT / 4);
    rc = ensure_buffers(c, c->mpuCount);
    if (rc != PSGPU_RET_SUCCESS) return rc;
    // alone: no OTHER context has a run pending on the device (this context's own earlier
    // runs share its stream, so they never overlap this one)
    const int others = g_pendingRuns[c->device & 63].load() - (c->pending ? 1 : 0);
    c->alone = others == 0;
    // the launches with in-kernel waits (k_surface, k_front) only while at most 3 other contexts
    // of the process have runs in flight on the device: with more, the waiting blocks of all
    // their launches can hold every slot of an XCD that another launch's awaited blocks still
    // need (blocks go to the XCDs round-robin, each XCD dispatching its share in order), and the
    // waits end only at their bounds (6-8 engines on a C4 share: protocol errors, ms per step;
    // profiles/r06_engines_waits.txt)
    c->crowded = others >= kMaxWaitingPeers;
    rc = enqueue(c, s);
    if (rc != PSGPU_RET_SUCCESS) return rc;
    c->runStream = s;
    set_pending(c, true);
    c->haveResult = false;
    return PSGPU_RET_SUCCESS;
}

int psgpu_finish(psgpu_ctx* c, PsMeshInfo* info) {
    if (!c) return PSGPU_RET_PARAM_ERROR;
    if (c->pending) {
        int rc = set_device(c);
        if (rc != PSGPU_RET_SUCCESS) return rc;
        PSGPU_CHECK(hipStreamSynchronize(c->runStream));
        set_pending(c, false);
        // grow and re-run if the work queues or the compact outputs did not fit
        bool reran = false;
        for (int attempt = 0; attempt < 4; ++attempt) {
            const DevCounters& h = *c->hostCtr;
            uint32_t V = 0, T = 0, mv = 0, mt = 0, Q = 0;
            for (int k = 0; k < kShards; ++k) {
                V += h.shard[k].v;
                T += h.shard[k].t;
                Q += h.shard[k].p;
                mv = std::max(mv, h.shard[k].v);
                mt = std::max(mt, h.shard[k].t);
            }
            bool gridShort = c->mpuCount > 0 && Q > c->runMpb * c->runMpuBlocks;
            if (c->runFront) {  // k_front: each sub-queue against its own rows of S2 blocks
                uint32_t sub = 0;
                for (int k = 0; k < 8; ++k) sub = std::max(sub, h.shard[k].p);
                gridShort = c->mpuCount > 0 && sub > c->runMpb * (c->runMpuBlocks / 8u);
                c->lastSubMax = sub;
            } else {
                c->lastSubMax = 0;
            }
            c->lastQueued = Q;
            c->lastV = V;
            c->haveQueued = c->mpuCount > 0;
            c->seenV = std::max(c->seenV, V);
            c->seenT = std::max(c->seenT, T);
            c->seenShardV = std::max(c->seenShardV, mv);
            c->seenShardT = std::max(c->seenShardT, mt);
            if (!gridShort && V <= c->vcap && T <= c->tcap && mv <= c->vShardCap && mt <= c->tShardCap) break;
            if (attempt == 3) return PSGPU_RET_NOT_ENOUGH_MEM;  // still short after 3 regrowths
            c->vcap = std::max(c->vcap, V + V / 8 + 1024);
            c->tcap = std::max(c->tcap, T + T / 8 + 1024);
            c->vShardCap = std::max(c->vShardCap, mv + mv / 4 + 256);
            c->tShardCap = std::max(c->tShardCap, mt + mt / 4 + 256);
            rc = ensure_buffers(c, c->mpuCount);
            if (rc != PSGPU_RET_SUCCESS) return rc;
            rc = enqueue(c, c->runStream);
            if (rc != PSGPU_RET_SUCCESS) return rc;
            PSGPU_CHECK(hipStreamSynchronize(c->runStream));
            reran = true;
        }
        if (c->timing && c->mpuCount > 0) {
            for (int k = 0; k < kNumKernels; ++k) {
                float ms = 0.0f;
                if (hipEventElapsedTime(&ms, c->ev[k], c->ev[k + 1]) == hipSuccess) c->lastMs[k] = ms;
            }
        }
        const DevCounters& h = *c->hostCtr;
        if (c->mpuCount && (h.error | h.surfaceErr)) {
            // an in-kernel wait gave up (an offsets-scan look-back, or k_surface's wait for the
            // scan): the run's offsets are not trusted.  Re-run it once as k_vertex + k_finish,
            // the chain whose kernel boundaries order the scan; a second error fails the call.
            fprintf(stderr, "psgpu: device protocol error 0x%x (%s): re-running as separate launches\n",
                    h.error | h.surfaceErr, c->runFront ? (c->runSurface ? "k_front, k_surface" : "k_front")
                                                        : (c->runSurface ? "k_surface" : "k_vertex"));
            c->surfaceOff = true;
            rc = enqueue(c, c->runStream);
            c->surfaceOff = false;
            if (rc != PSGPU_RET_SUCCESS) return rc;
            PSGPU_CHECK(hipStreamSynchronize(c->runStream));
            reran = true;
            if (h.error | h.surfaceErr) {
                fprintf(stderr, "psgpu: device protocol error 0x%x\n", h.error | h.surfaceErr);
                return PSGPU_RET_DEVICE_ERROR;
            }
        }
        if (c->debug & (1 << 21)) {  // test hook: this finish fails as a protocol error would (one run)
            c->debug &= ~(1 << 21);
            return PSGPU_RET_DEVICE_ERROR;
        }
        uint32_t V = 0, T = 0, S = 0, P = 0, Q = 0;
        for (int k = 0; k < kShards; ++k) {
            V += h.shard[k].v;
            T += h.shard[k].t;
            S += h.shard[k].s;
            P += h.shard[k].p + h.shard[k].b;
            Q += h.shard[k].p;
        }
        PsMeshInfo& I = c->info;
        memset(&I, 0, sizeof(I));
        I.ctMPUs = c->mpuCount;
        I.ctPassedPrecheck = c->mpuCount ? P : 0;
        I.ctSurfaceMPUs = c->mpuCount ? S : 0;
        I.ctVertices = c->mpuCount ? V : 0;
        I.ctTriangles = c->mpuCount ? T : 0;
        I.firstOverflowMPU = (c->mpuCount && h.firstOverflow != 0x7fffffff) ? h.firstOverflow : -1;
        I.ctFieldMPUs = c->mpuCount ? Q : 0;
        I.ctLaneEvals = 8ull * c->mpuCount + 512ull * I.ctFieldMPUs + 8ull * I.ctVertices;
        I.launchFlags = c->mpuCount == 0 ? 0u
                        : (c->runSplit ? PSGPU_LAUNCH_TREE_SPLIT : 0u) | (c->runSurface ? PSGPU_LAUNCH_SURFACE : 0u) |
                              (c->runFront ? PSGPU_LAUNCH_FRONT : 0u) | (reran ? PSGPU_LAUNCH_RERUN : 0u);
        c->haveResult = true;
        if (c->countThreads) thread_results_add(c->serial, I.ctMPUs, I.ctSurfaceMPUs);
    }
    if (!c->haveResult) return PSGPU_RET_PARAM_ERROR;
    if (info) *info = c->info;
    return PSGPU_RET_SUCCESS;
}

int psgpu_download_stamps(psgpu_ctx* c, uint64_t* out, uint32_t* capOut) {
    int rc = psgpu_finish(c, nullptr);
    if (rc != PSGPU_RET_SUCCESS) return rc;
    if (capOut) *capOut = c->stamps ? c->stampCap : 0u;
    if (!c->stamps || !out) return c->stamps ? PSGPU_RET_SUCCESS : PSGPU_RET_PARAM_ERROR;
    PSGPU_CHECK(hipMemcpy(out, c->stamps, (size_t)kNumStampKernels * c->stampCap * 24 + (size_t)c->stampCap * 64,
                          hipMemcpyDeviceToHost));
    return PSGPU_RET_SUCCESS;
}

int psgpu_download_spans(psgpu_ctx* c, uint64_t* out, uint32_t* runs) {
    if (!c || !runs) return PSGPU_RET_PARAM_ERROR;
    *runs = c->spans ? c->spanNext : 0u;
    if (!c->spans || !out || c->spanNext == 0) return PSGPU_RET_SUCCESS;
    int rc = set_device(c);
    if (rc != PSGPU_RET_SUCCESS) return rc;
    if (c->pending) PSGPU_CHECK(hipStreamSynchronize(c->runStream));
    const size_t per = (size_t)2 * kNumStampKernels * kSpanLanes;
    std::vector<uint64_t> raw((size_t)c->spanNext * per);
    PSGPU_CHECK(hipMemcpy(raw.data(), c->spans, raw.size() * 8, hipMemcpyDeviceToHost));
    for (uint32_t r = 0; r < c->spanNext; ++r)
        for (int k = 0; k < kNumStampKernels; ++k) {
            uint64_t lo = ~0ull, hi = 0ull;
            for (int l = 0; l < kSpanLanes; ++l) {
                const uint64_t* s = &raw[r * per + 2 * ((size_t)k * kSpanLanes + l)];
                lo = std::min(lo, s[0]);
                hi = std::max(hi, s[1]);
            }
            out[(size_t)r * 2 * kNumStampKernels + 2 * k] = lo;
            out[(size_t)r * 2 * kNumStampKernels + 2 * k + 1] = hi;
        }
    return PSGPU_RET_SUCCESS;
}

int psgpu_thread_result_count(void) {
    std::lock_guard<std::mutex> lk(g_threadMu);
    return (int)g_threadCounts.size();
}

int psgpu_print_thread_results(int ctAttempts, uint32_t* lpThreadProcessed, uint32_t* lpThreadCrossed,
                               uint32_t capacity, int print) {
    if (ctAttempts <= 0) return PSGPU_RET_PARAM_ERROR;  // the reference divides by it
    std::lock_guard<std::mutex> lk(g_threadMu);
    const int n = (int)g_threadCounts.size();
    for (int i = 0; i < n; ++i) {
        // the reference's int pair divided by int (.cpp:421-424)
        const uint32_t pr = (uint32_t)(g_threadCounts[i].second.first / (uint64_t)ctAttempts);
        const uint32_t cr = (uint32_t)(g_threadCounts[i].second.second / (uint64_t)ctAttempts);
        if (lpThreadProcessed && (uint32_t)i < capacity) lpThreadProcessed[i] = pr;
        if (lpThreadCrossed && (uint32_t)i < capacity) lpThreadCrossed[i] = cr;
        if (print) printf("Thread#  %d, Processed MPUs %d, Crossed MPUs %d \n", i + 1, (int)pr, (int)cr);
    }
    if (print) fflush(stdout);
    g_threadCounts.clear();
    return n;
}

int psgpu_last_kernel_times(psgpu_ctx* c, float* ms, int maxKernels, const char** names) {
    if (!c) return 0;
    int n = std::min(maxKernels, kNumKernels);
    for (int k = 0; k < n; ++k) {
        if (ms) ms[k] = c->lastMs[k];
        if (names) names[k] = kKernelNames[k];
    }
    return n;
}

int psgpu_mesh_device(psgpu_ctx* c, PsMeshDevice* out) {
    if (!c || !out) return PSGPU_RET_PARAM_ERROR;
    int rc = psgpu_finish(c, nullptr);
    if (rc != PSGPU_RET_SUCCESS) return rc;
    out->pos = c->pos;
    out->nrm = c->nrm;
    out->col = c->col;
    out->tris = c->tris;
    out->mpuOffsets = c->offs;
    return PSGPU_RET_SUCCESS;
}

int psgpu_download_mesh(psgpu_ctx* c, float* pos, float* nrm, float* col, uint32_t* tris, uint64_t* mpuOffsets) {
    PsMeshInfo I;
    int rc = psgpu_finish(c, &I);
    if (rc != PSGPU_RET_SUCCESS) return rc;
    const size_t V = I.ctVertices, T = I.ctTriangles, N = I.ctMPUs;
    if (pos && V) PSGPU_CHECK(hipMemcpy(pos, c->pos, V * 12, hipMemcpyDeviceToHost));
    if (nrm && V) PSGPU_CHECK(hipMemcpy(nrm, c->nrm, V * 12, hipMemcpyDeviceToHost));
    if (col && V) PSGPU_CHECK(hipMemcpy(col, c->col, V * 12, hipMemcpyDeviceToHost));
    if (tris && T) PSGPU_CHECK(hipMemcpy(tris, c->tris, T * 12, hipMemcpyDeviceToHost));
    if (mpuOffsets) {
        if (N) PSGPU_CHECK(hipMemcpy(mpuOffsets, c->offs, (N + 1) * 8, hipMemcpyDeviceToHost));
        else mpuOffsets[0] = 0;
    }
    return PSGPU_RET_SUCCESS;
}

namespace {
// S1 survivors of the last run (global ids, ascending), from the per-MPU flags.
int survivors(psgpu_ctx* c, std::vector<uint32_t>& ids) {
    ids.clear();
    if (!c->mpuCount) return PSGPU_RET_SUCCESS;
    std::vector<uint8_t> passed(c->mpuCount);
    PSGPU_CHECK(hipMemcpy(passed.data(), c->passed, passed.size(), hipMemcpyDeviceToHost));
    for (uint32_t l = 0; l < c->mpuCount; ++l)
        if (passed[l]) ids.push_back(c->mpuBegin + l);
    return PSGPU_RET_SUCCESS;
}
}  // namespace

int psgpu_download_stats(psgpu_ctx* c, PsMpuStats* stats) {
    PsMeshInfo I;
    int rc = psgpu_finish(c, &I);
    if (rc != PSGPU_RET_SUCCESS || !stats) return rc == PSGPU_RET_SUCCESS ? PSGPU_RET_PARAM_ERROR : rc;
    std::vector<uint32_t> ids;
    rc = survivors(c, ids);
    if (rc != PSGPU_RET_SUCCESS) return rc;
    std::vector<uint64_t> cnt(c->mpuCount);
    if (c->mpuCount) PSGPU_CHECK(hipMemcpy(cnt.data(), c->counts, (size_t)c->mpuCount * 8, hipMemcpyDeviceToHost));
    memset(stats, 0, sizeof(PsMpuStats) * c->mpuCount);
    for (uint32_t m : ids) {
        PsMpuStats& s = stats[m - c->mpuBegin];
        s.passedPrecheck = 1;
        s.ctFieldEvals = 128;
    }
    for (uint32_t l = 0; l < c->mpuCount; ++l) {
        stats[l].ctVertices = (uint32_t)cnt[l];
        stats[l].ctTriangles = (uint32_t)(cnt[l] >> 32);
    }
    return PSGPU_RET_SUCCESS;
}
// MPUSTATS (PS_Polygonizer.h:201-207, written at .cpp:449-461): the per-MPU device ticks of
// the last run on the host's CLOCK_REALTIME nanosecond scale (legacy TBB's tick_count on
// Linux).  The device clock (s_memrealtime, wall-clock rate from the runtime) is mapped by
// bracketing one reading of it (k_clock_probe, stored straight into mapped host memory)
// between two host readings; of 8 tries the tightest bracket gives the offset, which is then
// good to half its width (a few microseconds; MPU ticks are tens of microseconds apart).
int psgpu_download_process_stats(psgpu_ctx* c, PsMpuProcessStats* out) {
    int rc = psgpu_finish(c, nullptr);
    if (rc != PSGPU_RET_SUCCESS) return rc;
    if (!out || !c->runTicks) return PSGPU_RET_PARAM_ERROR;
    const uint32_t n = c->mpuCount;
    if (!n) return PSGPU_RET_SUCCESS;
    std::vector<uint64_t> t((size_t)n * 4);
    PSGPU_CHECK(hipMemcpy(t.data(), c->mpuTicks, t.size() * 8, hipMemcpyDeviceToHost));
    int khz = 0;
    PSGPU_CHECK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, c->device));
    if (khz <= 0) return PSGPU_RET_DEVICE_ERROR;
    if (!c->clockProbe)
        PSGPU_CHECK(hipHostMalloc(reinterpret_cast<void**>(&c->clockProbe), 64,
                                  hipHostMallocMapped | hipHostMallocCoherent));
    uint64_t* dProbe = nullptr;
    PSGPU_CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&dProbe), c->clockProbe, 0));
    auto host_ns = [] {
        timespec ts;
        clock_gettime(CLOCK_REALTIME, &ts);
        return (int64_t)ts.tv_sec * 1000000000ll + (int64_t)ts.tv_nsec;
    };
    int64_t bestWidth = INT64_MAX, hostMid = 0;
    uint64_t devAt = 0;
    for (int k = 0; k < 8; ++k) {
        __atomic_store_n(c->clockProbe, 0ull, __ATOMIC_RELEASE);
        const int64_t h0 = host_ns();
        PSGPU_CHECK(launch_clock_probe(dProbe, c->stream));
        uint64_t d = 0;
        for (uint64_t spin = 0; (d = __atomic_load_n(c->clockProbe, __ATOMIC_ACQUIRE)) == 0ull; ++spin)
            if ((spin & 1023) == 1023 && hipStreamQuery(c->stream) != hipErrorNotReady) {
                d = __atomic_load_n(c->clockProbe, __ATOMIC_ACQUIRE);
                if (d == 0ull) return PSGPU_RET_DEVICE_ERROR;  // finished (or failed) without a reading
                break;
            }
        const int64_t h1 = host_ns();
        if (h1 - h0 < bestWidth) {
            bestWidth = h1 - h0;
            hostMid = h0 + (h1 - h0) / 2;
            devAt = d;
        }
    }
    PSGPU_CHECK(hipStreamSynchronize(c->stream));
    const double nsPerTick = 1.0e6 / (double)khz;
    auto to_ns = [&](uint64_t tick) { return hostMid + (int64_t)llround((double)((int64_t)(tick - devAt)) * nsPerTick); };
    for (uint32_t l = 0; l < n; ++l) {
        const uint64_t* r = &t[(size_t)4 * l];
        const bool s2 = r[2] != 0ull;
        out[l].threadID = s2 ? (r[3] >> 32) : (r[3] & 0xffffffffull);
        out[l].tickStart = to_ns(r[0]);
        out[l].tickEnd = to_ns(s2 ? r[2] : r[1]);
    }
    return PSGPU_RET_SUCCESS;
}

// Per-MPU work of the last run in lane-evaluations: 8 (S1) + 64 (field
// bounds of a survivor) or 512 (S2 cache of a queued survivor) + 8 per vertex (4 root
// samples, value and 3 normal samples).  Balances MPU ranges across devices.
int psgpu_mpu_costs(psgpu_ctx* c, uint32_t* costs) {
    PsMeshInfo I;
    int rc = psgpu_finish(c, &I);
    if (rc != PSGPU_RET_SUCCESS) return rc;
    if (!costs) return PSGPU_RET_PARAM_ERROR;
    const uint32_t n = c->mpuCount;
    if (!n) return PSGPU_RET_SUCCESS;
    std::vector<uint8_t> passed(n);
    std::vector<uint64_t> cnt(n);
    PSGPU_CHECK(hipMemcpy(passed.data(), c->passed, n, hipMemcpyDeviceToHost));
    PSGPU_CHECK(hipMemcpy(cnt.data(), c->counts, (size_t)n * 8, hipMemcpyDeviceToHost));
    for (uint32_t l = 0; l < n; ++l)
        costs[l] = 8u + (passed[l] == 1 ? 64u : 0u) + (passed[l] == 2 ? 512u : 0u) + 8u * (uint32_t)cnt[l];
    return PSGPU_RET_SUCCESS;
}

// Contiguous ranges of near-equal cost: bounds[k] = begin + the first index whose cost
// prefix reaches k/parts of the total (bounds[0] = begin, bounds[parts] = begin + n).
int psgpu_split_costs(const uint32_t* costs, uint32_t n, uint32_t parts, uint32_t begin, uint32_t* bounds) {
    if (!bounds || parts == 0 || (n && !costs)) return PSGPU_RET_PARAM_ERROR;
    uint64_t total = 0;
    for (uint32_t i = 0; i < n; ++i) total += costs[i];
    bounds[0] = begin;
    uint64_t acc = 0;
    uint32_t i = 0;
    for (uint32_t k = 1; k < parts; ++k) {
        const uint64_t target = (total * k + parts / 2) / parts;
        while (i < n && acc + costs[i] / 2 < target) acc += costs[i++];
        bounds[k] = begin + i;
    }
    bounds[parts] = begin + n;
    return PSGPU_RET_SUCCESS;
}

}  // extern "C"

namespace psgpu {
// The blocking export (Polygonize :360-371 into PolyMPUs, and the MPUSTATS of :372-376): one
// batch of async copies of the compact mesh, offsets, S1 flags and (for stats) counts into the
// context's pinned staging buffer (export_stage), one wait, then the host scatter
// (export_scatter).  Pageable destinations would cost a staged copy and a wait each (7 of
// them for a mesh plus statistics).  A group stages every part before it scatters the first,
// so the later parts' copies overlap the earlier parts' scatter.  Call after psgpu_finish.
int export_stage(psgpu_ctx* c, bool mesh, bool stats, ExportStage* st, hipEvent_t after) {
    const PsMeshInfo& I = c->info;
    ExportStage& S = *st;
    S.mesh = mesh;
    S.stats = stats;
    S.V = mesh ? I.ctVertices : 0;
    S.T = mesh ? I.ctTriangles : 0;
    S.N = c->mpuCount;
    auto up = [](size_t b) { return (b + 255) & ~(size_t)255; };
    const size_t N = S.N, V = S.V, T = S.T;
    // The per-piece flags sit at the front of the staging, at an offset no call moves: those
    // words only ever hold flags (an older call's epoch, or 0), never mesh or offset words, so
    // no stale word can equal this call's epoch (r04 kept them behind the mesh, where a call
    // with a smaller mesh found the previous call's packed triangles and offsets -- ADVICE r04)
    const size_t flagBytes = 4 * (size_t)kExportPieces * kExportPackBlocks * kExportFlagStride;
    S.oFlags = 0;
    S.oOffs = up(flagBytes);
    S.oPass = up(S.oOffs + (N + 1) * 8);
    S.oCnt = up(S.oPass + N);
    S.oMesh = up(S.oCnt + (stats ? N * 8 : 0));
    // the packed mesh: pack_words per piece; bounded by 4 extra words per piece
    S.meshBytes = mesh ? 4 * (pack_words(V, T) + 4 * kExportPieces) : 0;
    const size_t total = up(S.oMesh + S.meshBytes);
    if (total > c->hostStageCap) {
        if (c->hostStage) (void)hipHostFree(c->hostStage);
        c->hostStage = nullptr;
        c->hostStageCap = 0;
        const size_t cap = total + total / 4;
        // coherent: the export kernels write it directly over PCIe
        PSGPU_CHECK(hipHostMalloc(reinterpret_cast<void**>(&c->hostStage), cap,
                                  hipHostMallocMapped | hipHostMallocCoherent));
        c->hostStageCap = cap;
        memset(c->hostStage, 0, cap);  // no stale flag can equal an epoch
    }
    if (++c->exportEpoch == 0) {  // wrapped: clear every old flag
        memset(c->hostStage, 0, c->hostStageCap);
        c->exportEpoch = 1;
    }
    S.epoch = c->exportEpoch;
    unsigned char* h = c->hostStage;
    if (c->debug & (1 << 23)) {  // test hook: every word past the flags reads as this call's epoch
        // (the stream is idle: the previous export's scatter synchronised with it)
        uint32_t* w = reinterpret_cast<uint32_t*>(h + flagBytes);
        for (size_t i = 0, n = (c->hostStageCap - flagBytes) / 4; i < n; ++i) w[i] = S.epoch;
    }
    hipStream_t s = c->stream;
    for (hipEvent_t& e : c->exportEv)
        if (!e) PSGPU_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    unsigned char* hd = nullptr;  // the staging as the device addresses it
    PSGPU_CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&hd), h, 0));
    if (N) {
        MetaSrc ms{mesh ? c->offs : nullptr, c->passed, stats ? c->counts : nullptr, (uint32_t)N,
                   S.oOffs, S.oPass, S.oCnt};
        PSGPU_CHECK(launch_export_meta(ms, hd, s));
    }
    PSGPU_CHECK(hipEventRecord(c->exportEv[0], s));
    // the mesh packed piece by piece (MPU ranges of about 1 MB of mesh, at most 16: C3 0.535 vs
    // 0.570 ms with 2 MB) into one contiguous region by one kernel writing it over PCIe; the
    // host scatter of one piece overlaps the transfer of the next
    // 256 blocks: one wave per SIMD keeps the link busy; 1,024 or 2,048 were 1.8-4.5x slower,
    // every block's per-piece release (an L2 write-back) adding up (r04)
    S.packBlocks = kExportPackBlocks;
    S.pieces = (int)std::min<size_t>({(size_t)kExportPieces, std::max<size_t>(N, 1),
                                      1 + 4 * pack_words(V, T) / kExportPieceBytes});
    if (after) PSGPU_CHECK(hipStreamWaitEvent(s, after, 0));
    if (S.meshBytes && N) {
        PackSrc src{c->offs, c->pos, c->nrm, c->col, c->tris, (uint32_t)N, (uint32_t)S.pieces,
                    reinterpret_cast<uint32_t*>(hd + S.oFlags), S.epoch, S.packBlocks,
                    // test hook: the last block waits ~40 us before each piece's share
                    (c->debug & (1 << 24)) ? S.packBlocks - 1u : 0xffffffffu, 4000u};
        PSGPU_CHECK(launch_export_pack(src, reinterpret_cast<uint32_t*>(hd + S.oMesh), s));
    }
    PSGPU_CHECK(hipEventRecord(c->exportEv[1], s));
    return PSGPU_RET_SUCCESS;
}

int ScatterJob::prepare(psgpu_ctx* ctx, const ExportStage& st, PsMPU* out) {
    c = ctx;
    S = &st;
    mpus = out;
    PSGPU_CHECK(hipEventSynchronize(c->exportEv[0]));  // offsets, S1 flags, counts
    const unsigned char* h = c->hostStage;
    off = reinterpret_cast<const uint64_t*>(h + st.oOffs);
    passed = h + st.oPass;
    mesh = h + st.oMesh;
    flags = reinterpret_cast<const uint32_t*>(h + st.oFlags);
    side = c->cs * (float)PSGPU_CELLS_PER_MPU;
    active = out && st.mesh && !(c->debug & (1 << 22));  // bit 22: the transfers without the scatter
    if (!active) return PSGPU_RET_SUCCESS;
    // the pieces' MPU ranges and their places in the packed mesh (as k_export_pack laid them out)
    const size_t N = st.N;
    size_t base = 0;
    for (int k = 0; k <= st.pieces; ++k) pm[k] = (uint32_t)((uint64_t)N * (uint64_t)k / (uint64_t)st.pieces);
    for (int k = 0; k < st.pieces; ++k) {
        pv0[k] = (uint32_t)off[pm[k]];
        pt0[k] = (uint32_t)(off[pm[k]] >> 32);
        pnv[k] = (uint32_t)off[pm[k + 1]] - pv0[k];
        pbase[k] = base;
        base += 4 * pack_words(pnv[k], (uint32_t)(off[pm[k + 1]] >> 32) - pt0[k]);
    }
    return PSGPU_RET_SUCCESS;
}

// piece k is in when every block of k_export_pack has raised its flag for it; the kernel's
// event ends the wait should it fail.  One thread at a time reads the flags (they sit in
// memory the device writes over PCIe: sixteen threads polling them slowed the device's
// writes in some calls) and publishes the count of pieces in; the others watch that count.
bool ScatterJob::wait_piece(int k) {
    for (uint32_t spin = 1;; ++spin) {
        const int r = ready.load(std::memory_order_acquire);
        if (r > k) return true;
        if (r < 0) return false;  // the kernel failed
        bool idle = false;
        if (polling.compare_exchange_strong(idle, true, std::memory_order_acq_rel)) {
            int n = ready.load(std::memory_order_acquire);
            while (n >= 0 && n < S->pieces) {  // advance over every piece already in
                const uint32_t* f = flags + (size_t)n * S->packBlocks * kExportFlagStride;
                // from the first flag not yet seen up: every read of a flag still down is a read
                // of a line the device is about to write (one flag a line, kExportFlagStride)
                uint32_t b = pollBlock;
                while (b < S->packBlocks && __atomic_load_n(f + (size_t)b * kExportFlagStride, __ATOMIC_ACQUIRE) == S->epoch) ++b;
                pollBlock = b;
                if (b < S->packBlocks) {
                    if ((spin & 63) == 0) {
                        const hipError_t e = hipEventQuery(c->exportEv[1]);
                        if (e != hipErrorNotReady) {  // done (every flag must be up) or failed
                            while (b < S->packBlocks && __atomic_load_n(f + (size_t)b * kExportFlagStride, __ATOMIC_ACQUIRE) == S->epoch) ++b;
                            if (e != hipSuccess || b < S->packBlocks) n = -1;
                            else ++n;
                            pollBlock = 0;
                            ready.store(n, std::memory_order_release);
                            continue;
                        }
                    }
                    break;
                }
                if (trace) tPiece[n] = now_ns();
                pollBlock = 0;
                ready.store(++n, std::memory_order_release);
            }
            polling.store(false, std::memory_order_release);
            for (int i = 0; i < 256; ++i) __builtin_ia32_pause();  // ~1-2 us between reads of the flags
        }
        std::this_thread::yield();
    }
}

// MPUs [lb, le) into PolyMPUs (Polygonize :360-371); `have` = the pieces this thread has seen in
bool ScatterJob::range(uint32_t lb, uint32_t le, int* have) {
    int k = 0;
    while (k + 1 < S->pieces && lb >= pm[k + 1]) ++k;
    for (uint32_t l = lb; l < le; ++l) {
        while (k + 1 < S->pieces && l >= pm[k + 1]) ++k;
        const uint32_t v0 = (uint32_t)off[l], nv = (uint32_t)off[l + 1] - v0;
        const uint32_t t0 = (uint32_t)(off[l] >> 32), nt = (uint32_t)(off[l + 1] >> 32) - t0;
        const unsigned char* P = mesh + pbase[k];
        const float* pos = reinterpret_cast<const float*>(P) + 3 * (v0 - pv0[k]);
        const float* nrm = reinterpret_cast<const float*>(P + pnv[k] * 12) + 3 * (v0 - pv0[k]);
        const float* col = reinterpret_cast<const float*>(P + pnv[k] * 24) + 3 * (v0 - pv0[k]);
        const uint16_t* tri = reinterpret_cast<const uint16_t*>(P + pnv[k] * 36) + 3 * (t0 - pt0[k]);
        while (*have <= k) {  // this MPU's piece written (the pieces come in order)
            if (!wait_piece(*have)) return false;
            ++*have;
        }
        const uint32_t m = c->mpuBegin + l;
        const uint32_t kk = m % c->dims[2], j = (m / c->dims[2]) % c->dims[1], i = m / (c->dims[2] * c->dims[1]);
        PsMPU& M = mpus[l];
        M.bboxLo.x = c->primsHost.bboxLo.x + (float)i * side;
        M.bboxLo.y = c->primsHost.bboxLo.y + (float)j * side;
        M.bboxLo.z = c->primsHost.bboxLo.z + (float)kk * side;
        M.ctFieldEvals = passed[l] ? 128 : 0;
        M.ctVertices = (uint16_t)nv;
        M.ctTriangles = (uint16_t)nt;
        memcpy(M.vPos, pos, (size_t)nv * 12);
        memcpy(M.vNorm, nrm, (size_t)nv * 12);
        memcpy(M.vColor, col, (size_t)nv * 12);
        memcpy(M.triangles, tri, (size_t)nt * 6);
    }
    return true;
}

// thread k of nth: chunks of 128 MPUs dealt round robin (the surface lies in a few slabs of
// the range), in ascending order, so the pieces are waited for in the order they come
void ScatterJob::task(unsigned k, unsigned nth) {
    if (!active) return;
    if (trace) {
        int64_t z = 0;
        (void)tFirstTask.compare_exchange_strong(z, now_ns());
    }
    int have = 0;
    const uint32_t N = (uint32_t)S->N;
    for (uint32_t b = k * 128u; b < N; b += nth * 128u)
        if (!range(b, std::min<uint32_t>(N, b + 128u), &have)) {
            failed = true;
            return;
        }
}

int ScatterJob::finish(PsMpuStats* stats) {
    if (failed) return PSGPU_RET_DEVICE_ERROR;
    PSGPU_CHECK(hipStreamSynchronize(c->stream));  // the packing kernel done
    if (stats && S->stats) {
        const uint64_t* cnt = reinterpret_cast<const uint64_t*>(c->hostStage + S->oCnt);
        memset(stats, 0, sizeof(PsMpuStats) * S->N);
        for (uint32_t l = 0; l < S->N; ++l) {
            PsMpuStats& st = stats[l];
            if (passed[l]) {
                st.passedPrecheck = 1;
                st.ctFieldEvals = 128;
            }
            st.ctVertices = (uint32_t)(cnt[l] & 0xffffffffu);
            st.ctTriangles = (uint32_t)(cnt[l] >> 32);
        }
    }
    return PSGPU_RET_SUCCESS;
}

// The scatter is bound by the write-allocates of the sparse PolyMPUs layout (21.5 KB per MPU):
// several host threads, as the reference's TBB bodies fill it -- about one per 256 KB of mesh,
// at most 16 (C3 0.535 vs 0.586 ms with 8), kept in c's pool.  Runs jobs[0..n) in one pass: every thread takes its chunks of
// each job in turn.
int scatter_jobs(psgpu_ctx* c, ScatterJob* jobs, size_t n) {
    size_t bytes = 0;
    for (size_t j = 0; j < n; ++j) bytes += jobs[j].active ? jobs[j].S->meshBytes : 0;
    const unsigned nth = (unsigned)std::min<size_t>({16, std::max(1u, std::thread::hardware_concurrency()),
                                                    1 + bytes / (256 << 10)});
    std::function<void(unsigned)> task = [&](unsigned k) {
        for (size_t j = 0; j < n; ++j) jobs[j].task(k, nth);
    };
    // nth workers on the caller's NUMA node; the caller only waits
    if (nth > 1 && (!c->scatterPool || c->scatterPool->workers() < nth)) {
        c->scatterPool.reset();
        try {
            cpu_set_t node;
            const bool haveNode = ScatterPool::caller_node_cpus(&node);
            c->scatterPool.reset(new ScatterPool(nth, haveNode ? &node : nullptr));
        } catch (...) {  // no threads to be had: this caller scatters alone
            c->scatterPool.reset();
        }
    }
    if (nth > 1 && c->scatterPool) c->scatterPool->run(nth, task, false);
    else
        for (unsigned k = 0; k < nth; ++k) task(k);
    return PSGPU_RET_SUCCESS;
}

// PSGPU_EXPORT_TRACE=1: every blocking export prints its phases (ms from the call's start) to
// stderr -- kernels done, packing enqueued, metadata in, first scatter task, each piece in,
// scatter done, end (tools/blocking_seq.py collects them)
bool export_trace_on() {
    static const bool on = [] {
        const char* e = getenv("PSGPU_EXPORT_TRACE");
        return e && *e && *e != '0';
    }();
    return on;
}

int export_scatter(psgpu_ctx* c, const ExportStage& S, PsMPU* mpus, PsMpuStats* stats, const int64_t* tr) {
    ScatterJob job;
    job.trace = tr != nullptr;
    int rc = job.prepare(c, S, mpus);
    const int64_t tPrep = tr ? now_ns() : 0;
    if (rc == PSGPU_RET_SUCCESS) rc = scatter_jobs(c, &job, 1);
    const int64_t tScat = tr ? now_ns() : 0;
    if (rc == PSGPU_RET_SUCCESS) rc = job.finish(stats);
    if (tr) {
        const int64_t t0 = tr[0], tEnd = now_ns();
        auto ms = [t0](int64_t t) { return t ? (double)(t - t0) * 1e-6 : -1.0; };
        fprintf(stderr, "psgpu export: mpus %zu V %zu pieces %d | kernels %.3f packing %.3f meta %.3f first_task %.3f pieces",
                S.N, S.V, S.pieces, ms(tr[1]), ms(tr[2]), ms(tPrep), ms(job.tFirstTask.load()));
        for (int k = 0; k < S.pieces; ++k) fprintf(stderr, " %.3f", ms(job.tPiece[k]));
        fprintf(stderr, " | scatter %.3f end %.3f\n", ms(tScat), ms(tEnd));
    }
    return rc;
}
}  // namespace psgpu

namespace {
int export_blocking(psgpu_ctx* c, PsMPU* mpus, uint32_t capacity, uint32_t* outCt, PsMpuStats* stats,
                    int64_t tCall = 0) {
    int64_t tr[3] = {tCall ? tCall : now_ns(), 0, 0};
    const bool trace = export_trace_on();
    PsMeshInfo I;
    int rc = psgpu_finish(c, &I);
    if (rc != PSGPU_RET_SUCCESS) return rc;
    tr[1] = now_ns();
    if (outCt) *outCt = c->mpuCount;
    if (mpus) {
        if (c->mpuCount > capacity) return PSGPU_RET_MPU_OVERFLOW;
        if (I.firstOverflowMPU >= 0) return PSGPU_RET_MPU_VT_OVERFLOW;
    }
    if (!mpus && !stats) return PSGPU_RET_PARAM_ERROR;
    ExportStage st;
    rc = export_stage(c, mpus != nullptr, stats != nullptr, &st);
    if (rc != PSGPU_RET_SUCCESS) return rc;
    tr[2] = now_ns();
    return export_scatter(c, st, mpus, stats, trace ? tr : nullptr);
}
}  // namespace

extern "C" {

int psgpu_export_polympus(psgpu_ctx* c, PsMPU* mpus, uint32_t capacity, uint32_t* outCt) {
    if (!mpus) {  // the count (and overflow) check alone
        PsMeshInfo I;
        int rc = psgpu_finish(c, &I);
        if (rc != PSGPU_RET_SUCCESS) return rc;
        if (outCt) *outCt = c->mpuCount;
        if (c->mpuCount > capacity) return PSGPU_RET_MPU_OVERFLOW;
        if (I.firstOverflowMPU >= 0) return PSGPU_RET_MPU_VT_OVERFLOW;
        return PSGPU_RET_PARAM_ERROR;
    }
    return export_blocking(c, mpus, capacity, outCt, nullptr);
}

int psgpu_polygonize_mpus(psgpu_ctx* c, float cellsize, const PsSoaBlobPrims* prims, const PsSoaPrimMatrices* mats,
                          const PsSoaBlobOps* ops, PsMPU* mpus, uint32_t capacity, uint32_t* outCt,
                          PsMpuStats* stats) {
    if (!c || !prims) return PSGPU_RET_PARAM_ERROR;
    if (prims->ctPrims == 0) return PSGPU_RET_PARAM_ERROR;  // Polygonize :322-323
    const int64_t tCall = now_ns();
    int rc = psgpu_set_model(c, prims, mats, ops);
    if (rc != PSGPU_RET_SUCCESS) return rc;
    rc = psgpu_polygonize(c, cellsize, 0, 0xffffffffu, nullptr);
    if (rc != PSGPU_RET_SUCCESS) return rc;
    if (!mpus) {  // the reference's own errors first (count, overflow), then the null
        rc = psgpu_export_polympus(c, nullptr, capacity, outCt);
        return rc;
    }
    return export_blocking(c, mpus, capacity, outCt, stats, tCall);
}

int psgpu_polygonize_mpus_ex(psgpu_ctx* c, float cellsize, const PsSoaBlobPrims* prims, const PsSoaPrimMatrices* mats,
                             const PsSoaBlobOps* ops, PsMPU* mpus, uint32_t capacity, uint32_t* outCt,
                             PsMpuStats* stats, PsMpuProcessStats* processStats) {
    if (!c) return PSGPU_RET_PARAM_ERROR;
    if (!processStats) return psgpu_polygonize_mpus(c, cellsize, prims, mats, ops, mpus, capacity, outCt, stats);
    const int was = c->mpuTicksOpt;
    c->mpuTicksOpt = 1;  // this call's run records the ticks (Polygonize :379 hands lpProcessStats on)
    int rc = psgpu_polygonize_mpus(c, cellsize, prims, mats, ops, mpus, capacity, outCt, stats);
    c->mpuTicksOpt = was;
    // ctMPUs entries, as PolyMPUs: only on success (on -4 the caller's array may be shorter)
    if (rc == PSGPU_RET_SUCCESS) rc = psgpu_download_process_stats(c, processStats);
    return rc;
}

// Field probe (FieldComputer::fieldValue / fieldValueAndColor on arbitrary points).
// mode 0: 4-lane groups (consecutive points), 1: per point, 2: per point + colour.
int psgpu_field_values(psgpu_ctx* c, const float* xyz, uint32_t n, int mode, float* out, float* colOut) {
    if (!c || !c->haveModel || !xyz || !out || mode < 0 || mode > 2) return PSGPU_RET_PARAM_ERROR;
    int rc = set_device(c);
    if (rc != PSGPU_RET_SUCCESS) return rc;
    jit_poll(c, false);
    if (n == 0) return PSGPU_RET_SUCCESS;
    float *dx = nullptr, *dout = nullptr, *dcol = nullptr;
    PSGPU_CHECK(hipMalloc(&dx, (size_t)n * 12));
    PSGPU_CHECK(hipMalloc(&dout, (size_t)n * 4));
    PSGPU_CHECK(hipMalloc(&dcol, (size_t)n * 12));
    PSGPU_CHECK(hipMemcpy(dx, xyz, (size_t)n * 12, hipMemcpyHostToDevice));
    Params p = make_params(c);
    hipError_t e;
    if (c->jit) {
        void* args[] = {&p, &dx, &dout, &dcol, &n, &mode};
        e = hipModuleLaunchKernel(c->jit->probe, (n + 255) / 256, 1, 1, 256, 1, 1, 0, c->stream, args, nullptr);
    } else {
        e = launch_probe(p, c->stream, dx, dout, dcol, n, mode);
    }
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e == hipSuccess) e = hipMemcpy(out, dout, (size_t)n * 4, hipMemcpyDeviceToHost);
    if (e == hipSuccess && colOut) e = hipMemcpy(colOut, dcol, (size_t)n * 12, hipMemcpyDeviceToHost);
    (void)hipFree(dx);
    (void)hipFree(dout);
    (void)hipFree(dcol);
    return hip_fail(e, "psgpu_field_values");
}

// Host-only: build the device image of a model and compile its specialised kernels
// (no GPU needed).  Returns the code-object size, or a negative error code.
long psgpu_jit_compile(const PsSoaBlobPrims* prims, const PsSoaPrimMatrices* mats, const PsSoaBlobOps* ops,
                       int mode, char* log, size_t cap) {
    if (!prims || !mats || !ops) return PSGPU_RET_PARAM_ERROR;
    std::unique_ptr<DevModel> m(new DevModel);
    int rc = build_device_model(*prims, *mats, *ops, *m);
    if (rc != PSGPU_RET_SUCCESS) return rc;
    std::string err;
    long n = jit_compile_only(*m, (mode & 3) == 2, &err, (mode & 4) != 0);
    if (log && cap) {
        const size_t k = std::min(cap - 1, err.size());
        memcpy(log, err.data(), k);
        log[k] = 0;
    }
    return n < 0 ? PSGPU_RET_DEVICE_ERROR : n;
}

// Whether the current model runs on run-time specialised kernels (1) or the interpreter (0).
int psgpu_jit_active(psgpu_ctx* c) {
    if (!c) return 0;
    if (c->jitPending && set_device(c) == PSGPU_RET_SUCCESS) jit_poll(c, false);
    return c->jit ? 1 : 0;
}

int psgpu_jit_pending(psgpu_ctx* c) {
    if (!c) return 0;
    if (c->jitPending && set_device(c) == PSGPU_RET_SUCCESS) jit_poll(c, false);
    return c->jitPending ? 1 : 0;
}

int psgpu_jit_wait(psgpu_ctx* c) {
    if (!c) return 0;
    if ((c->jitPending || c->tier2Pending) && set_device(c) == PSGPU_RET_SUCCESS) {
        jit_poll(c, true);
        tier_poll(c, true);
    }
    return c->jit ? 1 : 0;
}

int psgpu_jit_tier(psgpu_ctx* c) {
    if (!c) return 0;
    if ((c->jitPending || c->tier2Pending) && set_device(c) == PSGPU_RET_SUCCESS) {
        jit_poll(c, false);
        tier_poll(c, false);
    }
    return c->tier;
}

// Generated specialised source for the current model (NUL-terminated, truncated to cap).
int psgpu_jit_source(psgpu_ctx* c, char* buf, size_t cap) {
    if (!c || !c->haveModel) return PSGPU_RET_PARAM_ERROR;
    const std::string s = jit_source(c->model, c->tier == 2 || c->useJit == 2, c->treeSplit != 0);
    if (buf && cap) {
        const size_t n = std::min(cap - 1, s.size());
        memcpy(buf, s.data(), n);
        buf[n] = 0;
    }
    return (int)s.size();
}

}  // extern "C"

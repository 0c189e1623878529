// Compat mode: ParsipHaptics' own polygonizer (CParsipOptimized over a COMPACTBLOBTREE,
// the GUI path) on gfx950.  C-ABI: include/parsip_gpu_gui.h.
//
// Reference: ParsipHaptics/include/CPolyParsipOptimized.cpp (setup :330-390, run
// :392-410, doMarchingCubes :130-327) and CompactBlobTree.cpp (fieldvalueOp/Prim
// :677-1092, baseColorOp :1124-1294, normal :433-450, ComputeRootNewtonRaphsonVEC4
// :1581-1622).  The CPU restatement that checks it is oracle/psgui.c.
//
// One polygonization = 5 kernels on the context's stream (+ one count read-back):
//   k_gui_classify  one wavefront per MPU: the octree test against every primitive (:164-183),
//                   the 8^3 field cache (lane = (y, z), one 8-point walk along x), configs with
//                   `f > iso`, per-MPU counts of new vertices / triangles / crossed cells;
//   k_gui_scan      one block: the MPU offsets (exclusive scan in lattice order);
//   k_gui_edges     one wavefront per MPU with a surface: vertex ids in the reference's
//                   creation order (the first cell in loop order that holds an edge, then
//                   the candidate order of its table row: every cell around a crossing
//                   edge lists it, so that cell is fixed by the edge's position) as a
//                   vertex task list, and the triangles per cell;
//   k_gui_vertices  one mesh vertex per lane over the whole lattice: Newton root, normal,
//                   colour (no MPU's vertex count sets a wave's length);
//   k_gui_totals    one block: CParsipOptimized's statistics.
// The tree walk is an interpreter over the compact arrays with a per-lane frame stack
// (n-ary operators fold their kids as they arrive), bit-exact with the oracle:
// -ffp-contract=off, IEEE division / sqrt, powf / cos / sin correctly rounded through
// double precision on both sides.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../include/parsip_gpu_gui.h"

namespace psgui {

constexpr int kG = PSGUI_GRID_DIM;       // corners per MPU edge
constexpr int kC = kG - 1;               // cells per MPU edge
constexpr int kCells = kC * kC * kC;     // 343
constexpr int kCorners = kG * kG * kG;   // 512
constexpr int kEdges = 3 * kC * kG * kG; // 1344
constexpr int kCellsPerLane = (kCells + 63) / 64;
constexpr float kFieldEps = 0.001f;      // FIELD_VALUE_EPSILON
constexpr float kNormalDelta = 0.001f;   // NORMAL_DELTA
constexpr float kEps = 0.0001f;          // mathHelper.h EPSILON (FLOAT_EQ)

struct Tree {
    const PsGuiPrim* __restrict__ P;
    const PsGuiOp* __restrict__ O;
    const uint32_t* __restrict__ K;
    const PsGuiMatrix* __restrict__ M;
    uint32_t nP, nO;
};

// Per (config, candidate position): edge | first-occurrence << 4 | valid << 5; per config
// the triangle count.  Built on the host from the MC table.
struct Tables {
    uint8_t cand[256][16];
    uint8_t ntri[256];
};

struct Params {
    Tree T;
    const Tables* tables;
    float lo[3];
    uint32_t dims[3];
    uint32_t n;          // lattice MPUs
    float cs, side, iso;
    float* fvc;          // n x 512 field cache
    uint64_t* counts;    // V | T << 32 per MPU
    uint64_t* offs;      // n + 1
    PsGuiMpuStats* stats;
    float* pos;
    float* nrm;
    float* col;
    uint32_t* tris;
    uint64_t* vtask;     // per mesh vertex: MPU | edge index << 32 (k_gui_edges -> k_gui_vertices)
    uint32_t nV;         // mesh vertices of the run
    PsGuiInfo* totals;
};

__device__ __forceinline__ float cr_pow(float x, float y) { return (float)pow((double)x, (double)y); }
__device__ __forceinline__ float cr_cos(float x) { return (float)cos((double)x); }
__device__ __forceinline__ float cr_sin(float x) { return (float)sin((double)x); }
__device__ __forceinline__ bool float_eq(float x, float v) { return ((v - kEps) < x) && (x < (v + kEps)); }
__device__ __forceinline__ float maxf(float a, float b) { return (a > b) ? a : b; }
__device__ __forceinline__ float absf(float n) { return n < 0 ? (0 - n) : n; }

struct V3 { float x, y, z; };
struct V4 { float x, y, z, w; };
__device__ __forceinline__ V3 sub(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ V3 add(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ V3 scale(V3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
__device__ __forceinline__ float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ float len2(V3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
__device__ __forceinline__ float dist2(V3 self, V3 a) {
    const float dx = a.x - self.x, dy = a.y - self.y, dz = a.z - self.z;
    return dx * dx + dy * dy + dz * dz;
}
__device__ __forceinline__ void normalize(V3& a) {
    const float d = sqrtf(a.x * a.x + a.y * a.y + a.z * a.z);
    if (d > 0) {
        const float r = 1.0f / d;
        a.x *= r; a.y *= r; a.z *= r;
    } else {
        a.x = a.y = a.z = 1;
    }
}
__device__ __forceinline__ V3 xyz(const float* f) { return {f[0], f[1], f[2]}; }
__device__ __forceinline__ float dot4(const float* r, V4 p) { return r[0] * p.x + r[1] * p.y + r[2] * p.z + r[3] * p.w; }

__device__ __forceinline__ float wyvill(float dd) {  // CFieldFunction.h:104-114
    if (dd >= 1.0f) return 0.0f;
    const float t = (1.0f - dd);
    return t * t * t;
}

__device__ float triangle_sqr_dist(V3 v0, V3 v1, V3 v2, V3 p) {  // CSkeletonTriangle.cpp:19-254
    const V3 dif = sub(v0, p), e0 = sub(v1, v0), e1 = sub(v2, v0);
    const float a00 = len2(e0), a01 = dot(e0, e1), a11 = len2(e1);
    const float b0 = dot(dif, e0), b1 = dot(dif, e1), c = len2(dif);
    const float det = absf(a00 * a11 - a01 * a01);
    float s = a01 * b1 - a11 * b0;
    float t = a01 * b0 - a00 * b1;
    float sq;
    if (s + t <= det) {
        if (s < 0.0f) {
            if (t < 0.0f) {
                if (b0 < 0.0f) {
                    if (-b0 >= a00) sq = a00 + 2.0f * b0 + c;
                    else { s = -b0 / a00; sq = b0 * s + c; }
                } else {
                    if (b1 >= 0.0f) sq = c;
                    else if (-b1 >= a11) sq = a11 + 2.0f * b1 + c;
                    else { t = -b1 / a11; sq = b1 * t + c; }
                }
            } else {
                if (b1 >= 0.0f) sq = c;
                else if (-b1 >= a11) sq = a11 + 2.0f * b1 + c;
                else { t = -b1 / a11; sq = b1 * t + c; }
            }
        } else if (t < 0.0f) {
            if (b0 >= 0.0f) sq = c;
            else if (-b0 >= a00) sq = a00 + 2.0f * b0 + c;
            else { s = -b0 / a00; sq = b0 * s + c; }
        } else {
            const float invDet = 1.0f / det;
            s *= invDet;
            t *= invDet;
            sq = s * (a00 * s + a01 * t + 2.0f * b0) + t * (a01 * s + a11 * t + 2.0f * b1) + c;
        }
    } else {
        float tmp0, tmp1, numer, denom;
        if (s < 0.0f) {
            tmp0 = a01 + b0;
            tmp1 = a11 + b1;
            if (tmp1 > tmp0) {
                numer = tmp1 - tmp0;
                denom = a00 - 2.0f * a01 + a11;
                if (numer >= denom) sq = a00 + 2.0f * b0 + c;
                else {
                    s = numer / denom;
                    t = 1.0f - s;
                    sq = s * (a00 * s + a01 * t + 2.0f * b0) + t * (a01 * s + a11 * t + 2.0f * b1) + c;
                }
            } else {
                if (tmp1 <= 0.0f) sq = a11 + 2.0f * b1 + c;
                else if (b1 >= 0.0f) sq = c;
                else { t = -b1 / a11; sq = b1 * t + c; }
            }
        } else if (t < 0.0f) {
            tmp0 = a01 + b1;
            tmp1 = a00 + b0;
            if (tmp1 > tmp0) {
                numer = tmp1 - tmp0;
                denom = a00 - 2.0f * a01 + a11;
                if (numer >= denom) sq = a11 + 2.0f * b1 + c;
                else {
                    t = numer / denom;
                    s = 1.0f - t;
                    sq = s * (a00 * s + a01 * t + 2.0f * b0) + t * (a01 * s + a11 * t + 2.0f * b1) + c;
                }
            } else {
                if (tmp1 <= 0.0f) sq = a00 + 2.0f * b0 + c;
                else if (b0 >= 0.0f) sq = c;
                else { s = -b0 / a00; sq = b0 * s + c; }
            }
        } else {
            numer = a11 + b1 - a01 - b0;
            if (numer <= 0.0f) sq = a11 + 2.0f * b1 + c;
            else {
                denom = a00 - 2.0f * a01 + a11;
                if (numer >= denom) sq = a00 + 2.0f * b0 + c;
                else {
                    s = numer / denom;
                    t = 1.0f - s;
                    sq = s * (a00 * s + a01 * t + 2.0f * b0) + t * (a01 * s + a11 * t + 2.0f * b1) + c;
                }
            }
        }
    }
    if (sq < 0.0f) sq = 0.0f;
    return sq;
}

// COMPACTBLOBTREE::fieldvaluePrim (CompactBlobTree.cpp:893-1092)
__device__ float prim_field(const Tree& T, uint32_t id, V4 p) {
    const PsGuiPrim& P = T.P[id];
    V3 pn = {p.x, p.y, p.z};
    if (P.idxMtx != 0) {
        const PsGuiMatrix& m = T.M[P.idxMtx];
        const V4 pp = {p.x, p.y, p.z, 1.0f};
        pn.x = dot4(m.r[0], pp);
        pn.y = dot4(m.r[1], pp);
        pn.z = dot4(m.r[2], pp);
    }
    switch (P.type) {
    case PSGUI_PRIM_POINT:
        return wyvill(dist2(pn, xyz(P.pos)));
    case PSGUI_PRIM_CYLINDER: {
        const V3 pos = sub(pn, xyz(P.pos));
        float y = dot(pos, xyz(P.dir));
        const float x = maxf(0.0f, sqrtf(len2(pos) - y * y) - P.res1[0]);
        if (y > 0.0f) y = maxf(0.0f, y - P.res2[0]);
        return wyvill(x * x + y * y);
    }
    case PSGUI_PRIM_TRIANGLE:
        return wyvill(triangle_sqr_dist(xyz(P.pos), xyz(P.res1), xyz(P.res2), pn));
    case PSGUI_PRIM_CUBE: {
        const V3 dif = sub(pn, xyz(P.pos));
        const float side = P.res1[0];
        float d2 = 0.0f;
        const float pr[3] = {dif.x * 1.0f + dif.y * 0.0f + dif.z * 0.0f, dif.x * 0.0f + dif.y * 1.0f + dif.z * 0.0f,
                             dif.x * 0.0f + dif.y * 0.0f + dif.z * 1.0f};
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            if (pr[a] < -1.0f * side) {
                const float d = pr[a] + side;
                d2 += d * d;
            } else if (pr[a] > side) {
                const float d = pr[a] - side;
                d2 += d * d;
            }
        }
        return wyvill(d2);
    }
    case PSGUI_PRIM_DISC:
    case PSGUI_PRIM_RING: {
        const V3 n = xyz(P.dir), c = xyz(P.pos);
        const float r = P.res1[0];
        const V3 pc = sub(pn, c);
        V3 dir = sub(pc, scale(n, dot(n, pc)));
        float dd;
        if (P.type == PSGUI_PRIM_DISC ? (sqrtf(len2(dir)) <= r) : false) {
            dd = absf(len2(pc) - len2(dir));
        } else if (P.type == PSGUI_PRIM_RING && float_eq(0.0f, len2(dir))) {
            dd = r * r + len2(pc);
        } else {
            normalize(dir);
            const V3 x = add(c, scale(dir, r));
            dd = len2(sub(x, pn));
        }
        return wyvill(dd);
    }
    case PSGUI_PRIM_LINE: {
        const V3 s = xyz(P.res1), e = xyz(P.res2);
        const V3 d = sub(e, s);
        V3 np = s;
        if (!(float_eq(0.0f, d.x) && float_eq(0.0f, d.y) && float_eq(0.0f, d.z))) {
            float delta = dot(sub(pn, s), d) / dot(d, d);
            if (delta < 0) delta = 0;
            else if (delta > 1) delta = 1;
            np = add(s, scale(d, delta));
        }
        return wyvill(dist2(np, pn));
    }
    case PSGUI_PRIM_QUADRICPOINT: {
        const float d2 = len2(sub(pn, xyz(P.pos)));
        const float R = P.res1[0];
        const float f = (1.0f - (d2 / (R * R)));
        return (f <= 0.0f) ? 0.0f : P.res2[0] * f * f;
    }
    default:
        return 0.0f;
    }
}

// The point an operator hands its kids: backward matrix (w -> 1), then the warp
// (CompactBlobTree.cpp:685-746, warps :1315-1536; a warped point is a fresh vec4f, w = 0).
__device__ V4 op_point(const Tree& T, const PsGuiOp& O, V4 p) {
    V4 q = p;
    if (O.idxMtx != 0) {
        const PsGuiMatrix& m = T.M[O.idxMtx];
        q = {dot4(m.r[0], p), dot4(m.r[1], p), dot4(m.r[2], p), 1.0f};
    }
    const float* prm = O.params;
    switch (O.type) {
    case PSGUI_OP_WARPBEND: {
        const float k = prm[0], y0 = prm[1], left = prm[2], right = prm[3];
        V4 out = {q.x, 0.0f, 0.0f, 0.0f};
        const float kDiv = 1.0f / k;
        float yh = 0.0f;
        if (q.y <= left) yh = left;
        else if ((q.y > left) && (q.y < right)) yh = q.y;
        else if (q.y >= right) yh = right;
        const float theta = k * (yh - y0);
        const float ct = cr_cos(theta), st = cr_sin(theta);
        const bool inside = (q.y >= left) && (q.y <= right);
        if (inside) out.y = -st * (q.z - kDiv) + y0;
        else if (q.y < left) out.y = -st * (q.z - kDiv) + y0 + ct * (q.y - left);
        else if (q.y > right) out.y = -st * (q.z - kDiv) + y0 + ct * (q.y - right);
        if (inside) out.z = ct * (q.z - kDiv) + kDiv;
        else if (q.y < left) out.z = ct * (q.z - kDiv) + kDiv + st * (q.y - left);
        else if (q.y > right) out.z = ct * (q.z - kDiv) + kDiv + st * (q.y - right);
        return out;
    }
    case PSGUI_OP_WARPTWIST: {
        const int axis = (int)prm[1];
        V4 out = {0.0f, 0.0f, 0.0f, 0.0f};
        if (axis == 0) {
            const float th = q.x * prm[0];
            out = {q.x, q.y * cr_cos(th) - q.z * cr_sin(th), q.y * cr_sin(th) + q.z * cr_cos(th), 0.0f};
        } else if (axis == 1) {
            const float th = q.y * prm[0];
            out = {q.x * cr_cos(th) - q.z * cr_sin(th), q.y, q.x * cr_sin(th) + q.z * cr_cos(th), 0.0f};
        } else if (axis == 2) {
            const float th = q.z * prm[0];
            out = {q.x * cr_cos(th) - q.y * cr_sin(th), q.x * cr_sin(th) + q.y * cr_cos(th), q.z, 0.0f};
        }
        return out;
    }
    case PSGUI_OP_WARPTAPER: {
        const float f = prm[0];
        const int along = (int)prm[1], taper = (int)prm[2];
        V4 out = {q.x, q.y, q.z, 0.0f};
        if (along == 0) {
            if (taper == 2) out.z = q.z * (1 + q.x * f);
            else out.y = q.y * (1 + q.x * f);
        } else if (along == 1) {
            if (taper == 2) out.z = q.z * (1 + q.y * f);
            else out.x = q.x * (1 + q.y * f);
        } else if (along == 2) {
            if (taper == 2) out.y = q.y * (1 + q.z * f);
            else out.x = q.x * (1 + q.z * f);
        }
        return out;
    }
    case PSGUI_OP_WARPSHEAR: {
        const float f = prm[0];
        const int along = (int)prm[1], dep = (int)prm[2];
        V4 out = {q.x, q.y, q.z, 0.0f};
        if (along == 1) out.y = (dep == 2) ? q.y + f * q.z : q.y + f * q.x;
        else if (along == 2) out.z = (dep == 1) ? q.z + f * q.y : q.z + f * q.x;
        else out.x = (dep == 2) ? q.x + f * q.z : q.x + f * q.y;
        return out;
    }
    default:
        return q;
    }
}

// One operator being folded: its kids arrive in order (fieldvalueOp :749-884 and, with
// COLOR, baseColorOp over the same walk's values :1124-1294).
struct Frame {
    V4 p;
    uint32_t op, next;
    float res, aux;   // field; colour selector (Union/Intersect/Dif) or weight sum (Blend/Ricci)
    float c[4];       // colour: selected or weighted sum
    float c0[4];      // first kid's colour (Blend/Ricci with a zero weight sum)
};

template <bool COLOR>
__device__ __forceinline__ void fold(const PsGuiOp& O, Frame& F, uint32_t i, float v, const float* c) {
    const int t = O.type;
    if (t == PSGUI_OP_BLEND || t == PSGUI_OP_RICCIBLEND) {
        F.res += (t == PSGUI_OP_BLEND) ? v : cr_pow(v, O.params[0]);
        if (COLOR) {
            F.c[0] += c[0] * v; F.c[1] += c[1] * v; F.c[2] += c[2] * v; F.c[3] += c[3] * v;
            F.aux += v;
            if (i == 0) { F.c0[0] = c[0]; F.c0[1] = c[1]; F.c0[2] = c[2]; F.c0[3] = c[3]; }
        }
        return;
    }
    if (i == 0) {
        F.res = v;
        if (COLOR) { F.aux = v; F.c[0] = c[0]; F.c[1] = c[1]; F.c[2] = c[2]; F.c[3] = c[3]; }
        return;
    }
    bool pick = false;
    switch (t) {
    case PSGUI_OP_UNION:
        if (v > F.res) F.res = v;
        if (COLOR && v > F.aux) { F.aux = v; pick = true; }
        break;
    case PSGUI_OP_INTERSECT:
        if (v < F.res) F.res = v;
        if (COLOR && v < F.aux) { F.aux = v; pick = true; }
        break;
    case PSGUI_OP_DIF:
    case PSGUI_OP_SMOOTHDIF: {
        const float cur = 1.0f - v;
        F.res = (t == PSGUI_OP_DIF) ? ((F.res < cur) ? F.res : cur) : F.res * cur;
        if (COLOR && cur < F.aux) { F.aux = cur; pick = true; }
    } break;
    default:  // warps: the first kid
        break;
    }
    if (COLOR && pick) { F.c[0] = c[0]; F.c[1] = c[1]; F.c[2] = c[2]; F.c[3] = c[3]; }
}

template <bool COLOR>
__device__ __forceinline__ float finalize(const PsGuiOp& O, Frame& F) {
    if (O.type == PSGUI_OP_RICCIBLEND) F.res = cr_pow(F.res, O.params[1]);
    if (COLOR && (O.type == PSGUI_OP_BLEND || O.type == PSGUI_OP_RICCIBLEND)) {
        if (F.aux == 0.0f) {
            F.c[0] = F.c0[0]; F.c[1] = F.c0[1]; F.c[2] = F.c0[2]; F.c[3] = F.c0[3];
        } else {
            const float r = 1.0f / F.aux;
            F.c[0] *= r; F.c[1] *= r; F.c[2] *= r; F.c[3] *= r;
        }
    }
    return F.res;
}

__device__ __forceinline__ void init_frame(const Tree& T, Frame& F, uint32_t op, V4 parentPoint) {
    F.p = op_point(T, T.O[op], parentPoint);
    F.op = op;
    F.next = 0;
    F.res = 0.0f;
    F.aux = 0.0f;
    F.c[0] = F.c[1] = F.c[2] = F.c[3] = 0.0f;
    F.c0[0] = F.c0[1] = F.c0[2] = F.c0[3] = 0.0f;
}

// COMPACTBLOBTREE::fieldvalue (:476-487) and, with COLOR, baseColor (:1095-1106) over the
// values of the same walk.
template <bool COLOR>
__device__ float field(const Tree& T, float x, float y, float z, float* colOut) {
    const V4 p = {x, y, z, 0.0f};
    if (T.nO == 0) {
        if (COLOR && T.nP) { colOut[0] = T.P[0].color[0]; colOut[1] = T.P[0].color[1]; colOut[2] = T.P[0].color[2]; colOut[3] = T.P[0].color[3]; }
        return T.nP ? prim_field(T, 0, p) : 0.0f;
    }
    Frame st[PSGUI_MAX_DEPTH];
    int sp = 0;
    init_frame(T, st[0], 0, p);
    for (;;) {
        Frame& F = st[sp];
        const PsGuiOp& O = T.O[F.op];
        if (F.next < (uint32_t)O.ctKids) {
            const uint32_t k = T.K[O.kidStart + F.next];
            const uint32_t i = F.next++;
            const uint32_t id = k & 0xffffu;
            if (k >> 16) {
                init_frame(T, st[++sp], id, F.p);
            } else {
                const float v = prim_field(T, id, F.p);
                fold<COLOR>(O, F, i, v, T.P[id].color);
            }
            continue;
        }
        const float v = finalize<COLOR>(O, F);
        if (sp == 0) {
            if (COLOR) { colOut[0] = F.c[0]; colOut[1] = F.c[1]; colOut[2] = F.c[2]; colOut[3] = F.c[3]; }
            return v;
        }
        Frame& Pf = st[--sp];
        fold<COLOR>(T.O[Pf.op], Pf, Pf.next - 1, v, F.c);
    }
}

__device__ __forceinline__ float wave_sum_f(float v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
__device__ __forceinline__ uint32_t wave_sum_u(uint32_t v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v) {
    const int lane = threadIdx.x & 63;
    uint32_t x = v;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    return x - v;
}

__device__ __forceinline__ void mpu_origin(const Params& p, uint32_t m, float o[3]) {
    const uint32_t k = m % p.dims[2], j = (m / p.dims[2]) % p.dims[1], i = m / (p.dims[2] * p.dims[1]);
    o[0] = p.lo[0] + (float)i * p.side;  // oct.lower + side * vec3f(i, j, k) (:378)
    o[1] = p.lo[1] + (float)j * p.side;
    o[2] = p.lo[2] + (float)k * p.side;
}

// corner index c = (i * 8 + j) * 8 + k; cell index = (i * 7 + j) * 7 + k (the loop order)
__device__ __forceinline__ int corner_of(int i, int j, int k) { return (i * kG + j) * kG + k; }

__device__ __forceinline__ uint32_t cell_config(const float* fv, int cell, float iso) {
    const int i = cell / (kC * kC), j = (cell / kC) % kC, k = cell % kC;
    uint32_t cfg = 0;
#pragma unroll
    for (int c = 0; c < 8; ++c)
        cfg |= (fv[corner_of(i + ((c >> 2) & 1), j + ((c >> 1) & 1), k + (c & 1))] > iso ? 1u : 0u) << c;
    return cfg;
}

// Edge e of a cell: lower corner offsets and axis (corner1/corner2, CCubeTable.h:43-44).
__constant__ int kCorner1[12] = {0, 2, 0, 1, 4, 6, 4, 5, 0, 1, 2, 3};
__constant__ int kAxisOf[12] = {2, 2, 1, 1, 2, 2, 1, 1, 0, 0, 0, 0};  // corner2 - corner1: 1 z, 2 y, 4 x

// The MPU-wide index of a cell's edge e, and whether this cell is the first (in loop order)
// of the cells that hold it: along each of the two other axes the edge's lower side is the
// owner unless the edge lies on the MPU's lower face.
__device__ __forceinline__ int edge_index(int i, int j, int k, int e, bool* owner) {
    const int c1 = kCorner1[e], a = kAxisOf[e];
    const int di = (c1 >> 2) & 1, dj = (c1 >> 1) & 1, dk = c1 & 1;
    const int ci = i + di, cj = j + dj, ck = k + dk;
    const bool oi = di == 1 || i == 0, oj = dj == 1 || j == 0, ok = dk == 1 || k == 0;
    if (a == 0) {
        *owner = oj && ok;
        return (ci * kG + cj) * kG + ck;
    }
    if (a == 1) {
        *owner = oi && ok;
        return kC * kG * kG + (ci * kC + cj) * kG + ck;
    }
    *owner = oi && oj;
    return 2 * kC * kG * kG + (ci * kG + cj) * kC + ck;
}

__device__ __forceinline__ void edge_corners(int idx, int c[2][3]) {
    int a, ci, cj, ck;
    if (idx < kC * kG * kG) {
        a = 0; ci = idx / (kG * kG); cj = (idx / kG) % kG; ck = idx % kG;
    } else if (idx < 2 * kC * kG * kG) {
        idx -= kC * kG * kG;
        a = 1; ci = idx / (kC * kG); cj = (idx / kG) % kC; ck = idx % kG;
    } else {
        idx -= 2 * kC * kG * kG;
        a = 2; ci = idx / (kG * kC); cj = (idx / kC) % kG; ck = idx % kC;
    }
    c[0][0] = ci; c[0][1] = cj; c[0][2] = ck;
    c[1][0] = ci + (a == 0); c[1][1] = cj + (a == 1); c[1][2] = ck + (a == 2);
}

// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(64) k_gui_classify(Params p) {
    __shared__ float fv[kCorners];
    const uint32_t m = blockIdx.x;
    const int lane = threadIdx.x;
    if (m >= p.n) return;
    float o[3];
    mpu_origin(p, m, o);
    // intersects (:117-127, :164-183): the MPU box against every primitive's octree
    const float side = (float)(kG - 1) * p.cs;
    const float hx = o[0] + side, hy = o[1] + side, hz = o[2] + side;
    bool hit = false;
    for (uint32_t t = lane; t < p.T.nP; t += 64) {
        const PsGuiPrim& P = p.T.P[t];
        hit = hit || !((P.octLo[0] >= hx) || (P.octHi[0] <= o[0]) || (P.octLo[1] >= hy) || (P.octHi[1] <= o[1]) ||
                       (P.octLo[2] >= hz) || (P.octHi[2] <= o[2]));
    }
    if (__ballot(hit) == 0ull) {
        if (lane == 0) {
            p.counts[m] = 0ull;
            p.stats[m] = PsGuiMpuStats{0u, 0u, 0u, 0u};
        }
        return;
    }
    // the field cache: corner (i, j, k) at org + cs * (i, j, k) (:193-238)
    const int j = lane >> 3, k = lane & 7;
    const float y = o[1] + p.cs * (float)j, z = o[2] + p.cs * (float)k;
    for (int i = 0; i < kG; ++i) {
        const float x = o[0] + p.cs * (float)i;
        const float f = field<false>(p.T, x, y, z, nullptr);
        fv[corner_of(i, j, k)] = f;
        p.fvc[(size_t)m * kCorners + corner_of(i, j, k)] = f;
    }
    __syncthreads();
    uint32_t nv = 0, nt = 0, nc = 0;
    for (int cell = lane; cell < kCells; cell += 64) {
        const uint32_t cfg = cell_config(fv, cell, p.iso);
        if (cfg == 0u || cfg == 255u) continue;
        nc++;
        nt += p.tables->ntri[cfg];
        const int ci = cell / (kC * kC), cj = (cell / kC) % kC, ck = cell % kC;
        for (int q = 0; q < 16; ++q) {
            const uint32_t e = p.tables->cand[cfg][q];
            if (!(e & 32u)) break;
            bool own;
            edge_index(ci, cj, ck, (int)(e & 15u), &own);
            nv += (own && (e & 16u)) ? 1u : 0u;
        }
    }
    nv = wave_sum_u(nv);
    nt = wave_sum_u(nt);
    nc = wave_sum_u(nc);
    if (lane == 0) {
        p.counts[m] = (uint64_t)nv | ((uint64_t)nt << 32);
        p.stats[m] = PsGuiMpuStats{(uint32_t)kCorners, nc, nv, nt};
    }
}

// exclusive scan of the per-MPU (V, T) words in lattice order (one block of 1024)
__global__ void __launch_bounds__(1024) k_gui_scan(Params p) {
    __shared__ uint64_t wsum[16];
    __shared__ uint64_t carry;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    if (t == 0) carry = 0ull;
    __syncthreads();
    for (uint32_t base = 0; base < p.n; base += 1024) {
        const uint32_t m = base + t;
        const uint64_t v = m < p.n ? p.counts[m] : 0ull;
        uint64_t x = v;
        for (int o = 1; o < 64; o <<= 1) {
            const uint64_t y = __shfl_up(x, o);
            if (lane >= o) x += y;
        }
        if (lane == 63) wsum[w] = x;
        __syncthreads();
        uint64_t before = carry;
        for (int q = 0; q < w; ++q) before += wsum[q];
        if (m < p.n) p.offs[m] = before + x - v;
        __syncthreads();
        if (t == 1023) carry = before + x;
        __syncthreads();
    }
    if (t == 0) p.offs[p.n] = carry;
}

// Per MPU with a surface (one wavefront): the reference's vertex creation order (edge ->
// vertex id, as a vertex task list for k_gui_vertices) and the triangles in cell order,
// table order (:312-317), with mesh-wide vertex ids.
__global__ void __launch_bounds__(64) k_gui_edges(Params p) {
    __shared__ float fv[kCorners];
    __shared__ uint16_t edgeVid[kEdges];
    const uint32_t m = blockIdx.x;
    const int lane = threadIdx.x;
    if (m >= p.n) return;
    const uint64_t cnt = p.counts[m];
    if (cnt == 0ull) return;
    const uint64_t off = p.offs[m];
    const uint32_t vOff = (uint32_t)off, tOff = (uint32_t)(off >> 32);
    for (int c = lane; c < kCorners; c += 64) fv[c] = p.fvc[(size_t)m * kCorners + c];
    __syncthreads();
    // per-lane contiguous cells [c0, c1): counts, then the lattice-order prefix
    const int c0 = lane * kCellsPerLane, c1 = min(kCells, c0 + kCellsPerLane);
    uint32_t cfgs[kCellsPerLane];
    uint32_t nvL = 0, ntL = 0;
    for (int r = 0; r < kCellsPerLane; ++r) {
        const int cell = c0 + r;
        uint32_t cfg = 0;
        if (cell < c1) cfg = cell_config(fv, cell, p.iso);
        if (cfg == 255u) cfg = 0u;
        cfgs[r] = cfg;
        if (cfg == 0u) continue;
        ntL += p.tables->ntri[cfg];
        const int ci = cell / (kC * kC), cj = (cell / kC) % kC, ck = cell % kC;
        for (int q = 0; q < 16; ++q) {
            const uint32_t e = p.tables->cand[cfg][q];
            if (!(e & 32u)) break;
            bool own;
            edge_index(ci, cj, ck, (int)(e & 15u), &own);
            nvL += (own && (e & 16u)) ? 1u : 0u;
        }
    }
    uint32_t vb = wave_excl_scan(nvL), tb = wave_excl_scan(ntL);
    uint32_t tbase[kCellsPerLane];
    // vertex ids in creation order: edge -> id (LDS), id -> (MPU, edge) task
    for (int r = 0; r < kCellsPerLane; ++r) {
        const int cell = c0 + r;
        tbase[r] = tb;
        if (cell >= c1) continue;
        const uint32_t cfg = cfgs[r];
        if (cfg == 0u) continue;
        tb += p.tables->ntri[cfg];
        const int ci = cell / (kC * kC), cj = (cell / kC) % kC, ck = cell % kC;
        for (int q = 0; q < 16; ++q) {
            const uint32_t e = p.tables->cand[cfg][q];
            if (!(e & 32u)) break;
            bool own;
            const int idx = edge_index(ci, cj, ck, (int)(e & 15u), &own);
            if (own && (e & 16u)) {
                edgeVid[idx] = (uint16_t)vb;
                p.vtask[(size_t)vOff + vb] = (uint64_t)m | ((uint64_t)idx << 32);
                vb++;
            }
        }
    }
    __syncthreads();
    for (int r = 0; r < kCellsPerLane; ++r) {
        const int cell = c0 + r;
        if (cell >= c1) break;
        const uint32_t cfg = cfgs[r];
        if (cfg == 0u) continue;
        const int ci = cell / (kC * kC), cj = (cell / kC) % kC, ck = cell % kC;
        const uint32_t nT = p.tables->ntri[cfg];
        const size_t t0 = (size_t)tOff + tbase[r];
        for (uint32_t q = 0; q < 3 * nT; ++q) {
            bool own;
            const int idx = edge_index(ci, cj, ck, (int)(p.tables->cand[cfg][q] & 15u), &own);
            p.tris[3 * t0 + q] = vOff + edgeVid[idx];
        }
    }
}

// One mesh vertex per lane over the whole lattice: Newton root (:282-289), normal (:293),
// colour (:294) of the vertex task's edge; field evaluations to its MPU's statistics.
__global__ void __launch_bounds__(256) k_gui_vertices(Params p) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= p.nV) return;
    const uint64_t task = p.vtask[g];
    const uint32_t m = (uint32_t)task;
    int cc[2][3];
    edge_corners((int)(task >> 32), cc);
    float o[3];
    mpu_origin(p, m, o);
    const float iso = p.iso;
    V4 p1 = {o[0] + p.cs * (float)cc[0][0], o[1] + p.cs * (float)cc[0][1], o[2] + p.cs * (float)cc[0][2], 0.0f};
    V4 p2 = {o[0] + p.cs * (float)cc[1][0], o[1] + p.cs * (float)cc[1][1], o[2] + p.cs * (float)cc[1][2], 0.0f};
    const float* fv = p.fvc + (size_t)m * kCorners;
    const float fp1 = fv[corner_of(cc[0][0], cc[0][1], cc[0][2])];
    const float fp2 = fv[corner_of(cc[1][0], cc[1][1], cc[1][2])];
    V4 x = (fabsf(fp1 - iso) < fabsf(fp2 - iso)) ? p1 : p2;
    const float inv = 1.0f / kFieldEps;
    float outF = 0.0f;
    int it;
    for (it = 0; it < PSGUI_ITERATIONS; ++it) {
        const float fp = field<false>(p.T, x.x, x.y, x.z, nullptr);
        float gx = field<false>(p.T, x.x + kFieldEps, x.y + 0.0f, x.z + 0.0f, nullptr);
        float gy = field<false>(p.T, x.x + 0.0f, x.y + kFieldEps, x.z + 0.0f, nullptr);
        float gz = field<false>(p.T, x.x + 0.0f, x.y + 0.0f, x.z + kFieldEps, nullptr);
        gx -= fp; gy -= fp; gz -= fp;
        gx *= inv; gy *= inv; gz *= inv;
        const float d = iso - fp;
        const float gi = 1.0f / (gx * gx + gy * gy + gz * gz + fp * fp);
        x.x = x.x + (d * gx) * gi;
        x.y = x.y + (d * gy) * gi;
        x.z = x.z + (d * gz) * gi;
        outF = field<false>(p.T, x.x, x.y, x.z, nullptr);
        if (fabsf(outF - iso) < kFieldEps) break;
    }
    // the reference's count: (i + 1) * 4 for the root, + 3 for the normal (:282-292)
    atomicAdd(&p.stats[m].fieldEvals, (uint32_t)((it + 1) * 4) + 3u);
    float c4[4];
    (void)field<true>(p.T, x.x, x.y, x.z, c4);  // baseColor over the last walk's values
    // normal (:433-450): forward differences, -1/delta, normalizeXYZ
    const float ninv = -1.0f / kNormalDelta;
    float nx = field<false>(p.T, x.x + kNormalDelta, x.y + 0.0f, x.z + 0.0f, nullptr);
    float ny = field<false>(p.T, x.x + 0.0f, x.y + kNormalDelta, x.z + 0.0f, nullptr);
    float nz = field<false>(p.T, x.x + 0.0f, x.y + 0.0f, x.z + kNormalDelta, nullptr);
    nx -= outF; ny -= outF; nz -= outF;
    nx *= ninv; ny *= ninv; nz *= ninv;
    const float dn = sqrtf(nx * nx + ny * ny + nz * nz);
    if (dn > 0) {
        const float r = 1.0f / dn;
        nx *= r; ny *= r; nz *= r;
    } else {
        nx = ny = nz = 1;
    }
    p.pos[3 * (size_t)g] = x.x; p.pos[3 * (size_t)g + 1] = x.y; p.pos[3 * (size_t)g + 2] = x.z;
    p.nrm[3 * (size_t)g] = nx; p.nrm[3 * (size_t)g + 1] = ny; p.nrm[3 * (size_t)g + 2] = nz;
    p.col[4 * (size_t)g] = c4[0]; p.col[4 * (size_t)g + 1] = c4[1];
    p.col[4 * (size_t)g + 2] = c4[2]; p.col[4 * (size_t)g + 3] = c4[3];
}

__global__ void __launch_bounds__(1024) k_gui_totals(Params p) {
    __shared__ unsigned long long ev;
    __shared__ uint32_t cells, processed, inter;
    if (threadIdx.x == 0) { ev = 0; cells = processed = inter = 0; }
    __syncthreads();
    unsigned long long e = 0;
    uint32_t c = 0, pr = 0, in = 0;
    for (uint32_t m = threadIdx.x; m < p.n; m += 1024) {
        const PsGuiMpuStats s = p.stats[m];
        e += s.fieldEvals;
        c += s.intersectedCells;
        pr += s.fieldEvals > 0 ? 1u : 0u;
        in += s.ctTriangles > 0 ? 1u : 0u;
    }
    atomicAdd(&ev, e);
    atomicAdd(&cells, c);
    atomicAdd(&processed, pr);
    atomicAdd(&inter, in);
    __syncthreads();
    if (threadIdx.x == 0) {
        PsGuiInfo& I = *p.totals;
        I.ctFieldEvals = ev;
        I.ctIntersectedCells = cells;
        I.ctProcessedMPUs = processed;
        I.ctIntersectedMPUs = inter;
        I.ctMPUs = inter;  // removeExtraPUs (:403-405, :573-592) keeps the MPUs with faces
        I.ctCellsInIntersectedMPUs = (uint64_t)kCells * inter;
        const uint64_t tot = p.offs[p.n];
        I.ctVertices = (uint32_t)tot;
        I.ctTriangles = (uint32_t)(tot >> 32);
    }
}

__global__ void k_gui_probe(Tree T, const float* xyz, uint32_t n, float* out, float* col4) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float c[4];
    out[i] = field<true>(T, xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2], c);
    if (col4)
        for (int a = 0; a < 4; ++a) col4[4 * i + a] = c[a];
}

}  // namespace psgui

// ===========================================================================
// Host side: the psgpu_gui context and the C-ABI.
struct psgpu_gui {
    int device = 0;
    hipStream_t stream = nullptr;
    // tree
    PsGuiPrim* dP = nullptr;
    PsGuiOp* dO = nullptr;
    uint32_t* dK = nullptr;
    PsGuiMatrix* dM = nullptr;
    uint32_t nP = 0, nO = 0;
    bool haveTree = false;
    psgui::Tables* dTables = nullptr;
    // lattice buffers
    size_t capMpu = 0, capV = 0, capT = 0;
    float* fvc = nullptr;
    uint64_t* counts = nullptr;
    uint64_t* offs = nullptr;
    PsGuiMpuStats* stats = nullptr;
    float *pos = nullptr, *nrm = nullptr, *col = nullptr;
    uint32_t* tris = nullptr;
    uint64_t* vtask = nullptr;
    PsGuiInfo* dTotals = nullptr;
    PsGuiInfo* hTotals = nullptr;  // pinned
    PsGuiInfo lattice{};
    bool pending = false, haveResult = false;
};

namespace {

int gui_fail(hipError_t e, const char* what) {
    if (e == hipSuccess) return PSGPU_RET_SUCCESS;
    fprintf(stderr, "psgpu_gui: %s failed: %s\n", what, hipGetErrorString(e));
    return e == hipErrorOutOfMemory ? PSGPU_RET_NOT_ENOUGH_MEM : PSGPU_RET_DEVICE_ERROR;
}
#define GUI_CHECK(expr)                                    \
    do {                                                   \
        const int rc_ = gui_fail((expr), #expr);           \
        if (rc_ != PSGPU_RET_SUCCESS) return rc_;          \
    } while (0)

template <class T>
hipError_t grow(T*& ptr, size_t& cap, size_t n) {
    if (n <= cap && ptr) return hipSuccess;
    if (ptr) (void)hipFree(ptr);
    ptr = nullptr;
    cap = 0;
    const hipError_t e = hipMalloc(&ptr, std::max<size_t>(n, 1) * sizeof(T));
    if (e == hipSuccess) cap = n;
    return e;
}

// The per-config candidate tables from the MC table the library generates (psgpu_tritable,
// digest-equal to CCubeTable.h's g_triTableCache, which is the same table as
// _CellConfigTable.h's).
void build_tables(psgui::Tables& t) {
    std::vector<int32_t> tri(256 * 16);
    psgpu_tritable(tri.data());
    memset(&t, 0, sizeof(t));
    for (int c = 0; c < 256; ++c) {
        int n = 0;
        for (int q = 0; q < 16; ++q) {
            const int e = tri[c * 16 + q];
            if (e < 0) break;
            bool first = true;
            for (int r = 0; r < q; ++r) first = first && tri[c * 16 + r] != e;
            t.cand[c][q] = (uint8_t)(e | (first ? 16 : 0) | 32);
            n++;
        }
        t.ntri[c] = (uint8_t)(n / 3);
    }
}

// Kid ids in range, no cycles (every op reached once from op 0), depth and types the walk
// supports.
int validate(const PsGuiPrim* P, uint32_t nP, const PsGuiOp* O, uint32_t nO, const uint32_t* K, uint32_t nK,
             uint32_t nM) {
    for (uint32_t i = 0; i < nP; ++i) {
        const int t = P[i].type;
        if (!(t == PSGUI_PRIM_POINT || t == PSGUI_PRIM_LINE || t == PSGUI_PRIM_CYLINDER || t == PSGUI_PRIM_DISC ||
              t == PSGUI_PRIM_RING || t == PSGUI_PRIM_CUBE || t == PSGUI_PRIM_TRIANGLE ||
              t == PSGUI_PRIM_QUADRICPOINT || t == PSGUI_PRIM_NULL))
            return PSGUI_RET_UNSUPPORTED;
        if (P[i].idxMtx >= nM && P[i].idxMtx != 0) return PSGPU_RET_PARAM_ERROR;
    }
    if (nO == 0) return nP ? PSGPU_RET_SUCCESS : PSGPU_RET_PARAM_ERROR;
    std::vector<int> seen(nO, 0);
    std::vector<std::pair<uint32_t, int>> stack{{0u, 1}};
    while (!stack.empty()) {
        const auto [op, depth] = stack.back();
        stack.pop_back();
        if (op >= nO || seen[op]) return PSGPU_RET_INVALID_BVH;
        seen[op] = 1;
        if (depth > PSGUI_MAX_DEPTH) return PSGUI_RET_UNSUPPORTED;
        const PsGuiOp& o = O[op];
        const int t = o.type;
        if (!(t == PSGUI_OP_UNION || t == PSGUI_OP_INTERSECT || t == PSGUI_OP_DIF || t == PSGUI_OP_SMOOTHDIF ||
              t == PSGUI_OP_BLEND || t == PSGUI_OP_RICCIBLEND || t == PSGUI_OP_WARPTWIST ||
              t == PSGUI_OP_WARPTAPER || t == PSGUI_OP_WARPBEND || t == PSGUI_OP_WARPSHEAR))
            return PSGUI_RET_UNSUPPORTED;  // PCM's contact state is shared and order dependent
        if (o.ctKids <= 0) return PSGUI_RET_UNSUPPORTED;
        if (o.idxMtx >= nM && o.idxMtx != 0) return PSGPU_RET_PARAM_ERROR;
        if ((uint64_t)o.kidStart + (uint64_t)o.ctKids > nK) return PSGPU_RET_PARAM_ERROR;
        for (int i = 0; i < o.ctKids; ++i) {
            const uint32_t k = K[o.kidStart + i];
            const uint32_t id = k & 0xffffu;
            if (k >> 16) stack.push_back({id, depth + 1});
            else if (id >= nP) return PSGPU_RET_PARAM_ERROR;
        }
    }
    return PSGPU_RET_SUCCESS;
}

psgui::Params make_params(psgpu_gui* g) {
    psgui::Params p;
    memset(&p, 0, sizeof(p));
    p.T = {g->dP, g->dO, g->dK, g->dM, g->nP, g->nO};
    p.tables = g->dTables;
    return p;
}

}  // namespace

extern "C" {

int psgpu_gui_create(int device, psgpu_gui** out) {
    if (!out) return PSGPU_RET_PARAM_ERROR;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return PSGPU_RET_DEVICE_ERROR;
    psgpu_gui* g = new psgpu_gui();
    g->device = device;
    int rc = gui_fail(hipSetDevice(device), "hipSetDevice");
    if (rc == PSGPU_RET_SUCCESS) rc = gui_fail(hipStreamCreateWithFlags(&g->stream, hipStreamNonBlocking), "stream");
    if (rc == PSGPU_RET_SUCCESS) rc = gui_fail(hipMalloc(&g->dTables, sizeof(psgui::Tables)), "tables");
    if (rc == PSGPU_RET_SUCCESS) rc = gui_fail(hipMalloc(&g->dTotals, sizeof(PsGuiInfo)), "totals");
    if (rc == PSGPU_RET_SUCCESS) rc = gui_fail(hipHostMalloc(&g->hTotals, sizeof(PsGuiInfo), 0), "pinned");
    if (rc == PSGPU_RET_SUCCESS) {
        psgui::Tables t;
        build_tables(t);
        rc = gui_fail(hipMemcpy(g->dTables, &t, sizeof(t), hipMemcpyHostToDevice), "tables upload");
    }
    if (rc != PSGPU_RET_SUCCESS) {
        psgpu_gui_destroy(g);
        return rc;
    }
    *out = g;
    return PSGPU_RET_SUCCESS;
}

void psgpu_gui_destroy(psgpu_gui* g) {
    if (!g) return;
    (void)hipSetDevice(g->device);
    if (g->stream) (void)hipStreamSynchronize(g->stream);
    void* bufs[] = {g->dP, g->dO, g->dK, g->dM, g->dTables, g->fvc, g->counts, g->offs, g->stats,
                    g->pos, g->nrm, g->col, g->tris, g->vtask, g->dTotals};
    for (void* b : bufs)
        if (b) (void)hipFree(b);
    if (g->hTotals) (void)hipHostFree(g->hTotals);
    if (g->stream) (void)hipStreamDestroy(g->stream);
    delete g;
}

int psgpu_gui_set_tree(psgpu_gui* g, const PsGuiPrim* prims, uint32_t ctPrims, const PsGuiOp* ops, uint32_t ctOps,
                       const uint32_t* kids, uint32_t ctKids, const PsGuiMatrix* mtx, uint32_t ctMtx) {
    if (!g || (ctPrims && !prims) || (ctOps && !ops) || (ctKids && !kids) || ctMtx == 0 || !mtx)
        return PSGPU_RET_PARAM_ERROR;
    if (ctPrims > 0xffffu || ctOps > 0xffffu) return PSGPU_RET_PARAM_ERROR;  // kid ids are 16 bits
    const int vr = validate(prims, ctPrims, ops, ctOps, kids, ctKids, ctMtx);
    if (vr != PSGPU_RET_SUCCESS) return vr;
    GUI_CHECK(hipSetDevice(g->device));
    if (g->pending) GUI_CHECK(hipStreamSynchronize(g->stream));
    void* old[] = {g->dP, g->dO, g->dK, g->dM};
    for (void* b : old)
        if (b) (void)hipFree(b);
    g->dP = nullptr; g->dO = nullptr; g->dK = nullptr; g->dM = nullptr;
    GUI_CHECK(hipMalloc(&g->dP, std::max<size_t>(ctPrims, 1) * sizeof(PsGuiPrim)));
    GUI_CHECK(hipMalloc(&g->dO, std::max<size_t>(ctOps, 1) * sizeof(PsGuiOp)));
    GUI_CHECK(hipMalloc(&g->dK, std::max<size_t>(ctKids, 1) * sizeof(uint32_t)));
    GUI_CHECK(hipMalloc(&g->dM, (size_t)ctMtx * sizeof(PsGuiMatrix)));
    if (ctPrims) GUI_CHECK(hipMemcpy(g->dP, prims, ctPrims * sizeof(PsGuiPrim), hipMemcpyHostToDevice));
    if (ctOps) GUI_CHECK(hipMemcpy(g->dO, ops, ctOps * sizeof(PsGuiOp), hipMemcpyHostToDevice));
    if (ctKids) GUI_CHECK(hipMemcpy(g->dK, kids, ctKids * sizeof(uint32_t), hipMemcpyHostToDevice));
    GUI_CHECK(hipMemcpy(g->dM, mtx, ctMtx * sizeof(PsGuiMatrix), hipMemcpyHostToDevice));
    g->nP = ctPrims;
    g->nO = ctOps;
    g->haveTree = true;
    g->haveResult = false;
    return PSGPU_RET_SUCCESS;
}

int psgpu_gui_polygonize(psgpu_gui* g, const float octLo[3], const float octHi[3], float cellsize, float isovalue) {
    if (!g || !octLo || !octHi || !g->haveTree || !(cellsize > 0.0f)) return PSGPU_RET_PARAM_ERROR;
    GUI_CHECK(hipSetDevice(g->device));
    if (g->pending) GUI_CHECK(hipStreamSynchronize(g->stream));
    g->pending = false;
    g->haveResult = false;
    // setup (:348-385): cells per axis ceil(side / cellsize), MPUs of 7 cells, rounded up
    psgui::Params p = make_params(g);
    uint64_t n = 1;
    for (int a = 0; a < 3; ++a) {
        const float sideA = octHi[a] - octLo[a];
        const double c = std::ceil((double)(sideA / cellsize));
        if (!(c >= 0.0) || c > 1e7) return PSGPU_RET_PARAM_ERROR;
        const int cells = (int)c;
        p.dims[a] = (uint32_t)(cells / psgui::kC + (cells % psgui::kC != 0 ? 1 : 0));
        p.lo[a] = octLo[a];
        n *= p.dims[a];
    }
    if (n > (1u << 24)) return PSGPU_RET_NOT_ENOUGH_MEM;
    p.n = (uint32_t)n;
    p.cs = cellsize;
    p.side = (float)psgui::kC * cellsize;
    p.iso = isovalue;
    memset(&g->lattice, 0, sizeof(g->lattice));
    for (int a = 0; a < 3; ++a) g->lattice.dims[a] = p.dims[a];
    g->lattice.ctLatticeMPUs = p.n;
    if (p.n == 0) {
        g->haveResult = true;
        return PSGPU_RET_SUCCESS;
    }
    if (p.n > g->capMpu) {
        void* bufs[] = {g->fvc, g->counts, g->offs, g->stats};
        for (void* b : bufs)
            if (b) (void)hipFree(b);
        g->fvc = nullptr; g->counts = nullptr; g->offs = nullptr; g->stats = nullptr;
        g->capMpu = 0;
        GUI_CHECK(hipMalloc(&g->fvc, (size_t)p.n * psgui::kCorners * sizeof(float)));
        GUI_CHECK(hipMalloc(&g->counts, (size_t)p.n * sizeof(uint64_t)));
        GUI_CHECK(hipMalloc(&g->offs, ((size_t)p.n + 1) * sizeof(uint64_t)));
        GUI_CHECK(hipMalloc(&g->stats, (size_t)p.n * sizeof(PsGuiMpuStats)));
        g->capMpu = p.n;
    }
    p.fvc = g->fvc;
    p.counts = g->counts;
    p.offs = g->offs;
    p.stats = g->stats;
    p.totals = g->dTotals;
    hipLaunchKernelGGL(psgui::k_gui_classify, dim3(p.n), dim3(64), 0, g->stream, p);
    GUI_CHECK(hipGetLastError());
    hipLaunchKernelGGL(psgui::k_gui_scan, dim3(1), dim3(1024), 0, g->stream, p);
    GUI_CHECK(hipGetLastError());
    uint64_t tot = 0;
    GUI_CHECK(hipMemcpyAsync(&tot, g->offs + p.n, sizeof(tot), hipMemcpyDeviceToHost, g->stream));
    GUI_CHECK(hipStreamSynchronize(g->stream));
    const size_t V = (uint32_t)tot, T = (uint32_t)(tot >> 32);
    if (V > g->capV || !g->pos) {
        void* bufs[] = {g->pos, g->nrm, g->col, g->vtask};
        for (void* b : bufs)
            if (b) (void)hipFree(b);
        g->pos = nullptr; g->nrm = nullptr; g->col = nullptr; g->vtask = nullptr;
        g->capV = 0;
        const size_t cv = std::max<size_t>(V + V / 8, 1024);
        GUI_CHECK(hipMalloc(&g->pos, cv * 12));
        GUI_CHECK(hipMalloc(&g->nrm, cv * 12));
        GUI_CHECK(hipMalloc(&g->col, cv * 16));
        GUI_CHECK(hipMalloc(&g->vtask, cv * 8));
        g->capV = cv;
    }
    GUI_CHECK(grow(g->tris, g->capT, 3 * std::max<size_t>(T + T / 8, 1024)));
    p.pos = g->pos;
    p.nrm = g->nrm;
    p.col = g->col;
    p.tris = g->tris;
    p.vtask = g->vtask;
    p.nV = (uint32_t)V;
    hipLaunchKernelGGL(psgui::k_gui_edges, dim3(p.n), dim3(64), 0, g->stream, p);
    GUI_CHECK(hipGetLastError());
    if (V > 0) {
        hipLaunchKernelGGL(psgui::k_gui_vertices, dim3((unsigned)((V + 255) / 256)), dim3(256), 0, g->stream, p);
        GUI_CHECK(hipGetLastError());
    }
    hipLaunchKernelGGL(psgui::k_gui_totals, dim3(1), dim3(1024), 0, g->stream, p);
    GUI_CHECK(hipGetLastError());
    GUI_CHECK(hipMemcpyAsync(g->hTotals, g->dTotals, sizeof(PsGuiInfo), hipMemcpyDeviceToHost, g->stream));
    g->pending = true;
    return PSGPU_RET_SUCCESS;
}

int psgpu_gui_finish(psgpu_gui* g, PsGuiInfo* info) {
    if (!g) return PSGPU_RET_PARAM_ERROR;
    if (g->pending) {
        GUI_CHECK(hipSetDevice(g->device));
        GUI_CHECK(hipStreamSynchronize(g->stream));
        g->pending = false;
        PsGuiInfo I = *g->hTotals;
        for (int a = 0; a < 3; ++a) I.dims[a] = g->lattice.dims[a];
        I.ctLatticeMPUs = g->lattice.ctLatticeMPUs;
        g->lattice = I;
        g->haveResult = true;
    }
    if (!g->haveResult) return PSGPU_RET_PARAM_ERROR;
    if (info) *info = g->lattice;
    return PSGPU_RET_SUCCESS;
}

int psgpu_gui_download(psgpu_gui* g, float* pos, float* nrm, float* col4, uint32_t* tris, uint64_t* mpuOffsets,
                       PsGuiMpuStats* stats) {
    PsGuiInfo I;
    const int rc = psgpu_gui_finish(g, &I);
    if (rc != PSGPU_RET_SUCCESS) return rc;
    const size_t V = I.ctVertices, T = I.ctTriangles, N = I.ctLatticeMPUs;
    if (N == 0) {
        if (mpuOffsets) mpuOffsets[0] = 0;
        return PSGPU_RET_SUCCESS;
    }
    if (pos && V) GUI_CHECK(hipMemcpy(pos, g->pos, V * 12, hipMemcpyDeviceToHost));
    if (nrm && V) GUI_CHECK(hipMemcpy(nrm, g->nrm, V * 12, hipMemcpyDeviceToHost));
    if (col4 && V) GUI_CHECK(hipMemcpy(col4, g->col, V * 16, hipMemcpyDeviceToHost));
    if (tris && T) GUI_CHECK(hipMemcpy(tris, g->tris, T * 12, hipMemcpyDeviceToHost));
    if (mpuOffsets) GUI_CHECK(hipMemcpy(mpuOffsets, g->offs, (N + 1) * 8, hipMemcpyDeviceToHost));
    if (stats) GUI_CHECK(hipMemcpy(stats, g->stats, N * sizeof(PsGuiMpuStats), hipMemcpyDeviceToHost));
    return PSGPU_RET_SUCCESS;
}

int psgpu_gui_field_values(psgpu_gui* g, const float* xyz, uint32_t n, float* out, float* col4) {
    if (!g || !g->haveTree || (n && (!xyz || !out))) return PSGPU_RET_PARAM_ERROR;
    if (n == 0) return PSGPU_RET_SUCCESS;
    GUI_CHECK(hipSetDevice(g->device));
    float *dx = nullptr, *dout = nullptr, *dcol = nullptr;
    GUI_CHECK(hipMalloc(&dx, (size_t)n * 12));
    GUI_CHECK(hipMalloc(&dout, (size_t)n * 4));
    GUI_CHECK(hipMalloc(&dcol, (size_t)n * 16));
    int rc = gui_fail(hipMemcpy(dx, xyz, (size_t)n * 12, hipMemcpyHostToDevice), "upload");
    if (rc == PSGPU_RET_SUCCESS) {
        hipLaunchKernelGGL(psgui::k_gui_probe, dim3((n + 63) / 64), dim3(64), 0, g->stream, make_params(g).T, dx, n,
                           dout, dcol);
        rc = gui_fail(hipGetLastError(), "probe");
    }
    if (rc == PSGPU_RET_SUCCESS) rc = gui_fail(hipStreamSynchronize(g->stream), "probe sync");
    if (rc == PSGPU_RET_SUCCESS) rc = gui_fail(hipMemcpy(out, dout, (size_t)n * 4, hipMemcpyDeviceToHost), "download");
    if (rc == PSGPU_RET_SUCCESS && col4)
        rc = gui_fail(hipMemcpy(col4, dcol, (size_t)n * 16, hipMemcpyDeviceToHost), "download");
    (void)hipFree(dx);
    (void)hipFree(dout);
    (void)hipFree(dcol);
    return rc;
}

}  // extern "C"

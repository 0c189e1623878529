// Compat mode device code (CParsipOptimized over a COMPACTBLOBTREE):
// the compact tree walk and the kernel bodies, shared by the static interpreter kernels
// (psgpu_gui.hip) and the per-tree kernels generated at run time (psgpu_gui_jit.cpp,
// compiled by hiprtc with this header embedded).  Reference: CompactBlobTree.cpp
// (fieldvalueOp/Prim :677-1092, baseColorOp :1124-1294, normal :433-450,
// ComputeRootNewtonRaphsonVEC4 :1581-1622), CPolyParsipOptimized.cpp (:130-327).
#pragma once
#ifdef __HIPCC_RTC__
typedef unsigned char uint8_t;
typedef unsigned short uint16_t;
typedef unsigned int uint32_t;
typedef int int32_t;
typedef unsigned long long uint64_t;
typedef long long int64_t;
#include "parsip_gpu_gui.h"
#else
#include <hip/hip_runtime.h>

#include <cmath>

#include "../../include/parsip_gpu_gui.h"
#endif

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
    // exact culling (psgpu_gui_cull.cpp): per primitive / operator a world box (lo xyz, -,
    // hi xyz, -) outside which its field / value is exactly +0; nullptr: no culling
    const float* __restrict__ S;
    const float* __restrict__ OS;
    // masked != 0: per-wave live bits (primitives / operators 0-127) replace the per-point
    // box tests -- set by a kernel whose wave's points all lie in a known box
    uint64_t pm0, pm1, om0, om1;
    uint32_t masked;
    // trees with PCM / Instance nodes (the extended walk): per operator its parent operator
    // (0xffff: the root), and the PCM contact state the run reads (left, right)
    const uint16_t* __restrict__ parent;
    const float* __restrict__ pcm;
};

// Does any active lane's point lie in box b?  (A NaN coordinate counts as inside.)
__device__ __forceinline__ bool box_live(const float* b, float x, float y, float z) {
    const bool out = (x < b[0]) || (y < b[1]) || (z < b[2]) || (x > b[4]) || (y > b[5]) || (z > b[6]);
    return __ballot(!out) != 0ull;
}
__device__ __forceinline__ bool bit_of(uint64_t w0, uint64_t w1, uint32_t i) {
    return ((i < 64 ? (w0 >> i) : (w1 >> (i - 64))) & 1ull) != 0ull;
}
// Primitive / operator i reached by a point of the wave (T.S / T.OS non-null)
__device__ __forceinline__ bool prim_live(const Tree& T, uint32_t i, float x, float y, float z) {
    return T.masked ? bit_of(T.pm0, T.pm1, i) : box_live(T.S + 8 * i, x, y, z);
}
__device__ __forceinline__ bool op_live(const Tree& T, uint32_t i, float x, float y, float z) {
    return T.masked ? bit_of(T.om0, T.om1, i) : box_live(T.OS + 8 * i, x, y, z);
}
// Live bits of every node whose box meets [lo, hi] (one wave, all lanes active): a node
// whose box misses it is +0 at every point inside it.
__device__ __forceinline__ void mask_for_box(Tree& T, float lx, float ly, float lz, float hx, float hy, float hz) {
    if (!T.S || T.nP > 128u || T.nO > 128u) return;
    const uint32_t lane = threadIdx.x & 63u;
    auto meets = [&](const float* b) {
        return !(hx < b[0] || hy < b[1] || hz < b[2] || lx > b[4] || ly > b[5] || lz > b[6]);
    };
    T.pm0 = __ballot(lane < T.nP && meets(T.S + 8 * lane));
    T.pm1 = __ballot(lane + 64u < T.nP && meets(T.S + 8 * (lane + 64u)));
    T.om0 = __ballot(lane < T.nO && meets(T.OS + 8 * lane));
    T.om1 = __ballot(lane + 64u < T.nO && meets(T.OS + 8 * (lane + 64u)));
    T.masked = 1u;
}

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
    float* pcmState;     // extended walk: [0..1] the state the run reads (T.pcm), [2..3] the
                         // run's maxima (atomic max), copied to [0..1] when the run ends
};

// Ricci's powf, correctly rounded through f64 (one out-of-line copy: it is large).  A far
// primitive's field is +0, and pow(+0, y > 0) = +0 (C99 F.9.4.4) without the f64 pow.
__device__ __attribute__((noinline)) float cr_pow_f64(float x, float y) { return (float)pow((double)x, (double)y); }
__device__ __forceinline__ float cr_pow(float x, float y) {
    if (__float_as_uint(x) == 0u && y > 0.0f) return 0.0f;
    return cr_pow_f64(x, y);
}
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

// COMPACTBLOBTREE::fieldvaluePrim (CompactBlobTree.cpp:893-1092).  `type` and `hasMtx` are
// the primitive's own fields: the interpreter reads them, generated code passes literals.
__device__ __forceinline__ float prim_field_k(const Tree& T, const PsGuiPrim& P, int type, bool hasMtx, V4 p) {
    V3 pn = {p.x, p.y, p.z};
    if (hasMtx) {
        const PsGuiMatrix& m = T.M[P.idxMtx];
        const V4 pp = {p.x, p.y, p.z, 1.0f};
        pn.x = dot4(m.r[0], pp);
        pn.y = dot4(m.r[1], pp);
        pn.z = dot4(m.r[2], pp);
    }
    switch (type) {
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
        if (type == PSGUI_PRIM_DISC ? (sqrtf(len2(dir)) <= r) : false) {
            dd = absf(len2(pc) - len2(dir));
        } else if (type == PSGUI_PRIM_RING && float_eq(0.0f, len2(dir))) {
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
__device__ float prim_field(const Tree& T, uint32_t id, V4 p) {
    const PsGuiPrim& P = T.P[id];
    return prim_field_k(T, P, P.type, P.idxMtx != 0, p);
}

// The point an operator hands its kids: backward matrix (w -> 1), then the warp
// (CompactBlobTree.cpp:685-746, warps :1315-1536; a warped point is a fresh vec4f, w = 0).
__device__ __forceinline__ V4 op_point_k(const Tree& T, const PsGuiOp& O, int type, bool hasMtx, V4 p) {
    V4 q = p;
    if (hasMtx) {
        const PsGuiMatrix& m = T.M[O.idxMtx];
        q = {dot4(m.r[0], p), dot4(m.r[1], p), dot4(m.r[2], p), 1.0f};
    }
    const float* prm = O.params;
    switch (type) {
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
__device__ V4 op_point(const Tree& T, const PsGuiOp& O, V4 p) { return op_point_k(T, O, O.type, O.idxMtx != 0, p); }

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
__device__ __forceinline__ void fold_k(const PsGuiOp& O, int t, Frame& F, uint32_t i, float v, const float* c) {
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
__device__ __forceinline__ void fold(const PsGuiOp& O, Frame& F, uint32_t i, float v, const float* c) {
    fold_k<COLOR>(O, O.type, F, i, v, c);
}

template <bool COLOR>
__device__ __forceinline__ float finalize_k(const PsGuiOp& O, int t, Frame& F) {
    if (t == PSGUI_OP_RICCIBLEND) F.res = cr_pow(F.res, O.params[1]);
    if (COLOR && (t == PSGUI_OP_BLEND || t == PSGUI_OP_RICCIBLEND)) {
        if (F.aux == 0.0f) {
            F.c[0] = F.c0[0]; F.c[1] = F.c0[1]; F.c[2] = F.c0[2]; F.c[3] = F.c0[3];
        } else {
            const float r = 1.0f / F.aux;
            F.c[0] *= r; F.c[1] *= r; F.c[2] *= r; F.c[3] *= r;
        }
    }
    return F.res;
}
template <bool COLOR>
__device__ __forceinline__ float finalize(const PsGuiOp& O, Frame& F) { return finalize_k<COLOR>(O, O.type, F); }

__device__ __forceinline__ void init_frame_k(const Tree& T, Frame& F, uint32_t op, int type, bool hasMtx,
                                             V4 parentPoint) {
    F.p = op_point_k(T, T.O[op], type, hasMtx, parentPoint);
    F.op = op;
    F.next = 0;
    F.res = 0.0f;
    F.aux = 0.0f;
    F.c[0] = F.c[1] = F.c[2] = F.c[3] = 0.0f;
    F.c0[0] = F.c0[1] = F.c0[2] = F.c0[3] = 0.0f;
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
                // a culled primitive's field is exactly +0 at every lane's point
                const float v = (T.S == nullptr || prim_live(T, id, x, y, z)) ? prim_field(T, id, F.p) : 0.0f;
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

// The interpreter as the kernels' evaluator (generated code supplies its own `JitField`).
struct InterpField {
    template <bool COLOR>
    __device__ static float eval(const Tree& T, float x, float y, float z, float* colOut) {
        return field<COLOR>(T, x, y, z, colOut);
    }
    template <bool COLOR>
    __device__ static float eval_call(const Tree& T, float x, float y, float z, float* colOut) {
        return field<COLOR>(T, x, y, z, colOut);
    }
};

__device__ __forceinline__ float wave_min_f(float v) {
    for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ float wave_max_f(float v) {
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
    return v;
}
// Live masks from the AABB of the 64 lanes' points (all lanes active); a NaN coordinate
// anywhere keeps the per-point box tests.
__device__ __forceinline__ void wave_mask(Tree& T, float px, float py, float pz) {
    if (!T.S || T.nP > 128u || T.nO > 128u) return;
    if (__ballot(!(px == px) || !(py == py) || !(pz == pz)) != 0ull) return;
    mask_for_box(T, wave_min_f(px), wave_min_f(py), wave_min_f(pz), wave_max_f(px), wave_max_f(py), wave_max_f(pz));
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
// The extended walk: trees with PCM (precise contact modelling) or Instance nodes.  The
// interpreter's frame walk plus
//   - Instance (fieldvaluePrim :1069-1078): the instance's backward matrix, then its origin
//     node evaluated at that point with w = 1 (an origin operator is pushed as a frame of
//     the same stack); its colour is the origin's colour from the main walk's stored values
//     (baseColorPrim :1108-1122), i.e. the origin subtree walked again at the point the
//     main walk hands the origin (the ancestor chain's op_point from the root);
//   - PCM (fieldvalueOp :763-806, computePCM :490-570): the two kids' values, then
//     interpenetration (both >= iso: the larger plus iso minus the smaller, the smaller
//     raising the run's compression maximum), propagation (one >= iso, the other > 1e-3:
//     gradientAtNode :617-643 at the point, marchTowardNode :572-592 to the other kid's
//     iso surface, the gradient there, computePropagationDeformation :594-614 with the
//     contact state the run started with) or the maximum; colour baseColorOp :1191-1200.
// No culling: the sub-walks leave the wave's points.  set_tree guarantees PCM has 2 kids,
// no PCM sits inside a PCM's kid subtree and no Instance inside an Instance's origin
// subtree, so every sub-walk below is one level deep (LEVEL 0 the walk itself, 1 the
// colour walk of an Instance's origin, 2 the value walk of a PCM kid).
constexpr float kIsoValue = 0.5f;          // ISO_VALUE (_constSettings.h:10)
constexpr float kIsoDistance = 0.454202f;  // ISO_DISTANCE (:11), marchTowardNode's first step

struct PcmAcc {
    float l, r;  // the largest compression met left / right (0: none)
};

struct XFrame {
    Frame f;
    int32_t inst;  // >= 0: the frame evaluates instance primitive `inst`'s origin operator
};

__device__ __forceinline__ void xinit(const Tree& T, XFrame& F, uint32_t op, V4 parentPoint, int32_t inst) {
    init_frame(T, F.f, op, parentPoint);
    F.inst = inst;
}

// the point an Instance hands its origin: its backward matrix applied to (p, 1), w = 1
__device__ __forceinline__ V4 instance_point(const Tree& T, const PsGuiPrim& P, V4 p) {
    V4 q = {p.x, p.y, p.z, 1.0f};
    if (P.idxMtx != 0) {
        const PsGuiMatrix& m = T.M[P.idxMtx];
        const V4 pp = {p.x, p.y, p.z, 1.0f};
        q.x = dot4(m.r[0], pp);
        q.y = dot4(m.r[1], pp);
        q.z = dot4(m.r[2], pp);
    }
    return q;
}
__device__ __forceinline__ uint32_t inst_origin(const PsGuiPrim& P) { return (uint32_t)(int)P.res1[0]; }
__device__ __forceinline__ bool inst_origin_is_op(const PsGuiPrim& P) { return P.res1[2] != 0.0f; }

template <bool COLOR>
__device__ __forceinline__ void xfold(const PsGuiOp& O, XFrame& F, uint32_t i, float v, const float* c) {
    if (O.type == PSGUI_OP_PCM) {  // kid 0 -> res / c, kid 1 -> aux / c0
        if (i == 0) {
            F.f.res = v;
            if (COLOR) { F.f.c[0] = c[0]; F.f.c[1] = c[1]; F.f.c[2] = c[2]; F.f.c[3] = c[3]; }
        } else {
            F.f.aux = v;
            if (COLOR) { F.f.c0[0] = c[0]; F.f.c0[1] = c[1]; F.f.c0[2] = c[2]; F.f.c0[3] = c[3]; }
        }
        return;
    }
    fold_k<COLOR>(O, O.type, F.f, i, v, c);
}

template <int LEVEL>
__device__ float xwalk_value(const Tree& T, uint32_t op0, V4 parentPoint);

// fieldAtNode (:646-652): a kid's value at p (a primitive kid may be an Instance)
template <int LEVEL>
__device__ float node_value(const Tree& T, uint32_t kid, V4 p) {
    const uint32_t id = kid & 0xffffu;
    if (kid >> 16) return xwalk_value<LEVEL>(T, id, p);
    const PsGuiPrim& P = T.P[id];
    if (P.type != PSGUI_PRIM_INSTANCE) return prim_field(T, id, p);
    const V4 q = instance_point(T, P, p);
    return inst_origin_is_op(P) ? xwalk_value<LEVEL>(T, inst_origin(P), q) : prim_field(T, inst_origin(P), q);
}

// gradientAtNode (:617-643): forward differences of a kid at p, (f(p + d e) - fp) * (1 / d)
template <int LEVEL>
__device__ V3 node_gradient(const Tree& T, uint32_t kid, V4 p, float fp) {
    const float inv = 1.0f / kNormalDelta;
    const float a0 = node_value<LEVEL>(T, kid, V4{p.x + kNormalDelta, p.y + 0.0f, p.z + 0.0f, p.w + 0.0f});
    const float a1 = node_value<LEVEL>(T, kid, V4{p.x + 0.0f, p.y + kNormalDelta, p.z + 0.0f, p.w + 0.0f});
    const float a2 = node_value<LEVEL>(T, kid, V4{p.x + 0.0f, p.y + 0.0f, p.z + kNormalDelta, p.w + 0.0f});
    return V3{(a0 - fp) * inv, (a1 - fp) * inv, (a2 - fp) * inv};
}

// computePropagationDeformation (:594-614)
__device__ __forceinline__ float pcm_deformation(float dist, float k, float a0, float w) {
    const float wh = 0.5f * w, w2 = w * w, w3 = w2 * w;
    if (dist >= 0.0f && dist < wh) {
        const float p1 = (4.0f * (w * k - 4.0f * a0)) / w3;
        const float p2 = (4.0f * (3.0f * a0 - w * k)) / w2;
        const float d2 = dist * dist, d3 = dist * d2;
        return p1 * d3 + p2 * d2 + k * dist;
    }
    if (dist >= wh && dist < w) return (4.0f * a0 + (dist - w) * (dist - w) * (4.0f * dist - w)) / w3;
    return 0.0f;
}

// The propagation term of computePCM (:524-564) for the kid `kid` with value fp at p.
template <int LEVEL>
__device__ float pcm_propagation(const Tree& T, uint32_t kid, V4 p, float fp, float a0, float w) {
    const V3 grad = node_gradient<LEVEL>(T, kid, p, fp);
    const V3 pp = {p.x, p.y, p.z};
    // marchTowardNode (:572-592): shrink-wrap steps along the gradient toward f = iso
    int dir = (fp < kIsoValue) ? 1 : -1;
    float step = kIsoDistance;
    V3 q = pp;
    for (int it = 0; it < PSGUI_PCM_MARCH_MAX && !(((kIsoValue - kFieldEps) < fp) && (fp < (kIsoValue + kFieldEps)));
         ++it) {
        const float s = step * (float)dir;
        q.x += grad.x * s;
        q.y += grad.y * s;
        q.z += grad.z * s;
        fp = node_value<LEVEL>(T, kid, V4{q.x, q.y, q.z, 0.0f});
        const int dir2 = (fp < kIsoValue) ? 1 : -1;
        if (dir != dir2) step *= 0.5f;
        dir = dir2;
    }
    const V3 g0 = node_gradient<LEVEL>(T, kid, V4{q.x, q.y, q.z, 0.0f}, fp);
    const float k = sqrtf(g0.x * g0.x + g0.y * g0.y + g0.z * g0.z);
    const float dx = q.x - pp.x, dy = q.y - pp.y, dz = q.z - pp.z;  // pp.distance(p0)
    const float d = sqrtf(dx * dx + dy * dy + dz * dz);
    return pcm_deformation(d, k, a0, w);
}

__device__ __forceinline__ const float* node_oct(const Tree& T, uint32_t kid, bool hi) {
    const uint32_t id = kid & 0xffffu;
    return (kid >> 16) ? (hi ? T.O[id].octHi : T.O[id].octLo) : (hi ? T.P[id].octHi : T.P[id].octLo);
}

// computePCM (:490-570) over the kids' values fp1, fp2 at p (the PCM's own point)
template <int LEVEL>
__device__ float pcm_field(const Tree& T, const PsGuiOp& O, V4 p, float fp1, float fp2, PcmAcc* acc) {
    const uint32_t k1 = T.K[O.kidStart], k2 = T.K[O.kidStart + 1];
    const float *lo1 = node_oct(T, k1, false), *hi1 = node_oct(T, k1, true);
    const float *lo2 = node_oct(T, k2, false), *hi2 = node_oct(T, k2, true);
    const bool crossed = !((lo1[0] >= hi2[0]) || (hi1[0] <= lo2[0]) || (lo1[1] >= hi2[1]) || (hi1[1] <= lo2[1]) ||
                           (lo1[2] >= hi2[2]) || (hi1[2] <= lo2[2]));  // intersects (_GlobalFunctions.h:34-44)
    if (!crossed) return maxf(fp1, fp2);
    if (fp1 >= kIsoValue && fp2 >= kIsoValue) {  // interpenetration
        if (fp1 > fp2) {
            if (acc && fp2 > acc->l) acc->l = fp2;
            return fp1 + (kIsoValue - fp2);
        }
        if (acc && fp1 > acc->r) acc->r = fp1;
        return fp2 + (kIsoValue - fp1);
    }
    if constexpr (LEVEL >= 2) {
        return maxf(fp1, fp2);  // not reached: set_tree rejects a PCM inside a PCM's kids
    } else {
        if (fp1 >= kIsoValue && fp2 > kFieldEps) return fp1 + pcm_propagation<2>(T, k2, p, fp2, O.params[2] * T.pcm[0], O.params[0]);
        if (fp2 >= kIsoValue && fp1 > kFieldEps) return fp2 + pcm_propagation<2>(T, k1, p, fp1, O.params[3] * T.pcm[1], O.params[1]);
        return maxf(fp1, fp2);
    }
}

template <bool COLOR, int LEVEL>
__device__ float xwalk(const Tree& T, uint32_t op0, V4 parentPoint, V4 rootPoint, float* colOut, PcmAcc* acc);

// An Instance's colour: its origin operator's colour in the main walk (LEVEL 0 only: no
// Instance sits inside an origin subtree).
__device__ void origin_colour(const Tree& T, uint32_t X, V4 rootPoint, float* c) {
    uint32_t path[PSGUI_MAX_DEPTH];
    int n = 0;
    for (uint32_t a = T.parent[X]; a != 0xffffu && n < PSGUI_MAX_DEPTH; a = T.parent[a]) path[n++] = a;
    V4 q = rootPoint;
    for (int j = n - 1; j >= 0; --j) q = op_point(T, T.O[path[j]], q);
    (void)xwalk<true, 1>(T, X, q, q, c, nullptr);
}

// fieldvalueOp from operator op0 (its parent's point `parentPoint`) and, with COLOR, its
// baseColorOp over the same walk's values.
template <bool COLOR, int LEVEL>
__device__ float xwalk(const Tree& T, uint32_t op0, V4 parentPoint, V4 rootPoint, float* colOut, PcmAcc* acc) {
    XFrame st[PSGUI_MAX_DEPTH];
    int sp = 0;
    xinit(T, st[0], op0, parentPoint, -1);
    for (;;) {
        XFrame& F = st[sp];
        const PsGuiOp& O = T.O[F.f.op];
        if (F.f.next < (uint32_t)O.ctKids) {
            const uint32_t k = T.K[O.kidStart + F.f.next];
            const uint32_t i = F.f.next++;
            const uint32_t id = k & 0xffffu;
            if (k >> 16) {
                xinit(T, st[++sp], id, F.f.p, -1);
                continue;
            }
            const PsGuiPrim& P = T.P[id];
            if (P.type != PSGUI_PRIM_INSTANCE) {
                xfold<COLOR>(O, F, i, prim_field(T, id, F.f.p), P.color);
                continue;
            }
            const V4 q = instance_point(T, P, F.f.p);
            const uint32_t o = inst_origin(P);
            if (inst_origin_is_op(P)) {
                xinit(T, st[++sp], o, q, (int32_t)id);
                continue;
            }
            xfold<COLOR>(O, F, i, prim_field(T, o, q), T.P[o].color);  // a primitive origin's colour
            continue;
        }
        float v;
        if (O.type == PSGUI_OP_PCM) {
            v = pcm_field<LEVEL>(T, O, F.f.p, F.f.res, F.f.aux, acc);
            if (COLOR && !(F.f.res > F.f.aux)) {
                F.f.c[0] = F.f.c0[0]; F.f.c[1] = F.f.c0[1]; F.f.c[2] = F.f.c0[2]; F.f.c[3] = F.f.c0[3];
            }
        } else {
            v = finalize_k<COLOR>(O, O.type, F.f);
        }
        if (sp == 0) {
            if (COLOR) { colOut[0] = F.f.c[0]; colOut[1] = F.f.c[1]; colOut[2] = F.f.c[2]; colOut[3] = F.f.c[3]; }
            return v;
        }
        const float* c = F.f.c;
        float ic[4];
        if constexpr (COLOR && LEVEL == 0) {
            if (F.inst >= 0) {
                origin_colour(T, F.f.op, rootPoint, ic);
                c = ic;
            }
        }
        XFrame& Pf = st[--sp];
        xfold<COLOR>(T.O[Pf.f.op], Pf, Pf.f.next - 1, v, c);
    }
}

template <int LEVEL>
__device__ float xwalk_value(const Tree& T, uint32_t op0, V4 parentPoint) {
    return xwalk<false, LEVEL>(T, op0, parentPoint, parentPoint, nullptr, nullptr);
}

// COMPACTBLOBTREE::fieldvalue / baseColor (:476-487, :1095-1106) over the extended walk;
// acc (may be null) collects the interpenetration maxima of this evaluation.
struct ExtField {
    template <bool COLOR>
    __device__ static float eval(const Tree& T, float x, float y, float z, float* colOut, PcmAcc* acc = nullptr) {
        const V4 p = {x, y, z, 0.0f};
        if (T.nO == 0) {
            if (COLOR && T.nP) { colOut[0] = T.P[0].color[0]; colOut[1] = T.P[0].color[1]; colOut[2] = T.P[0].color[2]; colOut[3] = T.P[0].color[3]; }
            return T.nP ? node_value<2>(T, 0u, p) : 0.0f;
        }
        return xwalk<COLOR, 0>(T, 0, p, p, colOut, acc);
    }
    template <bool COLOR>
    __device__ static float eval_call(const Tree& T, float x, float y, float z, float* colOut, PcmAcc* acc = nullptr) {
        return eval<COLOR>(T, x, y, z, colOut, acc);
    }
};
template <class EV>
struct IsExt {
    static constexpr bool value = false;
};
template <>
struct IsExt<ExtField> {
    static constexpr bool value = true;
};

// One wave's compression maxima into the run's (all 64 lanes active).
__device__ __forceinline__ void pcm_publish(const Params& p, const PcmAcc& a) {
    const float l = wave_max_f(a.l), r = wave_max_f(a.r);
    if ((threadIdx.x & 63u) == 0u) {
        if (l > 0.0f) atomicMax(reinterpret_cast<int*>(p.pcmState + 2), __float_as_int(l));
        if (r > 0.0f) atomicMax(reinterpret_cast<int*>(p.pcmState + 3), __float_as_int(r));
    }
}

// ---------------------------------------------------------------------------
// Kernel bodies over an evaluator EV (InterpField, ExtField or a generated JitField).
//
// One wavefront per MPU: the octree test against every primitive (:164-183), the 8^3
// field cache (lane = (y, z), one walk per x), configs with `f > iso`, per-MPU counts.
template <class EV>
__device__ __forceinline__ void classify_body(const Params& p, float* fv) {
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
    // the field cache: corner (i, j, k) at org + cs * (i, j, k) (:193-238); the x-slice i's
    // corners lie in {x} x [org.y, org.y + cs * 7] x [org.z, org.z + cs * 7] (the lanes' own
    // expressions at the extreme indices): one live mask per slice
    const float yHi = o[1] + p.cs * 7.0f, zHi = o[2] + p.cs * 7.0f;
    const int j = lane >> 3, k = lane & 7;
    const float y = o[1] + p.cs * (float)j, z = o[2] + p.cs * (float)k;
    PcmAcc acc{0.0f, 0.0f};
#pragma unroll 1
    for (int i = 0; i < kG; ++i) {
        const float x = o[0] + p.cs * (float)i;
        Tree T = p.T;
        mask_for_box(T, x, o[1], o[2], x, yHi, zHi);
        float f;
        if constexpr (IsExt<EV>::value) f = EV::template eval<false>(T, x, y, z, nullptr, &acc);
        else f = EV::template eval<false>(T, x, y, z, nullptr);
        fv[corner_of(i, j, k)] = f;
        p.fvc[(size_t)m * kCorners + corner_of(i, j, k)] = f;
    }
    if constexpr (IsExt<EV>::value) pcm_publish(p, acc);  // every corner is a reference evaluation
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

// The mesh vertices over the whole lattice, a quad of lanes per vertex: Newton root
// (:282-289), normal (:293), colour (:294) of the vertex task's edge; field evaluations to
// its MPU's statistics.  Each round every lane walks once -- lanes 0-2 at x + eps*e_a, lane 3
// at x -- so one round yields f(x) (the previous Newton step's value: its convergence test)
// and the whole gradient at x; a last round takes the normal samples (lanes 0-2) and the
// colour walk at x (lane 3).  Rounds per vertex: iterations + 3, against 4 walks per
// iteration + 4 in sequence with a lane per vertex (train scene, cellsize 0.13: 2.3 vs
// 6.1 ms; equal at 0.03); every evaluation is at the reference's point, the same bits.
template <class EV>
__device__ __forceinline__ void vertices_body(const Params& p) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t g = t >> 2;
    const int q = (int)(t & 3u);
    const bool valid = g < p.nV;  // whole quads: the four lanes share g
    const int base = (int)(threadIdx.x & 63u) & ~3;
    uint32_t m = 0;
    V4 x = {0.0f, 0.0f, 0.0f, 0.0f};
    const float iso = p.iso;
    if (valid) {
        const uint64_t task = p.vtask[g];
        m = (uint32_t)task;
        int cc[2][3];
        edge_corners((int)(task >> 32), cc);
        float o[3];
        mpu_origin(p, m, o);
        V4 p1 = {o[0] + p.cs * (float)cc[0][0], o[1] + p.cs * (float)cc[0][1], o[2] + p.cs * (float)cc[0][2], 0.0f};
        V4 p2 = {o[0] + p.cs * (float)cc[1][0], o[1] + p.cs * (float)cc[1][1], o[2] + p.cs * (float)cc[1][2], 0.0f};
        const float* fv = p.fvc + (size_t)m * kCorners;
        const float fp1 = fv[corner_of(cc[0][0], cc[0][1], cc[0][2])];
        const float fp2 = fv[corner_of(cc[1][0], cc[1][1], cc[1][2])];
        x = (fabsf(fp1 - iso) < fabsf(fp2 - iso)) ? p1 : p2;
    }
    const float inv = 1.0f / kFieldEps;
    float outF = 0.0f;
    int itFinal = PSGUI_ITERATIONS;
    bool done = !valid;
    // extended walk: the compression maxima of the evaluations the reference makes (lane 3's
    // x of every round; lanes 0-2's gradient samples only when the iteration goes on)
    PcmAcc run{0.0f, 0.0f};
    auto commit = [&](const PcmAcc& e) {
        run.l = e.l > run.l ? e.l : run.l;
        run.r = e.r > run.r ? e.r : run.r;
    };
    // every lane stays in the loop until the whole wave is done (finished quads walk their
    // last point again and ignore it), so each round's culling masks come from all 64 lanes
    for (int r = 0;; ++r) {
        if (__ballot(!done) == 0ull) break;
        float px = x.x, py = x.y, pz = x.z;
        if (q < 3) {  // x + eps * e_q, the reference's `+ 0.0f` kept
            px = x.x + (q == 0 ? kFieldEps : 0.0f);
            py = x.y + (q == 1 ? kFieldEps : 0.0f);
            pz = x.z + (q == 2 ? kFieldEps : 0.0f);
        }
        Tree T = p.T;
        wave_mask(T, px, py, pz);
        PcmAcc e{0.0f, 0.0f};
        float f;
        if constexpr (IsExt<EV>::value) f = EV::template eval_call<false>(T, px, py, pz, nullptr, &e);
        else f = EV::template eval_call<false>(T, px, py, pz, nullptr);
        const float fx = __shfl(f, base + 0), fy = __shfl(f, base + 1), fz = __shfl(f, base + 2);
        const float fc = __shfl(f, base + 3);
        if (done) continue;
        if (IsExt<EV>::value && q == 3) commit(e);
        if (r >= 1) {  // fc = f(x) = the step of iteration r - 1's outF
            outF = fc;
            if (fabsf(outF - iso) < kFieldEps) {
                itFinal = r - 1;
                done = true;
                continue;
            }
            if (r - 1 == PSGUI_ITERATIONS - 1) {  // the loop ran out: i == DEFAULT_ITERATIONS
                done = true;
                continue;
            }
        }
        if (IsExt<EV>::value && q < 3) commit(e);
        const float fp = fc;
        float gx = fx, gy = fy, gz = fz;
        gx -= fp; gy -= fp; gz -= fp;
        gx *= inv; gy *= inv; gz *= inv;
        const float d = iso - fp;
        const float gi = 1.0f / (gx * gx + gy * gy + gz * gz + fp * fp);
        x.x = x.x + (d * gx) * gi;
        x.y = x.y + (d * gy) * gi;
        x.z = x.z + (d * gz) * gi;
    }
    // normal samples (lanes 0-2) and baseColor over the walk at x (lane 3)
    float px = x.x, py = x.y, pz = x.z;
    if (q < 3) {
        px = x.x + (q == 0 ? kNormalDelta : 0.0f);
        py = x.y + (q == 1 ? kNormalDelta : 0.0f);
        pz = x.z + (q == 2 ? kNormalDelta : 0.0f);
    }
    float c4[4];
    Tree T = p.T;
    wave_mask(T, px, py, pz);
    float f;
    if constexpr (IsExt<EV>::value) {
        PcmAcc e{0.0f, 0.0f};  // normal samples; lane 3 re-walks x (the same maxima)
        f = EV::template eval_call<true>(T, px, py, pz, c4, &e);
        if (valid) commit(e);
        pcm_publish(p, run);
    } else {
        f = EV::template eval_call<true>(T, px, py, pz, c4);
    }
    float nx = __shfl(f, base + 0), ny = __shfl(f, base + 1), nz = __shfl(f, base + 2);
    const float col0 = __shfl(c4[0], base + 3), col1 = __shfl(c4[1], base + 3);
    const float col2 = __shfl(c4[2], base + 3), col3 = __shfl(c4[3], base + 3);
    if (q != 0 || !valid) return;
    atomicAdd(&p.stats[m].fieldEvals, (uint32_t)((itFinal + 1) * 4) + 3u);
    const float ninv = -1.0f / kNormalDelta;
    nx -= outF; ny -= outF; nz -= outF;
    nx *= ninv; ny *= ninv; nz *= ninv;
    const float dn = sqrtf(nx * nx + ny * ny + nz * nz);
    if (dn > 0) {
        const float rr = 1.0f / dn;
        nx *= rr; ny *= rr; nz *= rr;
    } else {
        nx = ny = nz = 1;
    }
    p.pos[3 * (size_t)g] = x.x; p.pos[3 * (size_t)g + 1] = x.y; p.pos[3 * (size_t)g + 2] = x.z;
    p.nrm[3 * (size_t)g] = nx; p.nrm[3 * (size_t)g + 1] = ny; p.nrm[3 * (size_t)g + 2] = nz;
    p.col[4 * (size_t)g] = col0; p.col[4 * (size_t)g + 1] = col1;
    p.col[4 * (size_t)g + 2] = col2; p.col[4 * (size_t)g + 3] = col3;
}

template <class EV>
__device__ __forceinline__ void probe_body(const Tree& T, const float* xyz, uint32_t n, float* out, float* col4) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float c[4];
    out[i] = EV::template eval<true>(T, xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2], c);
    if (col4)
        for (int a = 0; a < 4; ++a) col4[4 * i + a] = c[a];
}

}  // namespace psgui

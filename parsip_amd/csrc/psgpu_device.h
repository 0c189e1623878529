// psgpu_device.h — device code shared by the static kernels (psgpu_kernels.hip) and the
// run-time specialised kernels (psgpu_jit.cpp, compiled with hiprtc).  Must compile
// under hiprtc: no system headers.
//
// Reference semantics restated here (Parsip100/PS_SimdPoly/include/):
//   computePrimitiveField           PS_Polygonizer.cpp:934-1179
//   ComputeWyvillFieldValueSquare_  PS_Polygonizer.h:397-407
//   FieldComputer::fieldValue       PS_Polygonizer.cpp:1184-1376 (op-box pruning :1228-1252)
//   FieldComputer::fieldValueAndColor :1378-1551, normal :1598-1622
//   CMPUProcessor::process_cells_simd :475-829
// Every fp32 expression keeps the reference's operation order; builds use
// -ffp-contract=off, IEEE division/sqrt (sqrtf, '/') and IEEE denormals.  max/min are the
// SSE definitions (a>b?a:b, a<b?a:b; PS_SIMDVecN.h:388-389), masks are {0,1} multipliers.
#pragma once
#include "psgpu_model.h"

namespace psgpu {

// ---------------------------------------------------------------------------
// The model is read through the constant address space so that every wave-uniform
// access (walk program, op boxes, primitive parameters) is an s_load into SGPRs.
typedef const __attribute__((address_space(4))) DevModel* ModelPtr;
typedef const __attribute__((address_space(4))) DevPrim CPrim;
typedef const __attribute__((address_space(4))) DevOp COp;
typedef const __attribute__((address_space(4))) CubeTablesDev* TablePtr;
__device__ __forceinline__ ModelPtr as_const(const DevModel* m) { return (ModelPtr)m; }
__device__ __forceinline__ TablePtr as_const(const CubeTablesDev* t) { return (TablePtr)t; }

__device__ __forceinline__ Instr load_instr(ModelPtr M, int pc) {
    typedef const __attribute__((address_space(4))) uint32_t* CU32;
    const CU32 w = (CU32)(&M->instr[pc]);
    const uint32_t words[3] = {w[0], w[1], w[2]};
    Instr I;
    __builtin_memcpy(&I, words, 12);
    return I;
}

// +0.0f made by an instruction of the block it is written in: the culled branch of the
// generated walk (`else f = 0`) keeps its zeros instead of the compiler turning them into
// constants of a phi, which it materialises before the branch, on every path
// (PSGPU_ZERO_ASM 0: plain constants, experiments).
#ifndef PSGPU_ZERO_ASM
#define PSGPU_ZERO_ASM 0  // 1: isolated k_precheck / k_vertex 1-1.5 us slower, 4 engines 2 % slower (r04 A/B)
#endif
__device__ __forceinline__ float zero_f() {
#if PSGPU_ZERO_ASM
    float z;
    asm volatile("v_mov_b32 %0, 0" : "=v"(z));
    return z;
#else
    return 0.0f;
#endif
}
__device__ __forceinline__ float max_ref(float a, float b) { return a > b ? a : b; }
__device__ __forceinline__ float min_ref(float a, float b) { return a < b ? a : b; }
__device__ __forceinline__ float m01(bool c) { return c ? 1.0f : 0.0f; }
__device__ __forceinline__ int lane_id() { return __lane_id(); }
__device__ __forceinline__ uint64_t ballot(bool v) { return __ballot(v); }

// 1 if any lane of this lane's 4-lane group has v set (the reference's 4-wide SIMD
// group: VecNMask(inside) == PS_SIMD_ALLZERO, PS_Polygonizer.cpp:1243).
// DPP quad_perm swaps within each 4-lane group: [1,0,3,2] then [2,3,0,1].
__device__ __forceinline__ bool quad_any(bool v) {
    int x = v ? 1 : 0;
    x |= __builtin_amdgcn_mov_dpp(x, 0xB1, 0xF, 0xF, false);
    x |= __builtin_amdgcn_mov_dpp(x, 0x4E, 0xF, 0xF, false);
    return x != 0;
}

// GROUP 5 is GROUP 4 for the S2 cache (k_mpu): the 4 lanes of a group are 4 z-consecutive
// corners of one x-slice and one y row, and every point of a lane has the lane's y and z.
// The generated walk uses that to test a pruned op's box once per op for y and z (the
// group's z union by one quad OR) and per point for x alone: group_any(X | Y | Z) =
// X | Y | group_any(Z) when X and Y are the same in the 4 lanes -- the same decisions.
#ifndef PSGPU_S2_GROUP
#define PSGPU_S2_GROUP 4  // 5: the per-op y/z test -- isolated k_mpu 32.3 vs 35.1 us, but four engines
                          // in flight 0.0611-0.0624 vs 0.0555-0.0560 ms/step (r04 A/B,
                          // profiles/r04_kernel_variants_ab.txt): kept as an experiment
#endif
#ifndef PSGPU_S2_OCT
#define PSGPU_S2_OCT 0  // S2 by octant passes (k_precheck's per-octant proofs): 0 off, 1 when <= 4
                        // octants are unproven, 2 always (two passes when 5-8 are unproven)
#endif
constexpr int kS2Group = PSGPU_S2_GROUP;
template <int GROUP>
__device__ __forceinline__ bool group_any(bool v) {
    if (GROUP == 4 || GROUP == 5) return quad_any(v);
    return v;
}

// Cross-lane work on DPP (no LDS crossbar round trips): quad_perm [1,0,3,2] = 0xB1,
// [2,3,0,1] = 0x4E, row_half_mirror = 0x141, row_mirror = 0x140, row_shr:n = 0x110 + n,
// row_bcast:15 = 0x142, row_bcast:31 = 0x143.
#define PSGPU_DPP_F(v, ctrl) __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), (ctrl), 0xF, 0xF, false))

// Value of lane S of this lane's quad.
template <int S>
__device__ __forceinline__ float quad_bcast(float v) { return PSGPU_DPP_F(v, S * 0x55); }

// Wave-uniform min / max (NaNs must be excluded by the caller).
__device__ __forceinline__ float wave_min(float v) {
    v = fminf(v, PSGPU_DPP_F(v, 0xB1));
    v = fminf(v, PSGPU_DPP_F(v, 0x4E));
    v = fminf(v, PSGPU_DPP_F(v, 0x141));
    v = fminf(v, PSGPU_DPP_F(v, 0x140));
    return fminf(fminf(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0)),
                       __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16))),
                 fminf(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32)),
                       __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48))));
}
__device__ __forceinline__ float wave_max(float v) {
    v = fmaxf(v, PSGPU_DPP_F(v, 0xB1));
    v = fmaxf(v, PSGPU_DPP_F(v, 0x4E));
    v = fmaxf(v, PSGPU_DPP_F(v, 0x141));
    v = fmaxf(v, PSGPU_DPP_F(v, 0x140));
    return fmaxf(fmaxf(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0)),
                       __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16))),
                 fmaxf(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32)),
                       __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48))));
}
// Inclusive prefix sum over the wave (Hillis-Steele in 16-lane rows, then row broadcasts).
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, true);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, true);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, true);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, true);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);
    return v;
}
// PSGPU_FOR_N(stmt): stmt once for each point n < N (N <= 8, a template parameter in
// scope), unrolled by the preprocessor and `if constexpr` instead of a loop (the
// generated tree walks emit thousands of these; see psgpu_jit.cpp, Gen::FN).
#define PSGPU_N_AT(k, ...)                 \
    if constexpr (N > k) {                 \
        constexpr int n = k;               \
        __VA_ARGS__                        \
    }
#define PSGPU_FOR_N(...)                                                                              \
    {                                                                                                 \
        static_assert(N >= 1 && N <= 8, "PSGPU_FOR_N: 1..8 points per lane");                         \
        PSGPU_N_AT(0, __VA_ARGS__) PSGPU_N_AT(1, __VA_ARGS__) PSGPU_N_AT(2, __VA_ARGS__)              \
        PSGPU_N_AT(3, __VA_ARGS__) PSGPU_N_AT(4, __VA_ARGS__) PSGPU_N_AT(5, __VA_ARGS__)              \
        PSGPU_N_AT(6, __VA_ARGS__) PSGPU_N_AT(7, __VA_ARGS__)                                         \
    }

// Value of a wave-uniform lane (scalar read).
__device__ __forceinline__ uint32_t lane_value(uint32_t v, int lane) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, lane);
}
// A value the wave holds in every lane, as a scalar (SGPR): branches on it are scalar, and
// the compiler sees the uniformity its divergence analysis cannot prove (e.g. anything
// derived from threadIdx.x >> 6).
#ifndef PSGPU_DEFER_ATOMICS
#define PSGPU_DEFER_ATOMICS 1  // 0: wait for the queue reservations' atomics where they return (A/B)
#endif
#ifndef PSGPU_UNIFORM_CM
#define PSGPU_UNIFORM_CM 1  // 0: k_mpu's culling mask in VGPRs (experiments)
#endif
#ifndef PSGPU_UNIFORM_WAVE
#define PSGPU_UNIFORM_WAVE 0  // 1: the wave index through readfirstlane -- 2 % slower with four
                              // engines (r04 A/B); kept as an experiment
#endif
__device__ __forceinline__ uint32_t uniform(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ int wave_index() {
    return PSGPU_UNIFORM_WAVE ? (int)uniform(threadIdx.x >> 6) : (int)(threadIdx.x >> 6);
}
__device__ __forceinline__ uint64_t uniform64(uint64_t v) {
    return (uint64_t)uniform((uint32_t)v) | ((uint64_t)uniform((uint32_t)(v >> 32)) << 32);
}

// ---------------------------------------------------------------------------
// Primitive fields.  dist2 per skeleton type, then Wyvill.
// PR: a DevPrim in the constant address space (parameters loaded at run time) or a
// constexpr BakedPrim (parameters compiled into the code, psgpu_jit.cpp mode 2).
struct BakedPrim {
    float pos[3], dir[3], res[3], col[3], mat[12];
};
struct BakedOp {
    float lo[3], hi[3], resY;
};

// Parameter groups of the generated walk (psgpu_jit.cpp, mode 1): the parameters a subtree's
// walk reads, loaded into SGPRs together at the subtree's entry, so the wave waits for its
// scalar loads once per group instead of once per primitive (every wait is lgkmcnt(0):
// scalar loads return out of order).  The empty asm statements pin each value in an SGPR
// there, so the loads are not sunk back to their first use.
template <int TYPE>
__device__ __forceinline__ constexpr bool prim_uses_dir() {
    return TYPE == PSGPU_T_LINE || TYPE == PSGPU_T_CYLINDER || TYPE == PSGPU_T_DISC || TYPE == PSGPU_T_RING;
}
template <int TYPE>
__device__ __forceinline__ constexpr int prim_res_count() {
    return TYPE == PSGPU_T_CYLINDER ? 2 : ((TYPE == PSGPU_T_CUBE || TYPE == PSGPU_T_DISC || TYPE == PSGPU_T_RING) ? 1 : 0);
}
template <int TYPE>
__device__ __forceinline__ constexpr bool prim_uses_pos() {
    return TYPE == PSGPU_T_POINT || TYPE == PSGPU_T_LINE || TYPE == PSGPU_T_CYLINDER || TYPE == PSGPU_T_CUBE ||
           TYPE == PSGPU_T_DISC || TYPE == PSGPU_T_RING;
}
#define PSGPU_PIN(v) asm volatile("" ::"s"(v))
template <int TYPE, bool MAT>
__device__ __forceinline__ void load_prim(CPrim& S, BakedPrim& r) {
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        if (prim_uses_pos<TYPE>()) r.pos[k] = S.pos[k];
        if (prim_uses_dir<TYPE>()) r.dir[k] = S.dir[k];
        if (k < prim_res_count<TYPE>()) r.res[k] = S.res[k];
    }
    if (MAT) {
#pragma unroll
        for (int k = 0; k < 12; ++k) r.mat[k] = S.mat[k];
    }
}
template <int TYPE, bool MAT>
__device__ __forceinline__ void pin_prim(const BakedPrim& r) {
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        if (prim_uses_pos<TYPE>()) PSGPU_PIN(r.pos[k]);
        if (prim_uses_dir<TYPE>()) PSGPU_PIN(r.dir[k]);
        if (k < prim_res_count<TYPE>()) PSGPU_PIN(r.res[k]);
    }
    if (MAT) {
#pragma unroll
        for (int k = 0; k < 12; ++k) PSGPU_PIN(r.mat[k]);
    }
}
template <class OP>
__device__ __forceinline__ void load_op(OP& S, BakedOp& r) {
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        r.lo[k] = S.lo[k];
        r.hi[k] = S.hi[k];
    }
}
__device__ __forceinline__ void pin_op(const BakedOp& r) {
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        PSGPU_PIN(r.lo[k]);
        PSGPU_PIN(r.hi[k]);
    }
}

template <int TYPE, class PR>
__device__ __forceinline__ float prim_dist2(PR& P, float x, float y, float z) {
    float d2 = 0.0f;
    if (TYPE == PSGPU_T_POINT) {  // :975-983
        float dx = P.pos[0] - x, dy = P.pos[1] - y, dz = P.pos[2] - z;
        d2 = (dx * dx + dy * dy) + dz * dz;
    } else if (TYPE == PSGPU_T_LINE) {  // :984-1011 (pos = start, dir = end), not clamped
        float l0x = P.pos[0], l0y = P.pos[1], l0z = P.pos[2];
        float ldx = P.dir[0] - l0x, ldy = P.dir[1] - l0y, ldz = P.dir[2] - l0z;
        float ldd = (ldx * ldx + ldy * ldy) + ldz * ldz;
        float dx = x - l0x, dy = y - l0y, dz = z - l0z;
        float t = (dx * ldx + dy * ldy) + dz * ldz;
        t = t / ldd;
        dx = x - (l0x + t * ldx);
        dy = y - (l0y + t * ldy);
        dz = z - (l0z + t * ldz);
        d2 = (dx * dx + dy * dy) + dz * dz;
    } else if (TYPE == PSGPU_T_CYLINDER) {  // :1012-1039 (axis dir, r = resX, h = resY)
        float px = x - P.pos[0], py = y - P.pos[1], pz = z - P.pos[2];
        float yy = (px * P.dir[0] + py * P.dir[1]) + pz * P.dir[2];
        float rr = ((px * px + py * py) + pz * pz) - yy * yy;
        float xx = max_ref(0.0f, sqrtf(rr) - P.res[0]);
        float mask = m01(yy > 0.0f);
        yy = mask * max_ref(0.0f, yy - P.res[1]) + (1.0f - mask) * yy;
        d2 = xx * xx + yy * yy;
    } else if (TYPE == PSGPU_T_TRIANGLE) {  // :1040-1057 distance stub
        d2 = 3.402823466e+38f;
    } else if (TYPE == PSGPU_T_CUBE) {  // :1059-1097 (half side resX)
        float side = P.res[0], mside = -1.0f * P.res[0];
        float dif[3] = {x - P.pos[0], y - P.pos[1], z - P.pos[2]};
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            float mm = m01(mside > dif[a]);
            float mp = m01(dif[a] > side);
            float dl = (dif[a] + side) * mm + (dif[a] - side) * mp;
            d2 = (a == 0) ? dl * dl : d2 + dl * dl;
        }
    } else if (TYPE == PSGPU_T_DISC) {  // :1099-1132
        float dX = x - P.pos[0], dY = y - P.pos[1], dZ = z - P.pos[2];
        float nX = P.dir[0], nY = P.dir[1], nZ = P.dir[2], r = P.res[0];
        float dot = (nX * dX + nY * dY) + nZ * dZ;
        float rX = dX - nX * dot, rY = dY - nY * dot, rZ = dZ - nZ * dot;
        dot = (rX * rX + rY * rY) + rZ * rZ;
        float rs = 1.0f / sqrtf(dot);  // _mm_rsqrt_ps in the reference (vendor specific)
        rX = rX * rs; rY = rY * rs; rZ = rZ * rs;
        nX = r * rX - dX; nY = r * rY - dY; nZ = r * rZ - dZ;
        float mask = m01(r * r >= dot);
        d2 = mask * (((dX * dX + dY * dY) + dZ * dZ) - dot) + (1.0f - mask) * ((nX * nX + nY * nY) + nZ * nZ);
    } else if (TYPE == PSGPU_T_RING) {  // :1134-1173
        float dX = x - P.pos[0], dY = y - P.pos[1], dZ = z - P.pos[2];
        float nX = P.dir[0], nY = P.dir[1], nZ = P.dir[2], r = P.res[0];
        float dot = (nX * dX + nY * dY) + nZ * dZ;
        float rX = dX - nX * dot, rY = dY - nY * dot, rZ = dZ - nZ * dot;
        dot = (rX * rX + rY * rY) + rZ * rZ;
        float mask = m01(dot == 0.0f);
        dot = 1.0f / sqrtf(dot);
        rX = rX * dot; rY = rY * dot; rZ = rZ * dot;
        nX = r * rX - dX; nY = r * rY - dY; nZ = r * rZ - dZ;
        d2 = mask * (((r * r + dX * dX) + dY * dY) + dZ * dZ) + (1.0f - mask) * ((nX * nX + nY * nY) + nZ * nZ);
    }
    // any other code: no case in the reference switch, dist2 stays 0 (field 1)
    return d2;
}

__device__ __forceinline__ float wyvill(float d2) {
    float t = 1.0f - d2;
    float f = (t * t) * t;
    return max_ref(0.0f, f);
}

template <int TYPE, bool MAT, class PR>
__device__ __forceinline__ float prim_field_t(PR& P, float pX, float pY, float pZ) {
    float x = pX, y = pY, z = pZ;
    if (MAT) {  // :948-970, rows ((m0*x + m1*y) + m2*z) + m3
        x = ((P.mat[0] * pX + P.mat[1] * pY) + P.mat[2] * pZ) + P.mat[3];
        y = ((P.mat[4] * pX + P.mat[5] * pY) + P.mat[6] * pZ) + P.mat[7];
        z = ((P.mat[8] * pX + P.mat[9] * pY) + P.mat[10] * pZ) + P.mat[11];
    }
    return wyvill(prim_dist2<TYPE, PR>(P, x, y, z));
}

// run-time dispatch (interpreter)
__device__ __forceinline__ float prim_field(CPrim& P, float pX, float pY, float pZ) {
    float x = pX, y = pY, z = pZ;
    if (P.hasMatrix) {
        x = ((P.mat[0] * pX + P.mat[1] * pY) + P.mat[2] * pZ) + P.mat[3];
        y = ((P.mat[4] * pX + P.mat[5] * pY) + P.mat[6] * pZ) + P.mat[7];
        z = ((P.mat[8] * pX + P.mat[9] * pY) + P.mat[10] * pZ) + P.mat[11];
    }
    float d2;
    switch (P.type) {
    case PSGPU_T_POINT: d2 = prim_dist2<PSGPU_T_POINT, CPrim>(P, x, y, z); break;
    case PSGPU_T_LINE: d2 = prim_dist2<PSGPU_T_LINE, CPrim>(P, x, y, z); break;
    case PSGPU_T_CYLINDER: d2 = prim_dist2<PSGPU_T_CYLINDER, CPrim>(P, x, y, z); break;
    case PSGPU_T_TRIANGLE: d2 = prim_dist2<PSGPU_T_TRIANGLE, CPrim>(P, x, y, z); break;
    case PSGPU_T_CUBE: d2 = prim_dist2<PSGPU_T_CUBE, CPrim>(P, x, y, z); break;
    case PSGPU_T_DISC: d2 = prim_dist2<PSGPU_T_DISC, CPrim>(P, x, y, z); break;
    case PSGPU_T_RING: d2 = prim_dist2<PSGPU_T_RING, CPrim>(P, x, y, z); break;
    default: d2 = 0.0f; break;
    }
    return wyvill(d2);
}

// Binary op field (:1282-1338); `last` is the previous op's field (stale outField).
__device__ __forceinline__ float op_field(uint32_t type, float lf, float rf, float resY, float last) {
    switch (type) {
    case PSGPU_T_BLEND: return lf + rf;
    case PSGPU_T_RICCI: {  // fast_pow, PS_SIMDVecN.h:122-128 (rcp -> IEEE 1/x)
        const float base = lf + rf;
        float den = resY * base;
        den = resY - den;
        den = base + den;
        return base * (1.0f / den);
    }
    case PSGPU_T_UNION: return max_ref(lf, rf);
    case PSGPU_T_INTERSECT: return min_ref(lf, rf);
    case PSGPU_T_DIF: return min_ref(lf, 1.0f - rf);
    case PSGPU_T_SMOOTHDIF: return lf * (1.0f - rf);
    case 22: case 23: case 24: case 25: return lf;  // warps: identity
    default: return last;
    }
}

// Op colour weights (:1472-1522); returns false when the op keeps a colour instead.
__device__ __forceinline__ bool op_colour_weights(uint32_t type, float lf, float rf, float v, float* wl, float* wr) {
    switch (type) {
    case PSGPU_T_BLEND: case PSGPU_T_RICCI:
        *wl = 2.0f * (0.5f + lf) - 1.0f;
        *wr = 2.0f * (0.5f + rf) - 1.0f;
        return true;
    case PSGPU_T_UNION: case PSGPU_T_INTERSECT:
        *wl = m01((v - lf) == 0.0f);
        *wr = m01((v - rf) == 0.0f);
        return true;
    case PSGPU_T_DIF: case PSGPU_T_SMOOTHDIF:
        *wl = m01(lf == v);
        *wr = m01((1.0f - rf) == v);
        return true;
    default:
        return false;
    }
}

// ---------------------------------------------------------------------------
// Exact culling (never changes a bit of output).  A primitive whose support cannot
// reach any point of the wave has computed dist2 >= 1, i.e. field exactly +0, and
// is not evaluated.  Every cullable primitive has a skeleton segment (CullSeg) whose
// distance minus a radius bounds its distance from below and is 1-Lipschitz: Point
// (a point), infinite Line (an unbounded segment), capped Cylinder with |axis| = 1
// (its axis segment, radius r), axis-aligned Cube (its centre, radius s*sqrt(3)).  For
// the wave's AABB with centre c and half-diagonal h every point q then has
// d(q) >= d(c) - h.  The host marks a prim cullable only without a matrix and with
// finite, well-conditioned parameters; Cylinder also needs the AABB clear of its
// infinite axis (where the reference's sqrt of a rounded-negative value is NaN).  The
// margin d^2 >= 1.02 covers fp32 rounding of the reference formulas by orders of
// magnitude.  Triangle is a constant +0 (dist2 = FLT_MAX) and is always culled.
struct CullMask {
    uint64_t lo, hi;
};

// This lane's culling segments (prims `lane` and 64 + `lane`), loaded once and early: the
// loads do not depend on the box, so they overlap the rest of a kernel's prologue.
struct CullLanes {
    CullSeg s[2];
    bool two;  // ctPrims > 64
};

__device__ __forceinline__ CullSeg load_cullseg(ModelPtr M, int i) {
    typedef const __attribute__((address_space(4))) float* CF;
    const CF f = (CF)(&M->cull[i]);  // 12 consecutive floats: the compiler emits 16-B loads
    CullSeg S;
    S.a[0] = f[0]; S.a[1] = f[1]; S.a[2] = f[2];
    S.u[0] = f[3]; S.u[1] = f[4]; S.u[2] = f[5];
    S.invUU = f[6]; S.radius = f[7];
    S.tmin = f[8]; S.tmax = f[9]; S.axisClear = f[10]; S.pad = f[11];
    return S;
}

__device__ __forceinline__ CullLanes load_cull_lanes(ModelPtr M) {
    CullLanes L;
    L.two = M->ctPrims > 64u;
    L.s[0] = load_cullseg(M, lane_id());
    if (L.two) L.s[1] = load_cullseg(M, 64 + lane_id());
    return L;
}

// Is the segment's primitive exactly +0 over the box (centre c, half-diagonal h)?
__device__ __forceinline__ bool cull_one(const CullSeg& S, float cx, float cy, float cz, float h) {
    const float dx = cx - S.a[0], dy = cy - S.a[1], dz = cz - S.a[2];
    const float t = (dx * S.u[0] + dy * S.u[1] + dz * S.u[2]) * S.invUU;
    const float lx = dx - t * S.u[0], ly = dy - t * S.u[1], lz = dz - t * S.u[2];
    const float lineDist = __builtin_amdgcn_sqrtf(lx * lx + ly * ly + lz * lz);
    const float tc = fminf(fmaxf(t, S.tmin), S.tmax);
    const float ex = dx - tc * S.u[0], ey = dy - tc * S.u[1], ez = dz - tc * S.u[2];
    const float d = (__builtin_amdgcn_sqrtf(ex * ex + ey * ey + ez * ez) - S.radius) - h;
    return d > 0.0f && d * d >= 1.02f && (lineDist - h > S.axisClear);
}

__device__ __forceinline__ CullMask cull_mask_from(const CullLanes& L, float x0, float y0, float z0, float x1,
                                                   float y1, float z1) {
    CullMask cm{0ull, 0ull};
    if (!(x1 - x0 < 1e30f && y1 - y0 < 1e30f && z1 - z0 < 1e30f)) return cm;
    const float cx = 0.5f * (x0 + x1), cy = 0.5f * (y0 + y1), cz = 0.5f * (z0 + z1);
    const float hx = 0.5f * (x1 - x0), hy = 0.5f * (y1 - y0), hz = 0.5f * (z1 - z0);
    const float h = __builtin_amdgcn_sqrtf(hx * hx + hy * hy + hz * hz) * 1.0001f + 1e-6f;
    cm.lo = ballot(cull_one(L.s[0], cx, cy, cz, h));
    if (L.two) cm.hi = ballot(cull_one(L.s[1], cx, cy, cz, h));
    return cm;
}

__device__ __forceinline__ CullMask cull_mask_box(ModelPtr M, float x0, float y0, float z0, float x1, float y1,
                                                  float z1) {
    return cull_mask_from(load_cull_lanes(M), x0, y0, z0, x1, y1, z1);
}

// Cull mask for the AABB of this wave's points (all 64 lanes must participate),
// optionally grown by `ext` on the high side of every axis.
__device__ __forceinline__ CullMask cull_mask_points(const CullLanes& L, float px, float py, float pz, bool enable,
                                                     float ext = 0.0f) {
    if (!enable) return CullMask{0ull, 0ull};
    // a NaN coordinate (fminf/fmaxf would hide it) disables culling for the wave
    if (ballot(!(px == px) || !(py == py) || !(pz == pz)) != 0ull) return CullMask{0ull, 0ull};
    return cull_mask_from(L, wave_min(px), wave_min(py), wave_min(pz), wave_max(px) + ext, wave_max(py) + ext,
                          wave_max(pz) + ext);
}
__device__ __forceinline__ CullMask cull_mask_points(ModelPtr M, float px, float py, float pz, bool enable,
                                                     float ext = 0.0f) {
    if (!enable) return CullMask{0ull, 0ull};
    return cull_mask_points(load_cull_lanes(M), px, py, pz, true, ext);
}

__device__ __forceinline__ bool culled(const CullMask& cm, uint32_t i) {
    return i < 64 ? ((cm.lo >> i) & 1ull) : ((cm.hi >> (i - 64)) & 1ull);
}

// ---------------------------------------------------------------------------
// Field bounds over a box of lattice corners (k_precheck).  Most MPUs that pass S1 have
// no surface: every S2 corner is inside or every one is outside, and S2 only discards
// them (PS_Polygonizer.cpp:602-609).  An interval [lo, hi] of the field over the MPU's
// corners decides that outcome without evaluating them: hi < 0.5 (no corner inside)
// or lo >= 0.5 (no corner outside) gives exactly the reference result, 0 vertices and
// 0 triangles.  The bound is conservative by construction:
//  * each primitive's distance (Point, infinite Line, capped Cylinder, Cube: the same
//    functions the reference evaluates, all true Euclidean distances, 1-Lipschitz) is
//    evaluated at the box centre and widened by the half-diagonal h (+ 1e-4 and a
//    relative 1e-4); Wyvill is monotone in the distance; the field interval is widened
//    by kBoundEps, orders of magnitude above the fp32 rounding of either evaluation;
//  * ops are monotone interval maps (Blend, Union, Intersect, Dif, SmoothDif, warps);
//  * op-box pruning (depth > 3) is decided per quad of 4 z-consecutive corners: from
//    the box's exact corner coordinates the op is pruned for every quad (field 0),
//    for none (the op's interval), or for some (the interval joined with 0).
// Only models whose used primitives all have finite, well-conditioned parameters, no
// matrix, and a type above (or Triangle, field 0) are bounded (DevModel::boundable, set
// by the host; Ricci and unknown ops are excluded), so no corner can be NaN -- except a
// Cylinder on its own axis, where the bound gives up (ok = false) within 0.05 of it.
constexpr float kBoundEps = 2e-4f;

struct BoundBox {
    float cx, cy, cz, h;       // centre, half-diagonal (with margin)
    float xs[4], ys[4], zs[4]; // the box's corner coordinates per axis (z: one S2 quad)
};

template <int TYPE, class PR>
__device__ __forceinline__ float prim_true_dist(PR& P, float x, float y, float z, float* axisD) {
    float d2 = 0.0f;
    if (TYPE == PSGPU_T_POINT) {
        const float dx = x - P.pos[0], dy = y - P.pos[1], dz = z - P.pos[2];
        d2 = dx * dx + dy * dy + dz * dz;
    } else if (TYPE == PSGPU_T_LINE) {  // distance from the infinite line (the reference does not clamp)
        const float ux = P.dir[0] - P.pos[0], uy = P.dir[1] - P.pos[1], uz = P.dir[2] - P.pos[2];
        const float dx = x - P.pos[0], dy = y - P.pos[1], dz = z - P.pos[2];
        const float t = (dx * ux + dy * uy + dz * uz) / (ux * ux + uy * uy + uz * uz);
        const float ex = dx - t * ux, ey = dy - t * uy, ez = dz - t * uz;
        d2 = ex * ex + ey * ey + ez * ez;
    } else if (TYPE == PSGPU_T_CYLINDER) {  // solid cylinder: axis dir (unit), radius res0, height res1
        const float px = x - P.pos[0], py = y - P.pos[1], pz = z - P.pos[2];
        float yy = px * P.dir[0] + py * P.dir[1] + pz * P.dir[2];
        const float rr = px * px + py * py + pz * pz - yy * yy;
        const float r = __builtin_amdgcn_sqrtf(rr > 0.0f ? rr : 0.0f);
        *axisD = r;
        const float xx = fmaxf(r - P.res[0], 0.0f);
        yy = yy > 0.0f ? fmaxf(yy - P.res[1], 0.0f) : yy;
        d2 = xx * xx + yy * yy;
    } else if (TYPE == PSGPU_T_CUBE) {
        const float ex = fmaxf(fabsf(x - P.pos[0]) - P.res[0], 0.0f);
        const float ey = fmaxf(fabsf(y - P.pos[1]) - P.res[0], 0.0f);
        const float ez = fmaxf(fabsf(z - P.pos[2]) - P.res[0], 0.0f);
        d2 = ex * ex + ey * ey + ez * ez;
    }
    return __builtin_amdgcn_sqrtf(d2);
}

__device__ __forceinline__ float wyvill_of_dist(float d) {
    const float t = 1.0f - d * d;
    return t > 0.0f ? (t * t) * t : 0.0f;
}

// Field interval of one primitive over the box (TYPE: Point, Line, Cylinder or Cube).
template <int TYPE, class PR>
__device__ __forceinline__ void prim_bound(PR& P, const BoundBox& B, float* lo, float* hi, bool* ok) {
    float axisD = 1e30f;
    const float d = prim_true_dist<TYPE, PR>(P, B.cx, B.cy, B.cz, &axisD);
    if (TYPE == PSGPU_T_CYLINDER) *ok = *ok && (axisD - B.h > 0.05f);
    *hi = wyvill_of_dist(fmaxf(d - B.h, 0.0f)) + kBoundEps;
    *lo = wyvill_of_dist(d + B.h) - kBoundEps;
}

// Interval of a binary op (the monotone maps of op_field; Ricci/unknown types are not bounded).
__device__ __forceinline__ void bound_op(uint32_t type, float ll, float lh, float rl, float rh, float* lo, float* hi) {
    switch (type) {
    case PSGPU_T_BLEND: *lo = ll + rl; *hi = lh + rh; break;
    case PSGPU_T_UNION: *lo = fmaxf(ll, rl); *hi = fmaxf(lh, rh); break;
    case PSGPU_T_INTERSECT: *lo = fminf(ll, rl); *hi = fminf(lh, rh); break;
    case PSGPU_T_DIF: *lo = fminf(ll, 1.0f - rh); *hi = fminf(lh, 1.0f - rl); break;
    case PSGPU_T_SMOOTHDIF: {
        const float a = 1.0f - rh, b = 1.0f - rl;
        const float p0 = ll * a, p1 = ll * b, p2 = lh * a, p3 = lh * b;
        *lo = fminf(fminf(p0, p1), fminf(p2, p3));
        *hi = fmaxf(fmaxf(p0, p1), fmaxf(p2, p3));
    } break;
    default: *lo = ll; *hi = lh; break;  // warps: the left child
    }
}

// Op-box pruning of a depth > 3 op over the box's quads: a quad (x, y, 4 z) is pruned
// iff x, y and all 4 z lie outside the op box on their axes (PS_Polygonizer.cpp:1239-1243).
template <class OR>
__device__ __forceinline__ void bound_prune(OR& b, const BoundBox& B, float* lo, float* hi) {
    bool anyZ = false, allX = true, noX = true, allY = true, noY = true;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        anyZ = anyZ | ((B.zs[i] >= b.lo[2]) & (b.hi[2] >= B.zs[i]));
        const bool ix = (B.xs[i] >= b.lo[0]) & (b.hi[0] >= B.xs[i]);
        const bool iy = (B.ys[i] >= b.lo[1]) & (b.hi[1] >= B.ys[i]);
        allX = allX & ix; noX = noX & !ix;
        allY = allY & iy; noY = noY & !iy;
    }
    if (!anyZ && noX && noY) {  // every quad pruned: field exactly 0
        *lo = 0.0f;
        *hi = 0.0f;
    } else if (!(anyZ || allX || allY)) {  // some quads pruned
        *lo = fminf(*lo, 0.0f);
        *hi = fmaxf(*hi, 0.0f);
    }
}

// ---------------------------------------------------------------------------
// Interpreter evaluator: the flattened walk program of psgpu_model.h.
//   GROUP 4: pruning decided per 4-lane group (S1/S2 quads, S4 edge samples)
//   GROUP 1: per lane (S5: the reference evaluates 4 identical lanes)
//   COLOR  : fieldValueAndColor's colour walk as well; no subtree is skipped and lanes
//            inside a pruned subtree see field 0 for its prims and ops (the
//            reference's never-written arrays, defined as zero).
// `sl` is this lane's value stack in LDS (stride 64 floats; colour: 4 floats per slot).
struct InterpEval {
    ModelPtr M;
    float* sl;
    __device__ InterpEval(ModelPtr m, float* slots) : M(m), sl(slots) {}

    template <int GROUP, bool COLOR>
    __device__ __forceinline__ float eval(float px, float py, float pz, const CullMask& cm, float* colOut) const {
        const int n = (int)M->nInstr;
        const bool noOps = M->ctOps == 0;
        int resume = 0;
        float last = 0.0f, acc = 0.0f;
        float lc0 = 0.0f, lc1 = 0.0f, lc2 = 0.0f;
        constexpr int SW = COLOR ? 4 : 1;
        for (int pc = 0; pc < n; ++pc) {
            const Instr I = load_instr(M, pc);
            const bool act = pc >= resume;
            if (I.kind == kEnter) {
                COp& O = M->ops[I.idx];
                bool in = ((px >= O.lo[0]) & (O.hi[0] >= px)) | ((py >= O.lo[1]) & (O.hi[1] >= py)) |
                          ((pz >= O.lo[2]) & (O.hi[2] >= pz));
                bool anyIn = group_any<GROUP>(act && in);
                bool prune = act && !anyIn;
                if (prune) {
                    resume = I.skipTo;
                    sl[(I.out * SW) * 64] = 0.0f;
                    last = 0.0f;
                }
                if (!COLOR) {
                    if (ballot(pc + 1 >= resume) == 0ull) pc = I.skipTo - 1;
                }
            } else if (I.kind == kPrim) {
                if (COLOR) {
                    float f = 0.0f;
                    if (act && !culled(cm, I.idx)) f = prim_field(M->prims[I.idx], px, py, pz);
                    sl[(I.out * SW) * 64] = f;
                } else if (act) {
                    float f = 0.0f;
                    if (!culled(cm, I.idx)) f = prim_field(M->prims[I.idx], px, py, pz);
                    sl[I.out * 64] = f;
                }
            } else if (I.kind == kOp) {
                if (COLOR || act) {
                    const float lf = sl[(I.lslot * SW) * 64];
                    const float rf = sl[(I.rslot * SW) * 64];
                    float v = op_field(I.type, lf, rf, M->ops[I.idx].resY, last);
                    if (COLOR && !act) v = 0.0f;
                    sl[(I.out * SW) * 64] = v;
                    if (act) last = v;
                    if (COLOR) {
                        float cl0, cl1, cl2, cr0, cr1, cr2;
                        if (I.childKind & 2) {
                            cl0 = sl[(I.lslot * 4 + 1) * 64]; cl1 = sl[(I.lslot * 4 + 2) * 64]; cl2 = sl[(I.lslot * 4 + 3) * 64];
                        } else {
                            CPrim& P = M->prims[I.L];
                            cl0 = P.col[0]; cl1 = P.col[1]; cl2 = P.col[2];
                        }
                        if (I.childKind & 1) {
                            cr0 = sl[(I.rslot * 4 + 1) * 64]; cr1 = sl[(I.rslot * 4 + 2) * 64]; cr2 = sl[(I.rslot * 4 + 3) * 64];
                        } else {
                            CPrim& P = M->prims[I.R];
                            cr0 = P.col[0]; cr1 = P.col[1]; cr2 = P.col[2];
                        }
                        float wl, wr;
                        if (op_colour_weights(I.type, lf, rf, v, &wl, &wr)) {
                            lc0 = wl * cl0 + wr * cr0;
                            lc1 = wl * cl1 + wr * cr1;
                            lc2 = wl * cl2 + wr * cr2;
                        } else if (I.type >= 22 && I.type <= 25) {
                            lc0 = cl0; lc1 = cl1; lc2 = cl2;
                        }
                        sl[(I.out * 4 + 1) * 64] = lc0;
                        sl[(I.out * 4 + 2) * 64] = lc1;
                        sl[(I.out * 4 + 3) * 64] = lc2;
                    }
                }
            } else {  // kSumPrim
                float f = 0.0f;
                if (!culled(cm, I.idx)) f = prim_field(M->prims[I.idx], px, py, pz);
                acc = acc + f;
            }
        }
        if (COLOR) {
            if (noOps) {
                CPrim& P = M->prims[0];
                lc0 = P.col[0]; lc1 = P.col[1]; lc2 = P.col[2];
            }
            colOut[0] = lc0;
            colOut[1] = lc1;
            colOut[2] = lc2;
        }
        return noOps ? acc : last;
    }

    template <int GROUP, bool COLOR, int N>
    __device__ __forceinline__ void evaln(const float* px, const float* py, const float* pz, const CullMask& cm,
                                          float* out, float* colOut) const {
        static_assert(GROUP != 0, "the interpreter prunes per lane group, not per lane's points");
        for (int n = 0; n < N; ++n)
            out[n] = eval<GROUP, COLOR>(px[n], py[n], pz[n], cm, COLOR ? colOut + 3 * n : nullptr);
    }

    // field bounds are generated per tree (psgpu_jit.cpp); the interpreter never proves
    __device__ __forceinline__ void bound(const BoundBox&, const CullMask&, float* lo, float* hi, bool* ok) const {
        *lo = 0.0f;
        *hi = 0.0f;
        *ok = false;
    }
};

// ---------------------------------------------------------------------------
// Per-wave timeline (the reference's MPUSTATS / PrintThreadResults, PS_Polygonizer.h:201-207,
// .cpp:414-461, with waves for threads): when p.stamps is set every wave of kernel K
// records {start, end, item | hw id << 32} in the 100 MHz s_memrealtime clock, item = the
// MPU a k_mpu wave polygonized (0xffffffff: none) or the wave's global index.
__device__ __forceinline__ uint64_t stamp_now() { return __builtin_amdgcn_s_memrealtime(); }
__device__ __forceinline__ void stamp_end(const Params& p, int K, uint64_t t0, uint32_t item,
                                          const uint32_t blk = blockIdx.x) {
    const uint32_t w = blk * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (w >= p.stampCap) return;
    const uint64_t t1 = stamp_now();
    // HW_ID (CU, SIMD, SE; 32 bits) and XCC_ID (hwreg 20) as one word: hwid[15:0] | xcc << 16
    const uint32_t hw = (uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 4);
    const uint32_t xcc = (uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 20) & 15u;
    if (lane_id() == 0) {
        uint64_t* r = p.stamps + 3 * ((size_t)K * p.stampCap + w);
        r[0] = t0;
        r[1] = t1;
        r[2] = (uint64_t)item | ((uint64_t)((hw & 0xffffu) | (xcc << 16)) << 32);
    }
}
// Phase stamps inside one wave (debug bit 4096: k_mpu, 8192: k_precheck): 8 words per
// wave after the kernels' records; phase 0 = entry.
__device__ __forceinline__ void phase_stamp(const Params& p, int ph, uint32_t bit = 4096u) {
    if (!(p.debug & bit) || !p.stamps) return;
    const uint32_t w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (w >= p.stampCap) return;
    const uint64_t t = stamp_now();
    if (lane_id() == 0) p.stamps[3 * (size_t)kNumStampKernels * p.stampCap + 8 * (size_t)w + ph] = t;
}
// The same, taken only once `dep` has been computed (inline asm keeps the clock read after its
// producer and in program order with the other stamps): phases of k_finish (debug bit 2048;
// the stamps change the kernel's registers, so they exist only when PSGPU_FIN_PHASES is 1).
#ifndef PSGPU_MPU_LIVE_STAMP
#define PSGPU_MPU_LIVE_STAMP 0  // k_mpu's live-primitive word: measurement builds only (PSGPU_JIT_FLAGS)
#endif
#ifndef PSGPU_FIN_PHASES
#define PSGPU_FIN_PHASES 0  // compiled in only for the measurement (PSGPU_JIT_FLAGS=-DPSGPU_FIN_PHASES=1)
#endif
__device__ __forceinline__ void phase_stamp_after(const Params& p, int ph, uint32_t bit, float dep) {
    if (!PSGPU_FIN_PHASES || !(p.debug & bit) || !p.stamps) return;
    const uint32_t w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (w >= p.stampCap) return;
    uint64_t t;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) : "v"(dep));
    if (lane_id() == 0) p.stamps[3 * (size_t)kNumStampKernels * p.stampCap + 8 * (size_t)w + ph] = t;
}
// A kernel's span in one run (PSGPU_OPT_SPANS): every wave folds its start / end into one of
// 64 {min start, max end} pairs of the run's slot (chosen by block, so no address sees more
// than 1/64 of the waves' atomics); the host reduces the 64 pairs to the first wave start and
// the last wave end on the device clock.
__device__ __forceinline__ void span_end(const Params& p, int K, uint64_t t0) {
    const uint64_t t1 = stamp_now();
    if (lane_id() == 0) {
        uint64_t* s = p.spans + 2 * ((size_t)K * kSpanLanes + (blockIdx.x & (kSpanLanes - 1)));
        atomicMin(reinterpret_cast<unsigned long long*>(s), (unsigned long long)t0);
        atomicMax(reinterpret_cast<unsigned long long*>(s + 1), (unsigned long long)t1);
    }
}
// The reference's per-MPU MPUSTATS ticks (PS_Polygonizer.cpp:449-461: tickStart / tickEnd
// around process_cells_simd, the thread id), PSGPU_OPT_MPU_TICKS: the wave that ran S1 for
// the MPU records its start and end (k_precheck, lane g < 8 of the brick's MPU g), the wave
// that ran S2-S3 and made its vertex / triangle records raises the end (k_mpu).
__device__ __forceinline__ uint32_t wave_hw_id() {
    const uint32_t hw = (uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 4);
    const uint32_t xcc = (uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 20) & 15u;
    return (hw & 0xffffu) | (xcc << 16);
}
__device__ __forceinline__ void mpu_ticks_s1(const Params& p, uint32_t w, uint64_t t0) {
    uint64_t* r = p.mpuTicks + 4 * (size_t)w;
    r[0] = t0;
    r[1] = stamp_now();
    r[2] = 0ull;
    r[3] = (uint64_t)wave_hw_id();
}
__device__ __forceinline__ void mpu_ticks_s2(const Params& p, uint32_t m) {
    const uint64_t t = stamp_now();
    const uint32_t hw = wave_hw_id();
    if (lane_id() == 0) {
        uint64_t* r = p.mpuTicks + 4 * (size_t)(m - p.mpuBegin);
        atomicMax(reinterpret_cast<unsigned long long*>(r + 2), (unsigned long long)t);
        reinterpret_cast<uint32_t*>(r + 3)[1] = hw;
    }
}
#define PSGPU_STAMPED(K, ITEM, CALL)                                             \
    {                                                                             \
        const uint64_t t0_ = (p.stamps || p.spans) ? psgpu::stamp_now() : 0ull;  \
        uint32_t item_ = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);     \
        CALL;                                                                     \
        if (K == 1 && p.mpuTicks && ITEM != 0xffffffffu) psgpu::mpu_ticks_s2(p, ITEM); \
        if (p.stamps) psgpu::stamp_end(p, K, t0_, ITEM);                          \
        if (p.spans) psgpu::span_end(p, K, t0_);                                  \
    }

// ---------------------------------------------------------------------------
// Exact m / d from a multiply-high by floor((2^32 - 1) / d): the estimate never exceeds the
// quotient and falls short of it by at most 2.
__device__ __forceinline__ uint32_t div_by(uint32_t m, uint32_t d, uint32_t magic, uint32_t* rem) {
    uint32_t q = __umulhi(m, magic);
    uint32_t r = m - q * d;
    if (r >= d) { ++q; r -= d; }
    if (r >= d) { ++q; r -= d; }
    *rem = r;
    return q;
}

__device__ __forceinline__ void mpu_origin(const Params& p, uint32_t m, float o[3]) {
    uint32_t k, jk;
    const uint32_t i = div_by(m, p.dims[2] * p.dims[1], p.divMagic[1], &jk);
    const uint32_t j = div_by(jk, p.dims[2], p.divMagic[0], &k);
    o[0] = p.lo[0] + (float)i * p.side;
    o[1] = p.lo[1] + (float)j * p.side;
    o[2] = p.lo[2] + (float)k * p.side;
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) { return lane_value(wave_incl_scan(v), 63); }

// S1: 8 corners per MPU, lanes 0-3 z = lo, lanes 4-7 z = lo + side; (x,y) lanes
// (0,0),(1,0),(0,1),(1,1) (PS_Polygonizer.cpp:488-519).  One wavefront = one 2x2x2
// brick of MPUs (lanes 8g..8g+7: MPU g = bx*4 + by*2 + bz), so the wave's culling box
// is compact.  Failing MPUs get count 0 here; survivors are appended to the sharded
// queue pq (one atomic per wave; waves [s*K, (s+1)*K) with K = pShardCap / 8 append to
// shard s, so a shard cannot overflow).  k_mpu takes them in any order: the mesh order
// comes from the scan of the per-MPU counts (in k_vertex).
// SPLIT 2 (tree split, TreeEval::kSplit): two waves per brick, one per subtree of the root
// (evaln_part / bound_part), their values exchanged through LDS and combined by both
// (combine / bound_combine): the same values, half the walk per wave -- for launches whose
// span is the heaviest brick's walk (small rank shares, a single engine).  Every wave of the
// block reaches both barriers; the second wave of a brick stops after them.
// k_front's tag of this run's queue entries: never 0 (the ready words start zeroed, and are
// zeroed again whenever the counter sets restart from epoch 0)
__device__ __forceinline__ uint32_t front_tag(const Params& p) { return p.ctr->epoch + 1u; }

template <class EV, int SPLIT = 1, bool FRONT = false>
__device__ __forceinline__ void precheck_body(const Params& p, float* lds) {
    const int wave = wave_index();
    const int lane = lane_id();
    const int part = wave % SPLIT;  // subtree of the root this wave walks (SPLIT 2)
    const int slot = wave / SPLIT;  // the block's brick
    phase_stamp(p, 0, 8192u);
    const uint64_t tick0 = p.mpuTicks ? stamp_now() : 0ull;  // MPUSTATS tickStart
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        // the words k_surface only ever raises (its wait's timeout, from any wave, after block 0
        // published the rest): cleared here, before any kernel of the run can raise them
        p.hostCtr->surfaceErr = 0u;
        p.totals[7] = 0u;
    }
    EV ev(as_const(p.model), lds + wave * p.slotsPerLane * 64 + lane);
    CullLanes cl;  // loaded first: independent of everything below
    if (p.cull) cl = load_cull_lanes(as_const(p.model));
    const uint32_t W = blockIdx.x * (4u / SPLIT) + (uint32_t)slot;  // brick slot: decides the queue shard
    const uint32_t bzN = p.brickDims[2], byN = p.brickDims[1];
    const uint32_t nBricks = p.brickDims[0] * byN * bzN;
    const uint32_t B = W < nBricks ? (uint32_t)(((uint64_t)W * p.brickStride) % nBricks) : W;  // its brick
    const uint32_t g = (uint32_t)lane >> 3;
    const uint32_t mi = 2u * (p.brickI0 + B / (byN * bzN)) + ((g >> 2) & 1u);
    const uint32_t mj = 2u * ((B / bzN) % byN) + ((g >> 1) & 1u);
    const uint32_t mk = 2u * (B % bzN) + (g & 1u);
    const uint32_t mg = (mi * p.dims[1] + mj) * p.dims[2] + mk;
    const bool valid = W < nBricks && mi < p.dims[0] && mj < p.dims[1] && mk < p.dims[2] && mg >= p.mpuBegin &&
                       mg - p.mpuBegin < p.mpuCount;
    // A lane without an MPU of the range (a brick over the lattice's high faces or a range
    // end) takes the origin of the nearest lattice MPU, so the wave's culling box stays the
    // brick's: with MPU 0's origin there, the box of each of C3's 1,027 face bricks spans
    // the domain, every primitive stays live and those waves walk 3-5x longer (r03 timeline).
    const uint32_t ci = min(mi, p.dims[0] - 1u), cj = min(mj, p.dims[1] - 1u), ck = min(mk, p.dims[2] - 1u);
    const uint32_t m = valid ? mg : (ci * p.dims[1] + cj) * p.dims[2] + ck;
    float o[3];
    mpu_origin(p, m, o);
    const int c = lane & 7;
    const float X = (float)(c & 1), Y = (float)((c >> 1) & 1), Z = (float)(c >> 2);
    const float px = X * p.side + o[0];
    const float py = Y * p.side + o[1];
    const float pz = Z * p.side + o[2];
    float f = -1.0f;
    CullMask cm{0ull, 0ull};
    if constexpr (SPLIT == 2) {
        __shared__ float sF[4][64];
        cm = cull_mask_points(cl, px, py, pz, p.cull != 0);
        float fp = -1.0f;
        if (!(p.debug & 8u)) {
            if (part == 0) ev.template evaln_part<4, false, 1, 0>(&px, &py, &pz, cm, &fp, nullptr);
            else ev.template evaln_part<4, false, 1, 1>(&px, &py, &pz, cm, &fp, nullptr);
        }
        sF[wave][lane] = fp;
        __syncthreads();
        const float rv = sF[slot * 2][lane], lv = sF[slot * 2 + 1][lane];
        if (!(p.debug & 8u)) ev.template combine<false, 1>(&rv, nullptr, &lv, nullptr, cm, &f, nullptr);
    } else if (!(p.debug & 8u)) {  // ablation bit 3: S1 without the walk (nothing passes)
        cm = cull_mask_points(cl, px, py, pz, p.cull != 0);
        f = ev.template eval<4, false>(px, py, pz, cm, nullptr);
    } else if (p.debug & 16u) {  // bit 4: the culling mask only
        cm = cull_mask_points(cl, px, py, pz, p.cull != 0);
        f = (float)(cm.lo & 1ull) - 1.0f;
    }
    const uint64_t bal = ballot(valid && f > 0.0f);
    phase_stamp(p, 1, 8192u);
    if ((p.debug & 8192u) && p.stamps && lane == 0) {  // phase word 7: the wave's live primitives, S1 passes
        const uint32_t w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
        if (w < p.stampCap)
            p.stamps[3 * (size_t)kNumStampKernels * p.stampCap + 8 * (size_t)w + 7] =
                (uint64_t)(128 - __popcll(cm.lo) - __popcll(cm.hi)) | ((uint64_t)__popcll(bal) << 16);
    }
    uint32_t flags8 = 0;  // bit g: MPU of lanes 8g..8g+7 passed
#pragma unroll
    for (int q = 0; q < 8; ++q) flags8 |= (((bal >> (8 * q)) & 0xffull) != 0ull ? 1u : 0u) << q;
    // Survivors proven empty by field bounds (see prim_bound): lane c of an MPU bounds
    // the 4x4x4 corners [4X, 4X+3] x [4Y, 4Y+3] x [4Z, 4Z+3] of its S2 cache (its z range
    // is exactly one S2 quad); the wave's culling box covers every MPU of the brick.
    uint32_t proven8 = 0;
    uint64_t octOut = 0ull, octIn = 0ull;  // per lane (MPU g, octant c): proven all outside / all inside
    if ((p.debug & 1024u) && flags8 != 0u) __builtin_amdgcn_s_setprio(2);  // experiment: heavy waves first
    if constexpr (SPLIT == 2) {
        __shared__ float sLo[4][64], sHi[4][64];
        __shared__ uint32_t sOk[4][64];
        const bool doBound = p.bound && flags8 != 0u;  // the same for both waves of the brick
        float lo = 0.0f, hi = 0.0f;
        bool ok = true;
        BoundBox B;
        if (doBound) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                B.xs[i] = o[0] + (float)(4 * (c & 1) + i) * p.cs;
                B.ys[i] = o[1] + (float)(4 * ((c >> 1) & 1) + i) * p.cs;
                B.zs[i] = o[2] + (float)(4 * (c >> 2) + i) * p.cs;
            }
            const float hx = 0.5f * (B.xs[3] - B.xs[0]), hy = 0.5f * (B.ys[3] - B.ys[0]), hz = 0.5f * (B.zs[3] - B.zs[0]);
            B.cx = 0.5f * (B.xs[0] + B.xs[3]);
            B.cy = 0.5f * (B.ys[0] + B.ys[3]);
            B.cz = 0.5f * (B.zs[0] + B.zs[3]);
            B.h = __builtin_amdgcn_sqrtf(hx * hx + hy * hy + hz * hz) * 1.0001f + 1e-4f;
            if (part == 0) ev.template bound_part<0>(B, cm, &lo, &hi, &ok);
            else ev.template bound_part<1>(B, cm, &lo, &hi, &ok);
        }
        sLo[wave][lane] = lo;
        sHi[wave][lane] = hi;
        sOk[wave][lane] = ok ? 1u : 0u;
        __syncthreads();
        if (part != 0) return;  // the brick's first wave finishes it
        if (doBound) {
            const int r = slot * 2, l = slot * 2 + 1;
            ok = sOk[r][lane] != 0u && sOk[l][lane] != 0u;
            ev.bound_combine(sLo[r][lane], sHi[r][lane], sLo[l][lane], sHi[l][lane], cm, &lo, &hi);
            const uint64_t bOut = ballot(ok && hi < 0.5f), bIn = ballot(ok && lo >= 0.5f);
            octOut = bOut;
            octIn = bIn;
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const bool all = ((bOut >> (8 * q)) & 0xffull) == 0xffull || ((bIn >> (8 * q)) & 0xffull) == 0xffull;
                proven8 |= (all ? 1u : 0u) << q;
            }
            proven8 &= flags8;
        }
    } else if (p.bound && flags8 != 0u) {
        BoundBox B;
#pragma unroll
        for (int i = 0; i < 4; ++i) {  // the S2 coordinates (mpu_body): o + (float)index * cs
            B.xs[i] = o[0] + (float)(4 * (c & 1) + i) * p.cs;
            B.ys[i] = o[1] + (float)(4 * ((c >> 1) & 1) + i) * p.cs;
            B.zs[i] = o[2] + (float)(4 * (c >> 2) + i) * p.cs;
        }
        const float hx = 0.5f * (B.xs[3] - B.xs[0]), hy = 0.5f * (B.ys[3] - B.ys[0]), hz = 0.5f * (B.zs[3] - B.zs[0]);
        B.cx = 0.5f * (B.xs[0] + B.xs[3]);
        B.cy = 0.5f * (B.ys[0] + B.ys[3]);
        B.cz = 0.5f * (B.zs[0] + B.zs[3]);
        B.h = __builtin_amdgcn_sqrtf(hx * hx + hy * hy + hz * hz) * 1.0001f + 1e-4f;
        float lo = 0.0f, hi = 0.0f;
        bool ok = true;
        ev.bound(B, cm, &lo, &hi, &ok);
        const uint64_t bOut = ballot(ok && hi < 0.5f), bIn = ballot(ok && lo >= 0.5f);
        octOut = bOut;
        octIn = bIn;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const bool all = ((bOut >> (8 * q)) & 0xffull) == 0xffull || ((bIn >> (8 * q)) & 0xffull) == 0xffull;
            proven8 |= (all ? 1u : 0u) << q;
        }
        proven8 &= flags8;
        phase_stamp(p, 2, 8192u);
    }
    const uint32_t queue8 = flags8 & ~proven8;
    // lane g < 8 speaks for MPU g (its values are those of lane 8g)
    const uint32_t mOf = __shfl(m, lane * 8 & 63);
    const bool vOf = __shfl(valid ? 1 : 0, lane * 8 & 63) != 0;
    const bool pass = lane < 8 && ((queue8 >> lane) & 1u);
    if (lane < 8 && vOf) {
        // 0: failed S1; 1: passed, proven empty by field bounds; 2: passed, queued for S2
        p.passed[mOf - p.mpuBegin] = (uint8_t)(((flags8 >> lane) & 1u) + ((queue8 >> lane) & 1u));
        if (!pass) p.counts[mOf - p.mpuBegin] = 0ull;
        if (p.mpuTicks) mpu_ticks_s1(p, mOf - p.mpuBegin, tick0);
    }
    if (flags8 == 0u) return;
    const uint32_t shard = W / (p.pShardCap / 8u);
    if (lane == 1 && proven8 != 0u) atomicAdd(&p.ctr->shard[shard].b, (uint32_t)__popc(proven8));
    if (queue8 == 0u) return;
    // k_front: the block's sub-queue (blockIdx mod 8, the XCD of round-robin placement: a speed
    // choice only) at pq + q * fqCap, its count in shard q's p; otherwise the brick's shard
    const uint32_t qsel = FRONT ? (blockIdx.x & 7u) : shard;
    const uint32_t qbase = FRONT ? qsel * p.fqCap : shard * p.pShardCap;
    // the queue reservation's returning atomic is waited for only after the culling masks are
    // made (their round trip overlaps the mask computation; verdict r05 item 4)
    uint32_t baseAtomic = 0;
    if (lane == 0) baseAtomic = atomicAdd(&p.ctr->shard[qsel].p, (uint32_t)__popc(queue8));
    // Culling mask of each queued MPU, from this wave's culling segments (already in
    // registers): its box grown by the normal delta, for k_vertex / k_finish (mpuMasks) and,
    // with the queue entry, for S2 (k_mpu loads no culling data).  The grown box contains the
    // S2 box, so its mask is conservative there too; one mask per MPU instead of two (the
    // boxes differ by 0.001: the masks are the same but for primitives grazing the box).
    uint64_t mLo = 0ull, mHi = 0ull;  // lane q < 8: MPU q's mask, for its queue entry
    if (p.cull) {
        const float eg = 7.0f * p.cs + 0.001f;
        for (uint32_t qm = queue8; qm != 0u; qm &= qm - 1u) {
            const int q = __builtin_ctz(qm);
            const float ox = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(o[0]), 8 * q));
            const float oy = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(o[1]), 8 * q));
            const float oz = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(o[2]), 8 * q));
            const CullMask g = cull_mask_from(cl, ox, oy, oz, ox + eg, oy + eg, oz + eg);
            const uint32_t wq = lane_value(mOf, q) - p.mpuBegin;
            if (lane == 0) {
                p.mpuMasks[2 * wq] = g.lo;
                p.mpuMasks[2 * wq + 1] = g.hi;
            }
            if (lane == q) {
                mLo = g.lo;
                mHi = g.hi;
            }
        }
    }
    if (PSGPU_DEFER_ATOMICS) asm volatile("" : "+v"(baseAtomic) : "v"(mLo));  // the wait for the atomic goes here
    const uint32_t base = lane_value(baseAtomic, 0);
    if (pass) {  // lane q < 8 writes MPU q's entry
        const uint32_t slotq = qbase + base + (uint32_t)__popc(queue8 & ((1u << lane) - 1u));
        if (FRONT) {  // read in this launch by S2 waves on other CUs: write-through (sc1)
            __hip_atomic_store(&p.pq[slotq], mOf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (p.cull) {
                __hip_atomic_store(&p.pqMask[2 * slotq], mLo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&p.pqMask[2 * slotq + 1], mHi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        } else {
            p.pq[slotq] = mOf;
            if (p.cull) {
                p.pqMask[2 * slotq] = mLo;
                p.pqMask[2 * slotq + 1] = mHi;
            }
        }
        // the MPU's octants proven uniform by the same bounds: k_mpu evaluates only the others
        // (their inside bits are the proof's), bits 0-7 all outside, 8-15 all inside
        if (PSGPU_S2_OCT)
            p.pqOct[slotq] = (uint16_t)(((octOut >> (8 * lane)) & 0xffull) | (((octIn >> (8 * lane)) & 0xffull) << 8));
    }
    phase_stamp(p, 3, 8192u);
    if constexpr (FRONT) {
        // publish (MI355X_MICROARCH.md hand-off table, first row): the entries and masks were
        // stored sc1; once they have left this wave (vmcnt(0)), each queued MPU's ready word
        // takes the run's tag (sc1); S2 waves poll it with sc1 loads and then read the entry
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (pass) {
            const uint32_t slotq = qbase + base + (uint32_t)__popc(queue8 & ((1u << lane) - 1u));
            __hip_atomic_store(&p.fqReady[slotq], front_tag(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

#ifndef PSGPU_S2_N
#define PSGPU_S2_N (8 / PSGPU_MPU_WAVES)  // x-slices per walk: one walk per (y,z) needle shares each
                                          // primitive's uniform work and (y,z) terms over its points
#endif
// LDS per k_mpu block: per MPU of the block (4 / W of them): edgeVid[1536] u16 (passes 2-3) | cfg[344] u8 | vbase[344] u16 |
// tbase[344] u16 | the 8 inside-bit words of the S2 cache | qv, qt; then per wave the
// interpreter's value slots.  The S2 field values never leave registers: pass 1 needs
// only their inside bits (8 ballots, shared by the MPU's waves through LDS).
constexpr int kLdsEdge = 0;
constexpr int kLdsCfg = kLdsEdge + 1536 * 2;
constexpr int kLdsVbase = kLdsCfg + 344;
constexpr int kLdsTbase = kLdsVbase + 344 * 2;
constexpr int kLdsIns = ((kLdsTbase + 344 * 2) + 7) & ~7;
constexpr int kLdsQ = kLdsIns + 8 * 8;
constexpr int kLdsMpu = ((kLdsQ + 8) + 15) & ~15;
constexpr int kLdsTables = (int)((sizeof(CubeTablesDev) + 15) & ~(size_t)15);
constexpr int kLdsWaveSlots = kMpusPerBlock * kLdsMpu;  // interpreter slots follow

// Last cell c in [0, 343) with first[c] <= r (first[] = exclusive prefix of per-cell
// counts, non-decreasing, first[0] = 0, so that cell holds item r): binary lifting,
// 9 fixed LDS steps.
__device__ __forceinline__ int find_cell(const uint16_t* first, uint32_t r) {
    int lo = 0;
#pragma unroll
    for (int step = 256; step > 0; step >>= 1) {
        const int mid = lo + step;
        if (mid < 343 && (uint32_t)first[mid] <= r) lo = mid;
    }
    return lo;
}

// Barrier of the MPU's waves (the whole block when W > 1; LDS ordering within the wave
// when one wave does it all).
template <int WPM>
__device__ __forceinline__ void mpu_sync() {
    if (WPM > 1) {
        __syncthreads();
    } else {
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
}

// S2 over the octants k_precheck could not prove uniform (bounds of the 4x4x4 corners
// [4X, 4X+3] x [4Y, 4Y+3] x [4Z, 4Z+3], exactly the corner coordinates below): a pass walks up
// to 4 octants, 16 lanes each -- lane (slot, yy, zz), a 4-point x-needle per lane -- so every
// 4-lane pruning group is 4 z-consecutive corners z = 4Z..4Z+3 of one x and y, the
// reference's S2 quads (:550-610), and every corner's value is the one the 8x8x8 walk gives.
// Proven octants contribute their proof's inside bits.  ins[x] bit y*8 + z, as the 8-needle
// layout's ballots; returned by lane 0 into sIns.
template <int GROUP, class EV>
__device__ __forceinline__ void s2_octants(const EV& ev, const float o[3], float cs, const CullMask& cm, uint32_t oct,
                                           uint32_t U, int lane, uint64_t* sIns) {
    uint64_t ins[8];
#pragma unroll
    for (int x = 0; x < 8; ++x) ins[x] = 0ull;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        if ((oct >> (8 + c)) & 1u) {  // octant c = X | Y << 1 | Z << 2 proven all inside
            const uint64_t m = 0x0F0F0F0Full << (32 * ((c >> 1) & 1) + 4 * (c >> 2));
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                if (c & 1) ins[4 + i] |= m;
                else ins[i] |= m;
            }
        }
    }
    const int sl = lane >> 4, yy = (lane >> 2) & 3, zz = lane & 3;
    uint32_t rest = U;
#pragma unroll 1
    while (rest != 0u) {
        const uint32_t cur = rest;
        // this lane's octant: the sl-th set bit of cur (a lane past the pass's octants repeats
        // the first; its values are not used)
        uint32_t cl = cur;
        for (int j = 0; j < sl; ++j)
            if (cl & (cl - 1u)) cl &= cl - 1u;
            else cl = cur;
        if (sl >= __popc(cur)) cl = cur;
        const int c = __builtin_ctz(cl);
        const int X = c & 1, Y = (c >> 1) & 1, Z = c >> 2;
        float px[4], py[4], pz[4], f[4];
        const float yv = o[1] + (float)(4 * Y + yy) * cs;
        const float zv = o[2] + (float)(4 * Z + zz) * cs;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            px[i] = o[0] + (float)(4 * X + i) * cs;
            py[i] = yv;
            pz[i] = zv;
        }
        ev.template evaln<GROUP, false, 4>(px, py, pz, cm, f, nullptr);
        uint32_t slots = cur;  // the pass's octants in slot order
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint64_t b = ballot(f[i] >= 0.5f);
            uint32_t sc = slots;
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                if (sc == 0u) break;
                const int cs_ = __builtin_ctz(sc);
                sc &= sc - 1u;
                const uint32_t bits = (uint32_t)(b >> (16 * s)) & 0xffffu;
                const int Ys = (cs_ >> 1) & 1, Zs = cs_ >> 2;
                uint64_t v = 0ull;
#pragma unroll
                for (int r = 0; r < 4; ++r) v |= (uint64_t)((bits >> (4 * r)) & 0xfu) << ((4 * Ys + r) * 8 + 4 * Zs);
                if (cs_ & 1) ins[4 + i] |= v;
                else ins[i] |= v;
            }
        }
        // drop the pass's (up to) 4 octants
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (rest) rest &= rest - 1u;
    }
    if (lane == 0) {
#pragma unroll
        for (int x = 0; x < 8; ++x) sIns[x] = ins[x];
    }
}

// Per-MPU body: W = kMpuWaves wavefronts per MPU that passed S1 (and was not proven
// empty), 4 wavefronts per block.  Every wave of a block reaches every barrier: waves
// without an MPU (past the last survivor) or whose MPU has no surface just skip the work.
// SPLIT 2 (tree split): two waves per MPU, each walking one subtree of the root over all
// 8 x-slices (evaln_part), the values exchanged through LDS and combined by both waves
// (combine), which then share the record passes as the W > 1 x-slice split does.
// FRONT (k_front, the S2 blocks of the launch whose first p.preBlocks blocks run S1): block blk
// takes entries [MPB * (blk >> 3), MPB * (blk >> 3) + MPB) of sub-queue blk & 7 as their S1
// waves publish them (their ready words carry the run's tag), instead of the d-th survivor
// of the finished shard queues; an entry that is still untagged once every S1 block of its
// sub-queue has published is past the sub-queue's end.
template <class EV, int SPLIT = 1, bool FRONT = false>
__device__ __forceinline__ void mpu_body(const Params& p, unsigned char* smem, uint32_t* item,
                                         const uint32_t blk = blockIdx.x) {
    *item = 0xffffffffu;
    constexpr int WPM = SPLIT > 1 ? SPLIT : kMpuWaves;  // waves per MPU
    constexpr int MPB = 4 / WPM;                         // MPUs per block
    const int wave = wave_index();
    const int lane = lane_id();
    const int slot = wave / WPM;  // the block's MPU this wave works on
    const int part = wave % WPM;  // its share: x-slices [part * NX, part * NX + NX), or a subtree
    constexpr int NX = SPLIT > 1 ? 8 : 8 / kMpuWaves;
    // MPU d = block * (4 / W) + slot is the d-th queued survivor in shard order (dense over
    // the 64 shard queues: lane s holds shard s's count); the grid is sized by the host
    // from the last finished run, and a run with more survivors than that is re-run by finish()
    phase_stamp(p, 0);
    uint32_t d = blk * (uint32_t)MPB + (uint32_t)slot;
    ModelPtr M = as_const(p.model);
    const CubeTablesDev* tab = p.tables;  // global: L1 / L2 resident (an LDS copy per block measured slower, r05)
    bool live;
    uint32_t slotq = 0;
    if constexpr (FRONT) {
        const uint32_t q = blk & 7u, e = (blk >> 3) * (uint32_t)MPB + (uint32_t)slot;
        d = (e << 3) | q;  // spreads the MPU's vertex records over the shards
        __shared__ uint32_t sFront[4];  // per MPU of the block: entry | live << 31
        if (part == 0 && lane == 0) {
            slotq = q * p.fqCap + e;
            bool lv = false;
            if (e < p.fqCap) {
                const uint32_t tag = front_tag(p);
                const uint32_t need = p.preBlocks > q ? (p.preBlocks - q + 7u) / 8u : 0u;  // S1 blocks of q
                for (uint32_t spins = 0;; ++spins) {
                    if (__hip_atomic_load(&p.fqReady[slotq], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == tag) {
                        lv = true;
                        break;
                    }
                    // every S1 block of q published (each after its waves' entries and tags left them)
                    if ((spins & 7u) == 7u &&
                        __hip_atomic_load(&p.ctr->shard[q].s1Done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= need) {
                        lv = __hip_atomic_load(&p.fqReady[slotq], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == tag;
                        break;
                    }
                    // bounded (test hook PSGPU_OPT_DEBUG bit 27: a few spins against S1 blocks held
                    // back ~40 us): a broken protocol is flagged, finish re-runs as separate launches
                    if (spins > ((p.debug & (1u << 27)) ? 8u : (1u << 22))) {
                        atomicOr(&p.ctr->error, 4u);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
            }
            sFront[slot] = slotq | (lv ? 0x80000000u : 0u);
        }
        __syncthreads();  // the MPU's other wave reads the entry after the barrier its poller joined
        bool any = false;
#pragma unroll
        for (int k = 0; k < MPB; ++k) any |= (sFront[k] >> 31) != 0u;
        if (!any) return;  // no entry for this block (block-uniform)
        slotq = sFront[slot] & 0x7fffffffu;
        live = (sFront[slot] >> 31) != 0u;
    } else {
        // prologue: wave 0 reads the 64 shard counts (one 128-B line each) and scans them for
        // the block
        __shared__ uint32_t sIncl[kShards];
        if (wave == 0) {
            const uint32_t cnt = p.ctr->shard[lane].p;  // kShards == 64: one shard per lane
            sIncl[lane] = wave_incl_scan(cnt);
        }
        __syncthreads();
        // MPU d = block * (4 / W) + slot is the d-th queued survivor in shard order (dense over
        // the 64 shard queues); the grid is sized by the host from the last finished run, and
        // a run with more survivors than that is re-run by finish()
        const uint32_t incl = sIncl[lane];
        const uint32_t pcount = sIncl[kShards - 1];
        if (blk * (uint32_t)MPB >= pcount) return;  // whole block past the last survivor
        live = d < pcount;
        if (live) {
            const uint32_t pshard = (uint32_t)__popcll(ballot(incl <= d));  // first shard whose prefix passes d
            const uint32_t pidx = d - (pshard ? sIncl[pshard - 1] : 0u);
            slotq = uniform(pshard * p.pShardCap + pidx);
        }
    }
    uint32_t m = 0, w = 0;
    float o[3] = {0.0f, 0.0f, 0.0f};
    CullMask cm{0ull, 0ull};
    uint32_t oct = 0;  // k_precheck's octant proofs (PSGPU_S2_OCT)
    (void)oct;
    if (live) {
        if (FRONT) {  // published in this launch: sc1 loads (the stores were sc1)
            m = uniform(__hip_atomic_load(&p.pq[slotq], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            if (p.cull) {
                cm.lo = uniform64(__hip_atomic_load(&p.pqMask[2 * slotq], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
                cm.hi = uniform64(__hip_atomic_load(&p.pqMask[2 * slotq + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            }
        } else {
        m = uniform(p.pq[slotq]);
        if (p.cull) {  // the MPU box's culling mask, made by k_precheck: in SGPRs, so every
                       // per-primitive culling test of the walk is a scalar branch
#if PSGPU_UNIFORM_CM
            cm.lo = uniform64(p.pqMask[2 * slotq]);
            cm.hi = uniform64(p.pqMask[2 * slotq + 1]);
#else
            cm.lo = p.pqMask[2 * slotq];
            cm.hi = p.pqMask[2 * slotq + 1];
#endif
        }
        }
        if (PSGPU_S2_OCT) oct = uniform((uint32_t)p.pqOct[slotq]);
        *item = m;
        w = m - p.mpuBegin;  // slot of the MPU in the range: counts / offsets index
        mpu_origin(p, m, o);
    }
    phase_stamp(p, 1);
    if (WPM == 1 && !live) return;
    unsigned char* base = smem + slot * kLdsMpu;
    uint16_t* edgeVid = reinterpret_cast<uint16_t*>(base + kLdsEdge);
    uint8_t* cellCfg = base + kLdsCfg;
    uint16_t* cellV = reinterpret_cast<uint16_t*>(base + kLdsVbase);
    uint16_t* cellT = reinterpret_cast<uint16_t*>(base + kLdsTbase);
    uint64_t* sIns = reinterpret_cast<uint64_t*>(base + kLdsIns);
    uint32_t* sQ = reinterpret_cast<uint32_t*>(base + kLdsQ);
    EV ev(M, reinterpret_cast<float*>(smem + kLdsWaveSlots + wave * p.slotsPerLane * 64 * 4) + lane);
    const float cs = p.cs;

    float fs[NX];
    if (live) {
        // S2 (:550-610): corner (x, y, z) of the 8x8x8 cache, lane = y*8 + z, this wave's
        // NX x-slices per lane; quads = 4 consecutive z
        const int y = lane >> 3, z = lane & 7;
        const float py = o[1] + (float)y * cs;
        const float pz = o[2] + (float)z * cs;
        phase_stamp(p, 2);
        float pxs[NX], pys[NX], pzs[NX];
#pragma unroll
        for (int x = 0; x < NX; ++x) {
            pxs[x] = o[0] + (float)((SPLIT > 1 ? 0 : part * NX) + x) * cs;  // SPLIT: both waves walk all 8
            pys[x] = py;
            pzs[x] = pz;
        }
        if constexpr (SPLIT > 1) {
            if (part == 0) ev.template evaln_part<kS2Group, false, 8, 0>(pxs, pys, pzs, cm, fs, nullptr);
            else ev.template evaln_part<kS2Group, false, 8, 1>(pxs, pys, pzs, cm, fs, nullptr);
        } else {
#if PSGPU_S2_OCT
        const uint32_t U = ~(oct | (oct >> 8)) & 0xffu;  // octants without a proof
        if (WPM == 1 && (PSGPU_S2_OCT == 2 || __popc(U) <= 4)) {
            s2_octants<kS2Group>(ev, o, cs, cm, oct, U, lane, sIns);
        } else {
#else
        {
#endif
#if PSGPU_S2_N == 1
        // one walk per x-slice in a runtime loop: the walk's code stays resident in the
        // instruction cache (unrolled copies of a 32-primitive walk do not fit)
#pragma unroll 1
        for (int h = 0; h < NX; ++h) fs[h] = ev.template eval<kS2Group, false>(pxs[h], py, pz, cm, nullptr);
#else
#pragma unroll
        for (int h = 0; h < NX; h += PSGPU_S2_N)
            ev.template evaln<kS2Group, false, PSGPU_S2_N>(pxs + h, pys + h, pzs + h, cm, fs + h, nullptr);
#endif
        // inside bits of the 8x8x8 corners: ins[x] bit y*8 + z (lane order)
#pragma unroll
        for (int x = 0; x < NX; ++x) {
            const uint64_t b = ballot(fs[x] >= 0.5f);
            if (lane == 0) sIns[part * NX + x] = b;
        }
        }
        }
    }
    uint64_t ins[8];
    uint32_t inside = 0;
    if constexpr (SPLIT > 1) {  // the parts' values through LDS; both waves combine all 8 slices
        __shared__ float sS2[4][8][64];
        if (live) {
#pragma unroll
            for (int x = 0; x < 8; ++x) sS2[wave][x][lane] = fs[x];
        }
        phase_stamp(p, 3);
        __syncthreads();
        phase_stamp(p, 4);
        if (live) {
            float rv[8], lv[8], f8[8];
#pragma unroll
            for (int x = 0; x < 8; ++x) {
                rv[x] = sS2[slot * 2][x][lane];
                lv[x] = sS2[slot * 2 + 1][x][lane];
            }
            ev.template combine<false, 8>(rv, nullptr, lv, nullptr, cm, f8, nullptr);
#pragma unroll
            for (int x = 0; x < 8; ++x) {
                ins[x] = ballot(f8[x] >= 0.5f);
                inside += __popcll(ins[x]);
            }
        } else {
#pragma unroll
            for (int x = 0; x < 8; ++x) ins[x] = 0ull;
        }
    } else {
    phase_stamp(p, 3);
    mpu_sync<WPM>();
    phase_stamp(p, 4);
#pragma unroll
    for (int x = 0; x < 8; ++x) {
        ins[x] = live ? sIns[x] : 0ull;
        inside += __popcll(ins[x]);
    }
    }
    const bool work = live && inside != 0 && inside != 512 && !(p.debug & 1u);
    if (live && !work && part == 0 && lane == 0) p.counts[w] = 0ull;  // no vertices, no triangles
    if (WPM == 1 && !work) return;

    // S3 pass 1 (:647-691): config per cell (bit c = x*4 + y*2 + z, inside = f >= 0.5),
    // owned sign-changing edges (new vertices) and triangles; wave prefix sums give
    // the reference's discovery order over cells (i,j,k): one x-slab i per step, lane
    // j*8 + k, so the cell's corners are bits lane + {0, 1, 8, 9} of ins[i] and ins[i+1].
    // Every wave of the MPU computes V and T; the first writes the tables and counters.
    const uint64_t edgeBits = tab->edge;
    uint32_t V = 0, T = 0;
    // WPM 1: the record queues' bases stay in lane 0's registers (the returning atomics are not
    // waited for until pass 2 stores its first record: their round trip overlaps the record's
    // cell search; verdict r05 item 4: the record passes hold half of k_mpu's parked cycles)
    uint32_t qvAtomic = 0u, qtAtomic = 0u;
    if (work) {
        uint32_t carry = 0;  // V | T << 16 (both <= 343 * 12 per MPU: no carry between the halves)
        const int j = lane >> 3, k = lane & 7;
        const bool cellLane = j < 7 && k < 7;
        const uint32_t ownJK = tab->own[(j == 0 ? 2 : 0) | (k == 0 ? 1 : 0)];    // cells with i > 0
        const uint32_t ownJK0 = tab->own[4 | (j == 0 ? 2 : 0) | (k == 0 ? 1 : 0)];  // the i == 0 slab
#pragma unroll
        for (int i = 0; i < 7; ++i) {
            const int c = i * 49 + j * 7 + k;
            const uint32_t b0 = (uint32_t)(ins[i] >> lane), b1 = (uint32_t)(ins[i + 1] >> lane);
            uint32_t cfg = 0;
            if (cellLane)
                cfg = (b0 & 3u) | ((b0 >> 6) & 12u) | ((b1 & 3u) << 4) | (((b1 >> 8) & 3u) << 6);
            uint32_t nvt = 0;
            if (cfg != 0 && cfg != 255)
            {
                const uint32_t cn = tab->crossNtri[cfg];
                nvt = (uint32_t)__popc((i == 0 ? ownJK0 : ownJK) & cn & 0xfffu) | (cn & 0xffff0000u);
            }
            const uint32_t svt = wave_incl_scan(nvt);  // one scan for both counts
            if (cellLane && part == 0) {
                const uint32_t first = carry + svt - nvt;
                cellCfg[c] = (uint8_t)cfg;
                cellV[c] = (uint16_t)(first & 0xffffu);
                cellT[c] = (uint16_t)(first >> 16);
            }
            carry += lane_value(svt, 63);
        }
        V = carry & 0xffffu;
        T = carry >> 16;
        if (part == 0) {
            const uint32_t shard = d & (kShards - 1);
            if (lane == 0) {
                qvAtomic = atomicAdd(&p.ctr->shard[shard].v, V);
                qtAtomic = atomicAdd(&p.ctr->shard[w & (kShards - 1)].t, T);  // TriRec: shard = w & 63
                if (WPM > 1) {
                    sQ[0] = qvAtomic;
                    sQ[1] = qtAtomic;
                }
                p.counts[w] = (uint64_t)V | ((uint64_t)T << 32);
                if (T > 0) atomicAdd(&p.ctr->shard[shard].s, 1u);
                if (V > 512u || T > 512u) atomicMin(&p.ctr->firstOverflow, (int)m);
            }
        }
    }
    phase_stamp(p, 5);
#if PSGPU_MPU_LIVE_STAMP
    // phase word 7 (measurement builds only): the wave's live primitives, its MPU's V and T
    if ((p.debug & 4096u) && p.stamps && lane == 0 && live) {
        const uint32_t sw = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
        if (sw < p.stampCap)
            p.stamps[3 * (size_t)kNumStampKernels * p.stampCap + 8 * (size_t)sw + 7] =
                (uint64_t)(128 - __popcll(cm.lo) - __popcll(cm.hi)) | ((uint64_t)V << 16) | ((uint64_t)T << 32);
    }
#endif
    mpu_sync<WPM>();
    const bool recs = work && !(p.debug & 2u);  // ablation bit 1: pass 1 only
    const uint32_t shard = d & (kShards - 1);
    VertexKey* vk = p.vk + (size_t)shard * p.vShardCap;
    TriRec* tq = p.tq + (size_t)(w & (kShards - 1)) * p.tShardCap;

    // pass 2 (:703-762), one lane per new vertex r (batches of 64 dealt to the MPU's waves
    // in turn): its cell is the last cell whose first vertex id is <= r; it is that cell's
    // k-th owned crossing edge in first-occurrence order of the row, k = r - first id.
    // Records are written coalesced.
    if (recs) {
        uint32_t qv = WPM > 1 ? sQ[0] : 0u;
        for (uint32_t b0 = (uint32_t)part * 64u; b0 < V; b0 += 64u * WPM) {
            const uint32_t r = b0 + (uint32_t)lane;
            if (r < V) {
                const int c = find_cell(cellV, r);
                const uint32_t cfg = cellCfg[c];
                const int i = c / 49, j = (c / 7) % 7, k = c % 7;
                const uint32_t own = tab->own[(i == 0 ? 4 : 0) | (j == 0 ? 2 : 0) | (k == 0 ? 1 : 0)];
                const uint64_t order = tab->order[cfg];
                uint32_t left = r - cellV[c];
                int ed = 0;
                for (int q = 0; q < 12; ++q) {  // the (left+1)-th owned edge of the row order
                    ed = (int)((order >> (4 * q)) & 15u);
                    if ((own >> ed) & 1u) {
                        if (left == 0u) break;
                        --left;
                    }
                }
                const int eb = (int)((edgeBits >> (5 * ed)) & 31u);
                const int c1 = eb & 7, ax = eb >> 3;
                const int sx = i + ((c1 >> 2) & 1), sy = j + ((c1 >> 1) & 1), sz = k + (c1 & 1);
                edgeVid[((sx * 8 + sy) * 8 + sz) * 3 + ax] = (uint16_t)r;
                const uint32_t key = (uint32_t)sx | ((uint32_t)sy << 3) | ((uint32_t)sz << 6) | ((uint32_t)ax << 9);
                if (WPM == 1) {  // lane 0's atomic result, read only once the record is made (the
                                 // empty asm ties the read, and the wait for the atomic, to the key)
                    if (PSGPU_DEFER_ATOMICS) asm volatile("" : "+v"(qvAtomic) : "v"(key));
                    qv = lane_value(qvAtomic, 0);
                }
                const uint32_t g = qv + r;
                if (g < p.vShardCap) vk[g] = VertexKey{w, r | (key << 16)};
            }
        }
    }
    phase_stamp(p, 6);
    mpu_sync<WPM>();
    if (!recs || (p.debug & 4u)) return;  // ablation bit 2: no triangles

    // pass 3 (S6, :816-825), one lane per triangle r: its cell (last first-id <= r) and
    // the (r - first)-th triangle of the cell's table row
    const uint32_t qt = WPM > 1 ? sQ[1] : lane_value(qtAtomic, 0);
    for (uint32_t b0 = (uint32_t)part * 64u; b0 < T; b0 += 64u * WPM) {
        const uint32_t r = b0 + (uint32_t)lane;
        if (r < T) {
            const int c = find_cell(cellT, r);
            const uint32_t t = r - cellT[c];
            const int i = c / 49, j = (c / 7) % 7, k = c % 7;
            const uint64_t row = tab->row[cellCfg[c]];
            uint32_t v[3];
#pragma unroll
            for (int sv = 0; sv < 3; ++sv) {
                const int ed = (int)((row >> (4 * (t * 3 + sv))) & 15u);
                const int eb = (int)((edgeBits >> (5 * ed)) & 31u);
                const int c1 = eb & 7, ax = eb >> 3;
                const int sx = i + ((c1 >> 2) & 1), sy = j + ((c1 >> 1) & 1), sz = k + (c1 & 1);
                v[sv] = edgeVid[((sx * 8 + sy) * 8 + sz) * 3 + ax];
            }
            const uint32_t g = qt + r;
            if (g < p.tShardCap)
                tq[g] = TriRec{r | ((v[2] >> 10) << 11) | ((w >> 6) << 12), v[0] | (v[1] << 11) | ((v[2] & 1023u) << 22)};
        }
    }
}

// Batches of `per` records over the kShards queues: lane l holds shard l's batch
// count, so a batch index maps to (shard, first record) with one ballot.
// The block's copy of the 64 shard counts of one ShardCtr field (word `field`): the first
// 64 threads gather the 64 lines once per block; the caller syncs the block before use.
__device__ __forceinline__ void stage_shard_counts(const Params& p, int field, uint32_t* s) {
    if (threadIdx.x < (unsigned)kShards)
        s[threadIdx.x] = reinterpret_cast<const uint32_t*>(&p.ctr->shard[threadIdx.x])[field];
}

struct ShardBatches {
    uint32_t cnt, incl, total;
    __device__ ShardBatches(const uint32_t* staged, uint32_t cap, uint32_t per) {
        cnt = min(staged[lane_id()], cap);  // staged by stage_shard_counts
        const uint32_t nb = (cnt + per - 1) / per;
        incl = wave_incl_scan(nb);
        total = lane_value(incl, kShards - 1);
        perBatch = per;
        nbat = nb;
    }
    uint32_t perBatch, nbat;
    __device__ void locate(uint32_t b, uint32_t* shard, uint32_t* first, uint32_t* count) const {
        const uint32_t s = (uint32_t)__popcll(ballot(incl <= b));
        const uint32_t start = __shfl(incl - nbat, (int)s);
        *shard = s;
        *first = (b - start) * perBatch;
        *count = __shfl(cnt, (int)s);
    }
};

// Exclusive offsets of the per-MPU (V | T << 32) counts of the range, in MPU order (the
// reference's PolyMPUs order): offs[0] = 0, offs[w + 1] = inclusive sum.  Single pass,
// run by the first scanBlocks 256-thread blocks of k_vertex (all co-resident): each owns
// chunks of kScanItems counts (8 consecutive per thread, 64-B vector loads), publishes
// its aggregate, looks back over up to 64 predecessors at once (decoupled look-back),
// then scans.  V and T halves are scanned as two u32 DPP
// scans (their totals stay below 2^31).  Status words (state << 62 | T << 31 | V) start
// at zero: the previous run's k_finish cleared them.  All blocks are resident.
__device__ __forceinline__ uint64_t scan_word(uint32_t state, uint32_t v, uint32_t t) {
    return ((uint64_t)state << 62) | ((uint64_t)(t & 0x7fffffffu) << 31) | (uint64_t)(v & 0x7fffffffu);
}

struct Chunk8 {
    uint64_t c[8];
    __device__ void load(const uint64_t* counts, uint32_t e, uint32_t hi) {
        if (e + 8 <= hi) {
            const uint4* src = reinterpret_cast<const uint4*>(counts + e);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint4 q = src[i];
                c[2 * i] = (uint64_t)q.x | ((uint64_t)q.y << 32);
                c[2 * i + 1] = (uint64_t)q.z | ((uint64_t)q.w << 32);
            }
        } else {
#pragma unroll
            for (int i = 0; i < 8; ++i) c[i] = e + i < hi ? counts[e + i] : 0ull;
        }
    }
    __device__ void sum(uint32_t& v, uint32_t& t) const {
        v = 0u;
        t = 0u;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            v += (uint32_t)c[i];
            t += (uint32_t)(c[i] >> 32);
        }
    }
};

__device__ __forceinline__ void scan_counts_block(const Params& p, uint32_t b) {
    constexpr int kWaves = (int)(kScanItems / 512u);
    __shared__ uint32_t sWave[2][kWaves];
    __shared__ uint32_t sPrefix[2];
    const uint32_t n = p.mpuCount;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const uint32_t lo = b * p.scanChunks * kScanItems;
    const uint32_t hi = min(n, lo + p.scanChunks * kScanItems);
    // pass 1: the block's aggregate (the first chunk stays in registers)
    Chunk8 ch;
    ch.load(p.counts, lo + (uint32_t)t * 8u, hi);
    uint32_t sv, st;
    ch.sum(sv, st);
    for (uint32_t c = 1; c < p.scanChunks; ++c) {
        Chunk8 more;
        more.load(p.counts, lo + c * kScanItems + (uint32_t)t * 8u, hi);
        uint32_t a, bb;
        more.sum(a, bb);
        sv += a;
        st += bb;
    }
    const uint32_t wv_v = lane_value(wave_incl_scan(sv), 63), wv_t = lane_value(wave_incl_scan(st), 63);
    if (lane == 0) {
        sWave[0][wv] = wv_v;
        sWave[1][wv] = wv_t;
    }
    __syncthreads();
    if (wv == 0) {
        uint32_t aggV = 0u, aggT = 0u;
#pragma unroll
        for (int w = 0; w < kWaves; ++w) {
            aggV += sWave[0][w];
            aggT += sWave[1][w];
        }
        uint32_t exV = 0u, exT = 0u;
        if (b == 0) {
            if (lane == 0) __hip_atomic_store(&p.scanStatus[0], scan_word(2, aggV, aggT), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            if (lane == 0) __hip_atomic_store(&p.scanStatus[b], scan_word(1, aggV, aggT), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            int64_t j = (int64_t)b - 1;
            for (;;) {
                const int64_t idx = j - lane;
                uint32_t state = 2, v = 0u, tt = 0u;
                if (idx >= 0) {
                    uint64_t w = 0ull;
                    uint32_t spins = 0;  // bounded: a broken protocol ends the kernel, flagged
                    do {
                        w = __hip_atomic_load(&p.scanStatus[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    } while ((w >> 62) == 0ull && ++spins < (1u << 20));
                    if (p.debug & (1u << 26)) w = 0ull;  // test hook: every look-back times out
                    if ((w >> 62) == 0ull) {
                        atomicOr(&p.ctr->error, 1u);
                        w = scan_word(2, 0u, 0u);
                    }
                    state = (uint32_t)(w >> 62);
                    v = (uint32_t)(w & 0x7fffffffull);
                    tt = (uint32_t)((w >> 31) & 0x7fffffffull);
                }
                const uint64_t inc = ballot(state == 2);
                const bool stop = inc != 0ull;
                const int k = stop ? __builtin_ctzll(inc) : 63;  // newest predecessor with an inclusive prefix
                exV += lane_value(wave_incl_scan(lane <= k ? v : 0u), 63);
                exT += lane_value(wave_incl_scan(lane <= k ? tt : 0u), 63);
                if (stop) break;
                j -= 64;
            }
            if (lane == 0)
                __hip_atomic_store(&p.scanStatus[b], scan_word(2, exV + aggV, exT + aggT), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
        if (lane == 0) {
            sPrefix[0] = exV;
            sPrefix[1] = exT;
        }
    }
    if (b == 0 && t == 0) p.offs[0] = 0ull;
    __syncthreads();
    // pass 2: per thread 8 consecutive counts; one block-wide scan per chunk
    uint32_t carryV = sPrefix[0], carryT = sPrefix[1];
    for (uint32_t c = 0; c < p.scanChunks; ++c) {
        const uint32_t e0 = lo + c * kScanItems + (uint32_t)t * 8u;
        if (c > 0) {
            ch.load(p.counts, e0, hi);
            ch.sum(sv, st);
            __syncthreads();  // sWave reuse
        }
        const uint32_t iv = wave_incl_scan(sv), it = wave_incl_scan(st);
        if (lane == 63) {
            sWave[0][wv] = iv;
            sWave[1][wv] = it;
        }
        __syncthreads();
        uint32_t runV = carryV + iv - sv, runT = carryT + it - st;
        uint32_t totV = 0u, totT = 0u;
#pragma unroll
        for (int w = 0; w < kWaves; ++w) {
            const uint32_t a = sWave[0][w], bb = sWave[1][w];
            runV += w < wv ? a : 0u;
            runT += w < wv ? bb : 0u;
            totV += a;
            totT += bb;
        }
        uint64_t out[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            runV += (uint32_t)ch.c[i];
            runT += (uint32_t)(ch.c[i] >> 32);
            out[i] = (uint64_t)runV | ((uint64_t)runT << 32);
        }
#pragma unroll
        for (int i = 0; i < 8; ++i)
            if (e0 + i < hi) p.offs[e0 + i + 1] = out[i];
        carryV += totV;
        carryT += totT;
    }
}

// Cull mask for the AABB of N points per lane (all 64 lanes must participate),
// grown by `ext` on the high side of every axis.
template <int N>
__device__ __forceinline__ CullMask cull_mask_points_n(ModelPtr M, const float* px, const float* py, const float* pz,
                                                       bool enable, float ext = 0.0f) {
    if (!enable) return CullMask{0ull, 0ull};
    bool nan = false;
    float x0 = px[0], x1 = px[0], y0 = py[0], y1 = py[0], z0 = pz[0], z1 = pz[0];
#pragma unroll
    for (int n = 0; n < N; ++n) {
        nan = nan || !(px[n] == px[n]) || !(py[n] == py[n]) || !(pz[n] == pz[n]);
        x0 = fminf(x0, px[n]); x1 = fmaxf(x1, px[n]);
        y0 = fminf(y0, py[n]); y1 = fmaxf(y1, py[n]);
        z0 = fminf(z0, pz[n]); z1 = fmaxf(z1, pz[n]);
    }
    // a NaN coordinate (fminf/fmaxf would hide it) disables culling for the wave
    if (ballot(nan) != 0ull) return CullMask{0ull, 0ull};
    return cull_mask_box(M, wave_min(x0), wave_min(y0), wave_min(z0), wave_max(x1) + ext, wave_max(y1) + ext,
                         wave_max(z1) + ext);
}

// Culling mask of a wave whose lanes hold points of the MPUs w (range slots): the AND of
// those MPUs' masks (k_mpu, box grown by the normal delta), one scalar load pair per
// distinct MPU.  A primitive culled for every one of the boxes is +0 at all the points.
__device__ __forceinline__ CullMask cull_mask_mpus(const Params& p, uint32_t w) {
    CullMask cm{~0ull, ~0ull};
    bool todo = true;
    for (;;) {
        const uint64_t b = ballot(todo);
        if (b == 0ull) break;
        const uint32_t w0 = lane_value(w, (int)__builtin_ctzll(b));
        cm.lo &= p.mpuMasks[2 * w0];
        cm.hi &= p.mpuMasks[2 * w0 + 1];
        if (w == w0) todo = false;
    }
    return cm;
}

// The edge of a vertex record (PS_Polygonizer.cpp:722-724): e1 = lo + cs*s, e2 = e1 with
// e2[axis] += cs, d = e2 - e1, and its samples e1 + d * (l/3), l = 0..3 (:744-755).  k_vertex
// brackets the root with them; k_finish recomputes the root from the record (iv, scale)
// through the same expressions, so both kernels see the same bits.
struct EdgeSeg {
    float e[3], d[3];
};
__device__ __forceinline__ EdgeSeg edge_segment(const Params& p, uint32_t w, uint32_t key) {
    float o[3];
    mpu_origin(p, w + p.mpuBegin, o);  // the MPU origin, as k_mpu computed it
    const int sx = key & 7, sy = (key >> 3) & 7, sz = (key >> 6) & 7, ax = (key >> 9) & 3;
    const float cs = p.cs;
    EdgeSeg E;
    E.e[0] = o[0] + cs * (float)sx;
    E.e[1] = o[1] + cs * (float)sy;
    E.e[2] = o[2] + cs * (float)sz;
    E.d[0] = (ax == 0 ? E.e[0] + cs : E.e[0]) - E.e[0];
    E.d[1] = (ax == 1 ? E.e[1] + cs : E.e[1]) - E.e[1];
    E.d[2] = (ax == 2 ? E.e[2] + cs : E.e[2]) - E.e[2];
    return E;
}
__device__ __forceinline__ float edge_sample(float e, float d, int l) {
    const float third = 1.0f / 3.0f;
    return e + d * ((float)l * third);
}
// the linear root on [sample iv - 1, sample iv] (:756-762): a + scale * (b - a)
__device__ __forceinline__ void vertex_root(const EdgeSeg& E, uint32_t iv, float scale, float pos[3]) {
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const float a = edge_sample(E.e[c], E.d[c], (int)iv - 1);
        const float b = edge_sample(E.e[c], E.d[c], (int)iv);
        pos[c] = a + scale * (b - a);
    }
}

#ifndef PSGPU_V_N
#define PSGPU_V_N 1  // vertices per quad of lanes per k_vertex pass (2: bigger culling boxes, slower)
#endif

// Vertices: 16 * VN per wavefront pass, one quad of lanes per vertex and VN vertices
// per quad (vertex first + quad + 16n), each walk evaluating VN points per lane.
// Quad pruning: the 4 edge samples e1 + (e2-e1)*(l/3), l = 0..3 (:722-762), then the
// linear root.  The position goes into the vertex record; k_finish evaluates value,
// colour and normal there (:764-807) and places the vertex in the mesh.
template <class EV, int VPW = 16>
__device__ __forceinline__ void vertex_body(const Params& p, float* lds) {
    constexpr int VN = PSGPU_V_N;
    const int wave = wave_index();
    const int lane = lane_id();
    ModelPtr M = as_const(p.model);
    EV ev(M, lds + wave * (p.slotsPerLane * 4 * 64) + lane);
    const int j = lane & 3;
    if (blockIdx.x < p.scanBlocks) scan_counts_block(p, blockIdx.x);  // block-uniform
    __shared__ uint32_t sCnt[kShards];
    stage_shard_counts(p, 1, sCnt);  // ShardCtr::v
    __syncthreads();
    const uint32_t nWaves = gridDim.x * (blockDim.x >> 6);
if constexpr (VPW == 64) {
    // one lane per vertex: its 4 edge samples as one 4-point walk whose op-box pruning
    // groups the lane's 4 points (GROUP 0) as the quad layout groups the quad's lanes, so
    // every value is the same; packed fp32 and one set of uniform work per 4 samples
    // (more total throughput, a 4x longer walk per wave: chosen for large runs)
    const ShardBatches sb(sCnt, p.vShardCap, 64);
    for (uint32_t batch = blockIdx.x * (blockDim.x >> 6) + wave; batch < sb.total; batch += nWaves) {
        uint32_t shard, first, count;
        sb.locate(batch, &shard, &first, &count);
        uint32_t rr = first + (uint32_t)lane;
        const bool valid = rr < count;
        if (!valid) rr = first;
        const size_t rec = (size_t)shard * p.vShardCap + rr;
        const VertexKey R = p.vk[rec];
        const EdgeSeg E = edge_segment(p, R.w, R.vidKey >> 16);
        float xs[4], ys[4], zs[4], fs[4];
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2) {
            xs[s2] = edge_sample(E.e[0], E.d[0], s2);
            ys[s2] = edge_sample(E.e[1], E.d[1], s2);
            zs[s2] = edge_sample(E.e[2], E.d[2], s2);
        }
        CullMask cm{0ull, 0ull};
        if (p.cull) cm = cull_mask_mpus(p, R.w);
        if (p.debug & 256u) {  // ablation bit 8: no phase-A walk
#pragma unroll
            for (int s2 = 0; s2 < 4; ++s2) fs[s2] = xs[s2];
        } else {
            ev.template evaln<0, false, 4>(xs, ys, zs, cm, fs, nullptr);
        }
        // first sample whose inside state differs from sample 0, else 3 (:744-755); the
        // root itself is k_finish's (vertex_root)
        const bool st0 = fs[0] >= 0.5f;
        const int iv = ((fs[1] >= 0.5f) != st0) ? 1 : (((fs[2] >= 0.5f) != st0) ? 2 : 3);
        const float fa = iv == 1 ? fs[0] : (iv == 2 ? fs[1] : fs[2]);
        const float fb = iv == 1 ? fs[1] : (iv == 2 ? fs[2] : fs[3]);
        if (valid) p.vp[rec] = VertexPos{(0.5f - fa) / (fb - fa), (uint32_t)iv};
    }
} else {
    const ShardBatches sb(sCnt, p.vShardCap, 16 * VN);
    for (uint32_t batch = blockIdx.x * (blockDim.x >> 6) + wave; batch < sb.total; batch += nWaves) {
        uint32_t shard, first, count;
        sb.locate(batch, &shard, &first, &count);
        bool valid[VN];
        size_t rec[VN];
        float qx[VN], qy[VN], qz[VN];
        uint32_t wrec[VN];
#pragma unroll
        for (int n = 0; n < VN; ++n) {
            uint32_t rr = first + ((uint32_t)lane >> 2) + 16u * (uint32_t)n;
            valid[n] = rr < count;
            if (!valid[n]) rr = first;
            rec[n] = (size_t)shard * p.vShardCap + rr;
            const VertexKey R = p.vk[rec[n]];
            wrec[n] = R.w;
            const EdgeSeg E = edge_segment(p, R.w, R.vidKey >> 16);
            qx[n] = edge_sample(E.e[0], E.d[0], j);  // lane j of the quad: sample j
            qy[n] = edge_sample(E.e[1], E.d[1], j);
            qz[n] = edge_sample(E.e[2], E.d[2], j);
        }
        // every edge sample lies in its MPU's box (k_mpu's mask; the d^2 >= 1.02 margin
        // absorbs the last-bit rounding of e1 + cs vs lo + 7 cs)
        CullMask cm{0ull, 0ull};
        if (p.cull) {
            if (VN == 1) {
                cm = cull_mask_mpus(p, wrec[0]);
            } else {
                cm = cull_mask_points_n<VN>(M, qx, qy, qz, true);
            }
        }
        float f[VN];
        if (p.debug & 256u) {  // ablation bit 8: no phase-A walk
#pragma unroll
            for (int n = 0; n < VN; ++n) f[n] = qx[n];
        } else {
            ev.template evaln<4, false, VN>(qx, qy, qz, cm, f, nullptr);
        }
#pragma unroll
        for (int n = 0; n < VN; ++n) {
            float fs[4];
            fs[0] = quad_bcast<0>(f[n]);
            fs[1] = quad_bcast<1>(f[n]);
            fs[2] = quad_bcast<2>(f[n]);
            fs[3] = quad_bcast<3>(f[n]);
            // first sample whose inside state differs from sample 0, else 3 (:744-755)
            const bool st0 = fs[0] >= 0.5f;
            const int iv = ((fs[1] >= 0.5f) != st0) ? 1 : (((fs[2] >= 0.5f) != st0) ? 2 : 3);
            const float fa = iv == 1 ? fs[0] : (iv == 2 ? fs[1] : fs[2]);
            const float fb = iv == 1 ? fs[1] : (iv == 2 ? fs[2] : fs[3]);
            // into the record; k_finish recomputes the root there (vertex_root) and adds
            // normal and colour
            if (valid[n] && j == 0) p.vp[rec[n]] = VertexPos{(0.5f - fa) / (fb - fa), (uint32_t)iv};
        }
    }
}
}

#ifndef PSGPU_FIN_TRI_PREFETCH
#define PSGPU_FIN_TRI_PREFETCH 0  // measured neutral (isolated k_finish 27.8 us either way, r05)
#endif
// One lane's triangle record of a k_finish batch and its MPU's (V | T << 32) offset: the
// global triangle gt = T offset + local id, its corners = V offset + local vertex ids (S6,
// PS_Polygonizer.cpp:816-825, in the compact mesh's MPU order).
struct TriPre {
    TriRec R;
    uint64_t o;
    bool ok;
};
__device__ __forceinline__ TriPre tri_load(const Params& p, const ShardBatches& sb, uint32_t batch) {
    TriPre t;
    t.ok = false;
    t.R = TriRec{0u, 0u};
    t.o = 0ull;
    if (batch >= sb.total) return t;
    uint32_t shard, first, count;
    sb.locate(batch, &shard, &first, &count);
    const uint32_t i = first + lane_id();
    if (i >= count) return t;
    t.R = p.tq[(size_t)shard * p.tShardCap + i];
    t.o = p.offs[((t.R.a >> 12) << 6) | shard];  // the record's shard is w & 63
    t.ok = true;
    return t;
}
__device__ __forceinline__ void tri_store(const Params& p, const TriPre& t) {
    if (!t.ok) return;
    const uint32_t gt = (uint32_t)(t.o >> 32) + (t.R.a & 2047u);
    const uint32_t base = (uint32_t)t.o;
    if (gt >= p.tCap) return;  // finish() grows and re-runs
    p.tris[gt * 3 + 0] = base + (t.R.b & 2047u);
    p.tris[gt * 3 + 1] = base + ((t.R.b >> 11) & 2047u);
    p.tris[gt * 3 + 2] = base + ((t.R.b >> 22) | (((t.R.a >> 11) & 1u) << 10));
}

// Finish: per vertex fieldValueAndColor's value and colour walk (PS_Polygonizer.cpp:777-778,
// 1378-1551) and the three normal samples (:780-781, 1598-1622), then the triangle records
// -> global vertex ids.  Runs after k_vertex wrote the roots.  VPW 64: one lane per
// vertex walking its 4 points; VPW 16: a quad of lanes per vertex, one point each (a
// quarter of the walk per wave: shorter spans when the vertices do not fill the persistent
// grid, e.g. a small rank share; more total work otherwise).  Same values either way.
template <class EV, int VPW = 64>
__device__ __forceinline__ void finish_body(const Params& p, float* lds) {
    const int wave = wave_index();
    const int lane = lane_id();
    ModelPtr M = as_const(p.model);
    EV ev(M, lds + wave * (p.slotsPerLane * 4 * 64) + lane);
    const uint32_t nWaves = gridDim.x * (blockDim.x >> 6);
    const uint32_t wave0 = blockIdx.x * (blockDim.x >> 6) + wave;
    const float delta = 0.001f;
    const float inv = -1.0f / delta;
    phase_stamp_after(p, 0, 2048u, 0.0f);
    if (blockIdx.x == 0) {  // the run's counters for the host (mapped pinned memory)
        const uint32_t* src = reinterpret_cast<const uint32_t*>(p.ctr);
        uint32_t* dst = reinterpret_cast<uint32_t*>(p.hostCtr);
        for (uint32_t i = threadIdx.x; i < sizeof(DevCounters) / 4; i += blockDim.x) dst[i] = src[i];
        __threadfence_system();
        // the next run's counters and offsets-scan words (no kernel of this run touches them)
        uint32_t* nx = reinterpret_cast<uint32_t*>(p.ctrNext);
        const uint32_t nextEpoch = p.ctr->epoch + 1u;
        constexpr uint32_t kEpochWord = __builtin_offsetof(DevCounters, epoch) / 4;
        for (uint32_t i = threadIdx.x; i < sizeof(DevCounters) / 4; i += blockDim.x)
            nx[i] = i == 0 ? 0x7fffffffu : (i == kEpochWord ? nextEpoch : 0u);
        for (uint32_t i = threadIdx.x; i < kScanMaxBlocks; i += blockDim.x) p.scanStatusNext[i] = 0ull;
        if (threadIdx.x < 64) {  // the run's totals for the count exchange between parts (RCCL)
            const ShardCtr& sc = p.ctr->shard[threadIdx.x];
            const uint32_t tv = wave_sum(sc.v), tt = wave_sum(sc.t), tp = wave_sum(sc.p), tb = wave_sum(sc.b),
                           ts = wave_sum(sc.s);
            if (threadIdx.x == 0) {
                const uint32_t tot[8] = {p.mpuCount, tv, tt, tp + tb, ts, tp, (uint32_t)p.ctr->firstOverflow,
                                         p.ctr->error};
                for (int i = 0; i < 8; ++i) p.totals[i] = tot[i];
            }
        }
    }
    __shared__ uint32_t sCnt[2 * kShards];
    stage_shard_counts(p, 1, sCnt);            // ShardCtr::v
    stage_shard_counts(p, 2, sCnt + kShards);  // ShardCtr::t
    __syncthreads();
#if PSGPU_FIN_TRI_PREFETCH
    // the wave's first triangle batch loaded before the vertex walk: its records and their
    // MPUs' offsets do not depend on the walk, so their two dependent loads overlap it
    const ShardBatches sbp(sCnt + kShards, p.tShardCap, 64);
    const TriPre tp0 = tri_load(p, sbp, wave0);
#endif
    phase_stamp_after(p, 1, 2048u, 0.0f);
if constexpr (VPW == 16) {
    // a quad of lanes per vertex: lane j of the quad walks point j (p, p + delta e_x,
    // p + delta e_y, p + delta e_z) with the same per-point pruning (GROUP 1) as the
    // 4-point walk below, so every value is the same; lanes 0-2 of the quad then write
    // component j of position, normal and colour
    const ShardBatches sv(sCnt, p.vShardCap, 16);
    const int qj = lane & 3;
    for (uint32_t batch = wave0; batch < sv.total; batch += nWaves) {
        uint32_t shard, first, count;
        sv.locate(batch, &shard, &first, &count);
        uint32_t rec = first + (uint32_t)(lane >> 2);
        const bool valid = rec < count;
        if (!valid) rec = first;
        const size_t ri = (size_t)shard * p.vShardCap + rec;
        const VertexKey K = p.vk[ri];
        const VertexPos R = p.vp[ri];
        const uint32_t gi = (uint32_t)p.offs[K.w] + (K.vidKey & 0xffffu);
        float P[3];  // the root, recomputed from k_vertex's record with its expressions
        vertex_root(edge_segment(p, K.w, K.vidKey >> 16), R.iv, R.scale, P);
        // on its bracketing segment: inside the MPU box (no inf / NaN)
        const bool onSeg = R.scale >= 0.0f && R.scale <= 1.0f;
        float c[3] = {0.0f, 0.0f, 0.0f};
        float nx = 0.0f, ny = 0.0f, nz = 0.0f;
        if (!(p.debug & 32u)) {  // ablation bit 5: no walks
            CullMask cm{0ull, 0ull};
            if (p.cull) {
                if (ballot(!onSeg) == 0ull) cm = cull_mask_mpus(p, K.w);
                else cm = cull_mask_points(M, P[0], P[1], P[2], true, delta);
            }
            const float qx = qj == 1 ? P[0] + delta : P[0];
            const float qy = qj == 2 ? P[1] + delta : P[1];
            const float qz = qj == 3 ? P[2] + delta : P[2];
            float c4[3];
            const float g = ev.template eval<1, true>(qx, qy, qz, cm, c4);
            c[0] = quad_bcast<0>(c4[0]);
            c[1] = quad_bcast<0>(c4[1]);
            c[2] = quad_bcast<0>(c4[2]);
            const float vtx = quad_bcast<0>(g);
            nx = (quad_bcast<1>(g) - vtx) * inv;
            ny = (quad_bcast<2>(g) - vtx) * inv;
            nz = (quad_bcast<3>(g) - vtx) * inv;
            const float im = 1.0f / sqrtf((nx * nx + ny * ny) + nz * nz);
            nx = nx * im;
            ny = ny * im;
            nz = nz * im;
        }
        if (valid && qj < 3 && gi < p.vCap) {  // past vCap: finish() grows and re-runs
            const uint32_t o = gi * 3 + (uint32_t)qj;
            p.pos[o] = qj == 0 ? P[0] : (qj == 1 ? P[1] : P[2]);
            p.nrm[o] = qj == 0 ? nx : (qj == 1 ? ny : nz);
            p.col[o] = qj == 0 ? c[0] : (qj == 1 ? c[1] : c[2]);
        }
    }
} else if constexpr (VPW == 32) {
    // a pair of lanes per vertex: lane j of the pair walks points 2j, 2j + 1 of
    // {p, p + delta e_x, p + delta e_y, p + delta e_z} (per-point pruning, as above); the
    // partner's two values come over DPP; lane j writes component j, lane 0 also component 2
    const ShardBatches sv(sCnt, p.vShardCap, 32);
    const int pj = lane & 1;
    for (uint32_t batch = wave0; batch < sv.total; batch += nWaves) {
        uint32_t shard, first, count;
        sv.locate(batch, &shard, &first, &count);
        uint32_t rec = first + (uint32_t)(lane >> 1);
        const bool valid = rec < count;
        if (!valid) rec = first;
        const size_t ri = (size_t)shard * p.vShardCap + rec;
        const VertexKey K = p.vk[ri];
        const VertexPos R = p.vp[ri];
        const uint32_t gi = (uint32_t)p.offs[K.w] + (K.vidKey & 0xffffu);
        float P[3];  // the root, recomputed from k_vertex's record with its expressions
        vertex_root(edge_segment(p, K.w, K.vidKey >> 16), R.iv, R.scale, P);
        // on its bracketing segment: inside the MPU box (no inf / NaN)
        const bool onSeg = R.scale >= 0.0f && R.scale <= 1.0f;
        float c[3] = {0.0f, 0.0f, 0.0f};
        float nx = 0.0f, ny = 0.0f, nz = 0.0f;
        if (!(p.debug & 32u)) {  // ablation bit 5: no walks
            CullMask cm{0ull, 0ull};
            if (p.cull) {
                if (ballot(!onSeg) == 0ull) cm = cull_mask_mpus(p, K.w);
                else cm = cull_mask_points(M, P[0], P[1], P[2], true, delta);
            }
            // lane 0: p, p + delta e_x; lane 1: p + delta e_y, p + delta e_z
            const float qx[2] = {P[0], pj == 0 ? P[0] + delta : P[0]};
            const float qy[2] = {pj == 1 ? P[1] + delta : P[1], P[1]};
            const float qz[2] = {P[2], pj == 1 ? P[2] + delta : P[2]};
            float g[2], c6[6];
            ev.template evaln<1, true, 2>(qx, qy, qz, cm, g, c6);
            const float o0 = PSGPU_DPP_F(g[0], 0xB1), o1 = PSGPU_DPP_F(g[1], 0xB1);
            const float oc0 = PSGPU_DPP_F(c6[0], 0xB1), oc1 = PSGPU_DPP_F(c6[1], 0xB1),
                        oc2 = PSGPU_DPP_F(c6[2], 0xB1);
            c[0] = pj == 0 ? c6[0] : oc0;
            c[1] = pj == 0 ? c6[1] : oc1;
            c[2] = pj == 0 ? c6[2] : oc2;
            const float vtx = pj == 0 ? g[0] : o0;
            const float g1 = pj == 0 ? g[1] : o1;
            const float g2 = pj == 0 ? o0 : g[0];
            const float g3 = pj == 0 ? o1 : g[1];
            nx = (g1 - vtx) * inv;
            ny = (g2 - vtx) * inv;
            nz = (g3 - vtx) * inv;
            const float im = 1.0f / sqrtf((nx * nx + ny * ny) + nz * nz);
            nx = nx * im;
            ny = ny * im;
            nz = nz * im;
        }
        if (valid && gi < p.vCap) {  // past vCap: finish() grows and re-runs
            const uint32_t o = gi * 3 + (uint32_t)pj;
            p.pos[o] = pj == 0 ? P[0] : P[1];
            p.nrm[o] = pj == 0 ? nx : ny;
            p.col[o] = pj == 0 ? c[0] : c[1];
            if (pj == 0) {
                p.pos[gi * 3 + 2] = P[2];
                p.nrm[gi * 3 + 2] = nz;
                p.col[gi * 3 + 2] = c[2];
            }
        }
    }
} else {
    const ShardBatches sv(sCnt, p.vShardCap, 64);
    for (uint32_t batch = wave0; batch < sv.total; batch += nWaves) {
        uint32_t shard, first, count;
        sv.locate(batch, &shard, &first, &count);
        uint32_t rec = first + (uint32_t)lane;
        const bool valid = rec < count;
        if (!valid) rec = first;
        const size_t ri = (size_t)shard * p.vShardCap + rec;
        const VertexKey K = p.vk[ri];
        const VertexPos R = p.vp[ri];
        const uint32_t gi = (uint32_t)p.offs[K.w] + (K.vidKey & 0xffffu);
        float P[3];  // the root, recomputed from k_vertex's record with its expressions
        vertex_root(edge_segment(p, K.w, K.vidKey >> 16), R.iv, R.scale, P);
        // on its bracketing segment: inside the MPU box (no inf / NaN)
        const bool onSeg = R.scale >= 0.0f && R.scale <= 1.0f;
        float c[3] = {0.0f, 0.0f, 0.0f};
        float nx = 0.0f, ny = 0.0f, nz = 0.0f;
        phase_stamp_after(p, 2, 2048u, P[0] + P[1] + P[2]);  // records in, root recomputed
        if (!(p.debug & 32u)) {  // ablation bit 5: no walks
            // vertices on their segments: the MPU masks (boxes grown by delta) cover p and
            // every normal sample; otherwise the wave's own box grown by delta
            CullMask cm{0ull, 0ull};
            if (p.cull) {
                if (ballot(!onSeg) == 0ull) cm = cull_mask_mpus(p, K.w);
                else cm = cull_mask_points(M, P[0], P[1], P[2], true, delta);
            }
            phase_stamp_after(p, 3, 2048u, __uint_as_float((uint32_t)(cm.lo ^ cm.hi)));
#if PSGPU_FIN_PHASES
            const uint64_t nvalid = (uint64_t)__popcll(ballot(valid));
            if ((p.debug & 2048u) && p.stamps && lane == 0) {  // phase word 7: live primitives, vertices
                const uint32_t sw = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
                if (sw < p.stampCap)
                    p.stamps[3 * (size_t)kNumStampKernels * p.stampCap + 8 * (size_t)sw + 7] =
                        (uint64_t)(128 - __popcll(cm.lo) - __popcll(cm.hi)) | (nvalid << 16);
            }
#endif
            // value + colour at p and the normal's per-point fieldValue at p + delta*e_a
            // (:1598-1622) as four points of one walk (the colour of points 1-3 is dead
            // code); then SimdNormalize (rsqrt -> IEEE 1/sqrtf)
            const float qx[4] = {P[0], P[0] + delta, P[0], P[0]};
            const float qy[4] = {P[1], P[1], P[1] + delta, P[1]};
            const float qz[4] = {P[2], P[2], P[2], P[2] + delta};
            float g[4], c4[12];
            ev.template evaln<1, true, 4>(qx, qy, qz, cm, g, c4);
            phase_stamp_after(p, 4, 2048u, g[0] + g[1] + g[2] + g[3] + c4[0] + c4[1] + c4[2]);
            c[0] = c4[0];
            c[1] = c4[1];
            c[2] = c4[2];
            const float vtx = g[0];
            nx = (g[1] - vtx) * inv;
            ny = (g[2] - vtx) * inv;
            nz = (g[3] - vtx) * inv;
            const float im = 1.0f / sqrtf((nx * nx + ny * ny) + nz * nz);
            nx = nx * im;
            ny = ny * im;
            nz = nz * im;
        }
        if (valid && gi < p.vCap) {  // past vCap: finish() grows and re-runs
            p.pos[gi * 3 + 0] = P[0];
            p.pos[gi * 3 + 1] = P[1];
            p.pos[gi * 3 + 2] = P[2];
            p.nrm[gi * 3 + 0] = nx;
            p.nrm[gi * 3 + 1] = ny;
            p.nrm[gi * 3 + 2] = nz;
            p.col[gi * 3 + 0] = c[0];
            p.col[gi * 3 + 1] = c[1];
            p.col[gi * 3 + 2] = c[2];
        }
        phase_stamp_after(p, 5, 2048u, __uint_as_float(gi));
    }
}
    if (p.debug & 64u) return;  // ablation bit 6: no triangles
    const ShardBatches sb(sCnt + kShards, p.tShardCap, 64);
    uint32_t batch0 = wave0;
#if PSGPU_FIN_TRI_PREFETCH
    tri_store(p, tp0);
    batch0 += nWaves;
#endif
    for (uint32_t batch = batch0; batch < sb.total; batch += nWaves) {
        uint32_t shard, first, count;
        sb.locate(batch, &shard, &first, &count);
        const uint32_t t = first + lane;
        if (t >= count) continue;
        const TriRec R = p.tq[(size_t)shard * p.tShardCap + t];
        const uint64_t o = p.offs[((R.a >> 12) << 6) | shard];  // the record's shard is w & 63
        const uint32_t gt = (uint32_t)(o >> 32) + (R.a & 2047u);
        const uint32_t base = (uint32_t)o;
        if (gt >= p.tCap) continue;  // finish() grows and re-runs
        p.tris[gt * 3 + 0] = base + (R.b & 2047u);
        p.tris[gt * 3 + 1] = base + ((R.b >> 11) & 2047u);
        p.tris[gt * 3 + 2] = base + ((R.b >> 22) | (((R.a >> 11) & 1u) << 10));
    }
    phase_stamp_after(p, 6, 2048u, 0.0f);
}

// k_front (PSGPU_OPT_FRONT): k_precheck and k_mpu as one launch for small launches, with a
// dataflow hand-over instead of the kernel boundary (no grid barrier: r05's barrier version,
// k_front v1-v3 in profiles/r05_front_ab.txt, was slower than the boundary).  Blocks
// [0, preBlocks) run S1 exactly as k_precheck and publish each queued MPU (sc1 entry and
// culling mask, then the entry's ready word with the run's tag) into sub-queue blockIdx & 7;
// when all of a block's waves have published, its last wave counts the block done for its
// sub-queue.  The blocks after them run S2-S3 exactly as k_mpu on entries as they are
// published.  Every S1 block is dispatched before any S2 block (in-order dispatch), so a
// waiting S2 block never holds back the S1 block it waits for; every wait is bounded and a
// timeout fails the run as a protocol error (finish re-runs it as separate launches).
template <class EV, int SPLIT>
__device__ __forceinline__ void front_body(const Params& p, unsigned char* smem) {
    const uint64_t t0 = (p.stamps || p.spans) ? stamp_now() : 0ull;
    if (blockIdx.x < p.preBlocks) {  // block-uniform
        __shared__ uint32_t sArrive;
        if (threadIdx.x == 0) {
            sArrive = 0u;
            if (p.debug & (1u << 27)) {  // test hook: the S1 blocks publish ~40 us late
                const uint64_t h0 = stamp_now();
                while (stamp_now() - h0 < 4000u) __builtin_amdgcn_s_sleep(8);
            }
        }
        __syncthreads();
        precheck_body<EV, SPLIT, true>(p, reinterpret_cast<float*>(smem));
        if (p.stamps) stamp_end(p, 0, t0, blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
        if (p.spans) span_end(p, 0, t0);
        // the block's arrival: each wave after its own stores left it; the last one signals
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane_id() == 0 && atomicAdd(&sArrive, 1u) == (blockDim.x >> 6) - 1u)
            __hip_atomic_fetch_add(&p.ctr->shard[blockIdx.x & 7u].s1Done, 1u, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
    } else {
        const uint32_t blk = blockIdx.x - p.preBlocks;
        uint32_t item = 0xffffffffu;
        mpu_body<EV, SPLIT, true>(p, smem, &item, blk);
        if (p.stamps) stamp_end(p, 1, t0, item, blk);
        if (p.spans) span_end(p, 1, t0);
    }
}

// k_surface's wait for the offsets scan (every scan block released its offsets), bounded: a
// broken protocol flags the run (error bit 1) instead of hanging the device.
// The flag reaches the host through words block 0 never overwrites (surfaceErr, raised with
// a plain store; totals[7], raised atomically), so a timeout after block 0 published the
// counters still fails the run, and psgpu_finish re-runs it as k_vertex + k_finish.
__device__ __forceinline__ void surface_wait_scan(const Params& p) {
    if (lane_id() == 0) {
        uint32_t spins = 0;
        // test hook (PSGPU_OPT_DEBUG bit 25): a bound far below the scan blocks' delay
        const uint32_t bound = (p.debug & (1u << 25)) ? 4u : (1u << 22);
        while (__hip_atomic_load(&p.ctr->scanDone, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < p.scanBlocks) {
            __builtin_amdgcn_s_sleep(2);
            if (++spins > bound) {
                atomicOr(&p.ctr->error, 2u);
                atomicOr(&p.totals[7], 2u);
                p.hostCtr->surfaceErr = 2u;
                __threadfence_system();
                break;
            }
        }
    }
    // no agent-scope acquire here: on gfx950 it invalidates the XCD's L2 for every kernel on it
    // (measured: a 1/8 share 0.028 vs 0.015 ms/step).  The offsets are read with agent-scope
    // loads instead (surface_offs), which bypass the non-coherent caches and are issued only
    // after the flag was seen.
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
}
// an offsets word written by this launch's scan blocks (released before their scanDone count)
__device__ __forceinline__ uint64_t surface_offs(const Params& p, uint32_t i) {
    return __hip_atomic_load(&p.offs[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// k_surface (PSGPU_OPT_FUSED_SURFACE): k_vertex and k_finish in one launch for small launches
// (a rank's share; the launch floor, not the work, sets their step: DESIGN.md §5).  A quad of
// lanes per vertex for both walks -- the root's 4 edge samples (k_vertex's quad layout), then
// value + colour at the root and its 3 normal samples (k_finish's quad layout) -- with the
// root's bracket and scale kept in registers instead of the vertex record.  The first blocks
// run the offsets scan as in k_vertex and release it; a wave waits for every scan block only
// before its first mesh write.  Same values as the two kernels: the same expressions on the
// same records and the same culling masks.  The scan blocks have the lowest block ids, so they
// are dispatched before any waiting block of their XCD: the wait cannot starve them.
// VPW 64 (k_surface_w, PSGPU_OPT_FUSED_SURFACE 3): one lane per vertex for both walks -- the root's
// 4 edge samples as k_vertex's wide layout walks them, then value + colour and the 3 normal samples
// as k_finish's 64-vertex layout -- for launches whose vertices fill the device.
template <class EV, int VPW = 16>
__device__ __forceinline__ void surface_body(const Params& p, float* lds) {
    const int wave = wave_index();
    const int lane = lane_id();
    ModelPtr M = as_const(p.model);
    EV ev(M, lds + wave * (p.slotsPerLane * 4 * 64) + lane);
    const uint32_t nWaves = gridDim.x * (blockDim.x >> 6);
    const uint32_t wave0 = blockIdx.x * (blockDim.x >> 6) + wave;
    const float delta = 0.001f;
    const float inv = -1.0f / delta;
    if (blockIdx.x < p.scanBlocks) {  // block-uniform
        scan_counts_block(p, blockIdx.x);
        __syncthreads();  // the block's offsets stores are in L2
        if (threadIdx.x == 0) {
            if (p.debug & (1u << 25)) {  // test hook: the scan blocks count themselves done ~40 us late
                const uint64_t t0 = stamp_now();
                while (stamp_now() - t0 < 4000u) __builtin_amdgcn_s_sleep(8);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");  // ... and written back for the other XCDs
            __hip_atomic_fetch_add(&p.ctr->scanDone, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    if (blockIdx.x == 0) {  // k_finish's block-0 duties (finish_body), once every scan block is done:
        // a look-back timeout of any scan block (error bit 0) is then in the counters it publishes
        if (threadIdx.x < 64) surface_wait_scan(p);
        __syncthreads();
        const uint32_t err = __hip_atomic_load(&p.ctr->error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t* src = reinterpret_cast<const uint32_t*>(p.ctr);
        uint32_t* dst = reinterpret_cast<uint32_t*>(p.hostCtr);
        constexpr uint32_t kErrWord = __builtin_offsetof(DevCounters, error) / 4, kSurfWord = __builtin_offsetof(DevCounters, surfaceErr) / 4;
        for (uint32_t i = threadIdx.x; i < sizeof(DevCounters) / 4; i += blockDim.x)
            if (i != kSurfWord) dst[i] = i == kErrWord ? err : src[i];
        __threadfence_system();
        uint32_t* nx = reinterpret_cast<uint32_t*>(p.ctrNext);
        const uint32_t nextEpoch = p.ctr->epoch + 1u;
        constexpr uint32_t kEpochWord = __builtin_offsetof(DevCounters, epoch) / 4;
        for (uint32_t i = threadIdx.x; i < sizeof(DevCounters) / 4; i += blockDim.x)
            nx[i] = i == 0 ? 0x7fffffffu : (i == kEpochWord ? nextEpoch : 0u);
        for (uint32_t i = threadIdx.x; i < kScanMaxBlocks; i += blockDim.x) p.scanStatusNext[i] = 0ull;
        if (threadIdx.x < 64) {
            const ShardCtr& sc = p.ctr->shard[threadIdx.x];
            const uint32_t tv = wave_sum(sc.v), tt = wave_sum(sc.t), tp = wave_sum(sc.p), tb = wave_sum(sc.b),
                           ts = wave_sum(sc.s);
            if (threadIdx.x == 0) {
                const uint32_t tot[7] = {p.mpuCount, tv, tt, tp + tb, ts, tp, (uint32_t)p.ctr->firstOverflow};
                for (int i = 0; i < 7; ++i) p.totals[i] = tot[i];
                if (err) atomicOr(&p.totals[7], err);  // raised, never stored: zeroed by k_precheck
            }
        }
    }
    __shared__ uint32_t sCnt[2 * kShards];
    stage_shard_counts(p, 1, sCnt);            // ShardCtr::v
    stage_shard_counts(p, 2, sCnt + kShards);  // ShardCtr::t
    __syncthreads();
    bool scanSeen = blockIdx.x == 0;  // block 0 waited above
if constexpr (VPW == 64) {
    const ShardBatches sw(sCnt, p.vShardCap, 64);
    for (uint32_t batch = wave0; batch < sw.total; batch += nWaves) {
        uint32_t shard, first, count;
        sw.locate(batch, &shard, &first, &count);
        uint32_t rec = first + (uint32_t)lane;
        const bool valid = rec < count;
        if (!valid) rec = first;
        const size_t ri = (size_t)shard * p.vShardCap + rec;
        const VertexKey K = p.vk[ri];
        const EdgeSeg E = edge_segment(p, K.w, K.vidKey >> 16);
        // the root: the lane's 4 edge samples as one 4-point walk (vertex_body, 64 per wave)
        float xs[4], ys[4], zs[4], fs[4];
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2) {
            xs[s2] = edge_sample(E.e[0], E.d[0], s2);
            ys[s2] = edge_sample(E.e[1], E.d[1], s2);
            zs[s2] = edge_sample(E.e[2], E.d[2], s2);
        }
        CullMask cmv{0ull, 0ull};
        if (p.cull) cmv = cull_mask_mpus(p, K.w);
        if (p.debug & 256u) {  // ablation bit 8: no phase-A walk
#pragma unroll
            for (int s2 = 0; s2 < 4; ++s2) fs[s2] = xs[s2];
        } else {
            ev.template evaln<0, false, 4>(xs, ys, zs, cmv, fs, nullptr);
        }
        const bool st0 = fs[0] >= 0.5f;
        const int iv = ((fs[1] >= 0.5f) != st0) ? 1 : (((fs[2] >= 0.5f) != st0) ? 2 : 3);
        const float fa = iv == 1 ? fs[0] : (iv == 2 ? fs[1] : fs[2]);
        const float fb = iv == 1 ? fs[1] : (iv == 2 ? fs[2] : fs[3]);
        const float scale = (0.5f - fa) / (fb - fa);
        // value, colour and normal at the root (finish_body, 64 per wave)
        float P[3];
        vertex_root(E, (uint32_t)iv, scale, P);
        const bool onSeg = scale >= 0.0f && scale <= 1.0f;
        float c[3] = {0.0f, 0.0f, 0.0f};
        float nx = 0.0f, ny = 0.0f, nz = 0.0f;
        if (!(p.debug & 32u)) {  // ablation bit 5: no walks
            CullMask cm{0ull, 0ull};
            if (p.cull) {
                if (ballot(!onSeg) == 0ull) cm = cmv;  // cull_mask_mpus(p, K.w), as just made
                else cm = cull_mask_points(M, P[0], P[1], P[2], true, delta);
            }
            const float qx[4] = {P[0], P[0] + delta, P[0], P[0]};
            const float qy[4] = {P[1], P[1], P[1] + delta, P[1]};
            const float qz[4] = {P[2], P[2], P[2], P[2] + delta};
            float g[4], c4[12];
            ev.template evaln<1, true, 4>(qx, qy, qz, cm, g, c4);
            c[0] = c4[0];
            c[1] = c4[1];
            c[2] = c4[2];
            const float vtx = g[0];
            nx = (g[1] - vtx) * inv;
            ny = (g[2] - vtx) * inv;
            nz = (g[3] - vtx) * inv;
            const float im = 1.0f / sqrtf((nx * nx + ny * ny) + nz * nz);
            nx = nx * im;
            ny = ny * im;
            nz = nz * im;
        }
        if (!scanSeen) {
            surface_wait_scan(p);
            scanSeen = true;
        }
        const uint32_t gi = (uint32_t)surface_offs(p, K.w) + (K.vidKey & 0xffffu);
        if (valid && gi < p.vCap) {  // past vCap: finish() grows and re-runs
            p.pos[gi * 3 + 0] = P[0];
            p.pos[gi * 3 + 1] = P[1];
            p.pos[gi * 3 + 2] = P[2];
            p.nrm[gi * 3 + 0] = nx;
            p.nrm[gi * 3 + 1] = ny;
            p.nrm[gi * 3 + 2] = nz;
            p.col[gi * 3 + 0] = c[0];
            p.col[gi * 3 + 1] = c[1];
            p.col[gi * 3 + 2] = c[2];
        }
    }
} else {
    const ShardBatches sv(sCnt, p.vShardCap, 16);
    const int qj = lane & 3;
    for (uint32_t batch = wave0; batch < sv.total; batch += nWaves) {
        uint32_t shard, first, count;
        sv.locate(batch, &shard, &first, &count);
        uint32_t rec = first + (uint32_t)(lane >> 2);
        const bool valid = rec < count;
        if (!valid) rec = first;
        const size_t ri = (size_t)shard * p.vShardCap + rec;
        const VertexKey K = p.vk[ri];
        const EdgeSeg E = edge_segment(p, K.w, K.vidKey >> 16);
        // the root: lane j of the quad walks edge sample j (vertex_body, 16 per wave)
        const float sx = edge_sample(E.e[0], E.d[0], qj);
        const float sy = edge_sample(E.e[1], E.d[1], qj);
        const float sz = edge_sample(E.e[2], E.d[2], qj);
        CullMask cmv{0ull, 0ull};
        if (p.cull) cmv = cull_mask_mpus(p, K.w);
        float fv;
        if (p.debug & 256u) fv = sx;  // ablation bit 8: no phase-A walk
        else fv = ev.template eval<4, false>(sx, sy, sz, cmv, nullptr);
        const float fs0 = quad_bcast<0>(fv), fs1 = quad_bcast<1>(fv), fs2 = quad_bcast<2>(fv), fs3 = quad_bcast<3>(fv);
        const bool st0 = fs0 >= 0.5f;
        const int iv = ((fs1 >= 0.5f) != st0) ? 1 : (((fs2 >= 0.5f) != st0) ? 2 : 3);
        const float fa = iv == 1 ? fs0 : (iv == 2 ? fs1 : fs2);
        const float fb = iv == 1 ? fs1 : (iv == 2 ? fs2 : fs3);
        const float scale = (0.5f - fa) / (fb - fa);
        // value, colour and normal at the root (finish_body, 16 per wave)
        float P[3];
        vertex_root(E, (uint32_t)iv, scale, P);
        const bool onSeg = scale >= 0.0f && scale <= 1.0f;
        float c[3] = {0.0f, 0.0f, 0.0f};
        float nx = 0.0f, ny = 0.0f, nz = 0.0f;
        if (!(p.debug & 32u)) {  // ablation bit 5: no walks
            CullMask cm{0ull, 0ull};
            if (p.cull) {
                if (ballot(!onSeg) == 0ull) cm = cmv;  // cull_mask_mpus(p, K.w), as just made
                else cm = cull_mask_points(M, P[0], P[1], P[2], true, delta);
            }
            const float qx = qj == 1 ? P[0] + delta : P[0];
            const float qy = qj == 2 ? P[1] + delta : P[1];
            const float qz = qj == 3 ? P[2] + delta : P[2];
            float c4[3];
            const float g = ev.template eval<1, true>(qx, qy, qz, cm, c4);
            c[0] = quad_bcast<0>(c4[0]);
            c[1] = quad_bcast<0>(c4[1]);
            c[2] = quad_bcast<0>(c4[2]);
            const float vtx = quad_bcast<0>(g);
            nx = (quad_bcast<1>(g) - vtx) * inv;
            ny = (quad_bcast<2>(g) - vtx) * inv;
            nz = (quad_bcast<3>(g) - vtx) * inv;
            const float im = 1.0f / sqrtf((nx * nx + ny * ny) + nz * nz);
            nx = nx * im;
            ny = ny * im;
            nz = nz * im;
        }
        if (!scanSeen) {
            surface_wait_scan(p);
            scanSeen = true;
        }
        const uint32_t gi = (uint32_t)surface_offs(p, K.w) + (K.vidKey & 0xffffu);
        if (valid && qj < 3 && gi < p.vCap) {  // past vCap: finish() grows and re-runs
            const uint32_t o = gi * 3 + (uint32_t)qj;
            p.pos[o] = qj == 0 ? P[0] : (qj == 1 ? P[1] : P[2]);
            p.nrm[o] = qj == 0 ? nx : (qj == 1 ? ny : nz);
            p.col[o] = qj == 0 ? c[0] : (qj == 1 ? c[1] : c[2]);
        }
    }
}
    if (p.debug & 64u) return;  // ablation bit 6: no triangles
    const ShardBatches sb(sCnt + kShards, p.tShardCap, 64);
    if (wave0 < sb.total && !scanSeen) surface_wait_scan(p);
    for (uint32_t batch = wave0; batch < sb.total; batch += nWaves) {
        uint32_t shard, first, count;
        sb.locate(batch, &shard, &first, &count);
        const uint32_t t = first + lane;
        if (t >= count) continue;
        const TriRec R = p.tq[(size_t)shard * p.tShardCap + t];
        const uint64_t o = surface_offs(p, ((R.a >> 12) << 6) | shard);  // the record's shard is w & 63
        const uint32_t gt = (uint32_t)(o >> 32) + (R.a & 2047u);
        const uint32_t base = (uint32_t)o;
        if (gt >= p.tCap) continue;  // finish() grows and re-runs
        p.tris[gt * 3 + 0] = base + (R.b & 2047u);
        p.tris[gt * 3 + 1] = base + ((R.b >> 11) & 2047u);
        p.tris[gt * 3 + 2] = base + ((R.b >> 22) | (((R.a >> 11) & 1u) << 10));
    }
}

// Field probe for tests: mode 0 quads of consecutive points, 1 per point, 2 + colour.
template <class EV>
__device__ __forceinline__ void probe_body(const Params& p, float* lds, const float* xyz, float* out, float* colOut,
                                           uint32_t n, int mode) {
    const int wave = wave_index();
    ModelPtr M = as_const(p.model);
    EV ev(M, lds + wave * (p.slotsPerLane * 4 * 64) + lane_id());
    uint32_t i = blockIdx.x * 256 + threadIdx.x;
    const bool valid = i < n;
    if (!valid) i = (n ? n - 1 : 0);
    const float x = xyz[3 * i], y = xyz[3 * i + 1], z = xyz[3 * i + 2];
    const CullMask cm = cull_mask_points(M, x, y, z, p.cull != 0);
    float c[3] = {0.0f, 0.0f, 0.0f};
    float f;
    if (mode == 0) f = ev.template eval<4, false>(x, y, z, cm, nullptr);
    else if (mode == 1) f = ev.template eval<1, false>(x, y, z, cm, nullptr);
    else f = ev.template eval<1, true>(x, y, z, cm, c);
    if (valid) {
        out[i] = f;
        if (colOut) {
            colOut[3 * i] = c[0];
            colOut[3 * i + 1] = c[1];
            colOut[3 * i + 2] = c[2];
        }
    }
}

}  // namespace psgpu

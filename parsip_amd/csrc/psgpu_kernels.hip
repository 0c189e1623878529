// psgpu_kernels.hip — CDNA4 (gfx950) kernels of the BlobTree polygonizer.
//
// Pipeline for one polygonization of MPUs [begin, begin+count) (the reference's
// Polygonize + CMPUProcessor, PS_Polygonizer.cpp:315-385, 441-829):
//
//   k_precheck  8 lanes per MPU, 2 quads: S1 corner test F>0          (:483-540)
//   k_compact   one workgroup: ordered list of MPUs that passed S1
//   k_mpu       one wavefront per passing MPU: S2 8^3 field cache in LDS
//               (quads of 4 z-consecutive corners, :550-610), S3 cell configs
//               (:647-691), vertex ownership + wave prefix sums for the reference's
//               discovery order (:703-816), triangle records           (:816-825)
//   k_scan      one workgroup: per-MPU vertex/triangle offsets (compact mesh)
//   k_vertex    one quad per vertex: S4 4-sample root bracket (:722-762), then S5
//               field+colour and the 3 normal samples                  (:764-807)
//   k_tris      triangle records -> global vertex ids
//
// Every fp32 expression keeps the reference's operation order; the library is
// built with -ffp-contract=off, IEEE division/sqrt and IEEE denormals.  max/min are
// written as the SSE definitions (a>b?a:b, a<b?a:b) so NaN and -0 propagate
// exactly as _mm_max_ps/_mm_min_ps (PS_SIMDVecN.h:388-389).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "psgpu_model.h"

namespace psgpu {

__constant__ int8_t c_tri[256][16];
__constant__ uint8_t c_ntri[256];
__constant__ uint8_t c_corner1[12];
__constant__ uint8_t c_axis[12];



// The model is read through the constant address space so that every wave-uniform
// access (the walk program, op boxes, primitive parameters) becomes an s_load into
// SGPRs through the scalar cache instead of a per-lane vector load.
typedef const __attribute__((address_space(4))) DevModel* ModelPtr;
typedef const __attribute__((address_space(4))) DevPrim CPrim;
typedef const __attribute__((address_space(4))) DevOp COp;
__device__ __forceinline__ ModelPtr as_const(const DevModel* m) { return (ModelPtr)m; }

__device__ __forceinline__ Instr load_instr(ModelPtr M, int pc) {
    typedef const __attribute__((address_space(4))) uint32_t* CU32;
    const CU32 w = (CU32)(&M->instr[pc]);
    const uint32_t words[3] = {w[0], w[1], w[2]};
    Instr I;
    __builtin_memcpy(&I, words, 12);
    return I;
}

__device__ __forceinline__ float max_ref(float a, float b) { return a > b ? a : b; }
__device__ __forceinline__ float min_ref(float a, float b) { return a < b ? a : b; }
__device__ __forceinline__ float m01(bool c) { return c ? 1.0f : 0.0f; }
__device__ __forceinline__ int lane_id() { return __lane_id(); }

__device__ __forceinline__ uint64_t ballot(bool v) { return __ballot(v); }

// 1 if any lane of this lane's 4-lane group has v set.
__device__ __forceinline__ bool quad_any(bool v) {
    uint64_t b = ballot(v);
    uint64_t t = b | (b >> 1);
    t |= t >> 2;
    t &= 0x1111111111111111ull;
    t |= t << 1;
    t |= t << 2;
    return (t >> lane_id()) & 1ull;
}

// ---------------------------------------------------------------------------
// computePrimitiveField (PS_Polygonizer.cpp:934-1179) + Wyvill (h:397-407)
__device__ __forceinline__ float prim_field(CPrim& P, float pX, float pY, float pZ) {
    float x = pX, y = pY, z = pZ;
    if (P.hasMatrix) {
        const __attribute__((address_space(4))) float* M = P.mat;
        x = ((M[0] * pX + M[1] * pY) + M[2] * pZ) + M[3];
        y = ((M[4] * pX + M[5] * pY) + M[6] * pZ) + M[7];
        z = ((M[8] * pX + M[9] * pY) + M[10] * pZ) + M[11];
    }
    float d2 = 0.0f;
    switch (P.type) {
    case 3: {  // Point
        float dx = P.pos[0] - x, dy = P.pos[1] - y, dz = P.pos[2] - z;
        d2 = (dx * dx + dy * dy) + dz * dz;
    } break;
    case 2: {  // Line (pos = start, dir = end), projection not clamped
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
    } break;
    case 0: {  // Cylinder (pos, axis dir, r = resX, h = resY)
        float px = x - P.pos[0], py = y - P.pos[1], pz = z - P.pos[2];
        float yy = (px * P.dir[0] + py * P.dir[1]) + pz * P.dir[2];
        float rr = ((px * px + py * py) + pz * pz) - yy * yy;
        float xx = max_ref(0.0f, __fsqrt_rn(rr) - P.res[0]);
        float mask = m01(yy > 0.0f);
        yy = mask * max_ref(0.0f, yy - P.res[1]) + (1.0f - mask) * yy;
        d2 = xx * xx + yy * yy;
    } break;
    case 7:  // Triangle: distance stub
        d2 = 3.402823466e+38f;
        break;
    case 6: {  // Cube (half side resX)
        float side = P.res[0], mside = -1.0f * P.res[0];
        float dif[3] = {x - P.pos[0], y - P.pos[1], z - P.pos[2]};
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            float mm = m01(mside > dif[a]);
            float mp = m01(dif[a] > side);
            float dl = (dif[a] + side) * mm + (dif[a] - side) * mp;
            d2 = (a == 0) ? dl * dl : d2 + dl * dl;
        }
    } break;
    case 1: {  // Disc
        float dX = x - P.pos[0], dY = y - P.pos[1], dZ = z - P.pos[2];
        float nX = P.dir[0], nY = P.dir[1], nZ = P.dir[2], r = P.res[0];
        float dot = (nX * dX + nY * dY) + nZ * dZ;
        float rX = dX - nX * dot, rY = dY - nY * dot, rZ = dZ - nZ * dot;
        dot = (rX * rX + rY * rY) + rZ * rZ;
        float rs = 1.0f / __fsqrt_rn(dot);
        rX = rX * rs; rY = rY * rs; rZ = rZ * rs;
        nX = r * rX - dX; nY = r * rY - dY; nZ = r * rZ - dZ;
        float mask = m01(r * r >= dot);
        d2 = mask * (((dX * dX + dY * dY) + dZ * dZ) - dot) + (1.0f - mask) * ((nX * nX + nY * nY) + nZ * nZ);
    } break;
    case 4: {  // Ring
        float dX = x - P.pos[0], dY = y - P.pos[1], dZ = z - P.pos[2];
        float nX = P.dir[0], nY = P.dir[1], nZ = P.dir[2], r = P.res[0];
        float dot = (nX * dX + nY * dY) + nZ * dZ;
        float rX = dX - nX * dot, rY = dY - nY * dot, rZ = dZ - nZ * dot;
        dot = (rX * rX + rY * rY) + rZ * rZ;
        float mask = m01(dot == 0.0f);
        dot = 1.0f / __fsqrt_rn(dot);
        rX = rX * dot; rY = rY * dot; rZ = rZ * dot;
        nX = r * rX - dX; nY = r * rY - dY; nZ = r * rZ - dZ;
        d2 = mask * (((r * r + dX * dX) + dY * dY) + dZ * dZ) + (1.0f - mask) * ((nX * nX + nY * nY) + nZ * nZ);
    } break;
    default:  // no case in the reference switch: dist2 stays 0, field 1
        break;
    }
    float t = 1.0f - d2;
    float f = (t * t) * t;
    return max_ref(0.0f, f);
}

// ---------------------------------------------------------------------------
// Exact culling (an optimisation that never changes a bit of output): a primitive
// whose support (computed dist2 >= 1 => field exactly +0) cannot reach any point of
// the wave gets field +0 without evaluating it.  The wave's points lie in the AABB
// [bmin,bmax]; with centre c and half-diagonal h, every point q satisfies
// d(q) >= d(c) - h for the 1-Lipschitz distance functions of Point, Line (infinite
// line), Cube (box) and the capped Cylinder with |axis| = 1.  The host marks a prim
// cullable only when no matrix is attached and its dist2 cannot be NaN away from the
// skeleton (Cylinder additionally requires the AABB to stay clear of the infinite
// axis line, where the reference's sqrt of a rounded-negative value gives NaN).
// Margin 1.02 on d^2 covers fp32 rounding of the reference formulas by > 1e3 ulps.
__device__ __forceinline__ float cull_dist(CPrim& P, float cx, float cy, float cz, float* axisDist) {
    *axisDist = 1e30f;
    switch (P.type) {
    case 3: {
        float dx = cx - P.pos[0], dy = cy - P.pos[1], dz = cz - P.pos[2];
        return sqrtf(dx * dx + dy * dy + dz * dz);
    }
    case 2: {
        float ux = P.dir[0] - P.pos[0], uy = P.dir[1] - P.pos[1], uz = P.dir[2] - P.pos[2];
        float dx = cx - P.pos[0], dy = cy - P.pos[1], dz = cz - P.pos[2];
        float uu = ux * ux + uy * uy + uz * uz;
        float t = (dx * ux + dy * uy + dz * uz) / uu;
        float ex = dx - t * ux, ey = dy - t * uy, ez = dz - t * uz;
        return sqrtf(ex * ex + ey * ey + ez * ez);
    }
    case 0: {
        float dx = cx - P.pos[0], dy = cy - P.pos[1], dz = cz - P.pos[2];
        float yy = dx * P.dir[0] + dy * P.dir[1] + dz * P.dir[2];
        float rr = dx * dx + dy * dy + dz * dz - yy * yy;
        float rad = sqrtf(rr > 0.0f ? rr : 0.0f);
        *axisDist = rad;
        float ex = rad - P.res[0];
        ex = ex > 0.0f ? ex : 0.0f;
        float ey = yy < 0.0f ? -yy : (yy > P.res[1] ? yy - P.res[1] : 0.0f);
        return sqrtf(ex * ex + ey * ey);
    }
    case 6: {
        float s = P.res[0];
        float d[3] = {cx - P.pos[0], cy - P.pos[1], cz - P.pos[2]};
        float acc = 0.0f;
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            float e = fabsf(d[a]) - s;
            e = e > 0.0f ? e : 0.0f;
            acc += e * e;
        }
        return sqrtf(acc);
    }
    default:
        return 0.0f;
    }
}

// Per-wave cull mask over prims [0,128): bit set => field is exactly +0 for every
// point of this wave.  Lane l tests prims l and l+64 against the wave AABB.
struct CullMask {
    uint64_t lo, hi;
};

__device__ __forceinline__ float wave_min(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = fminf(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
    return v;
}

__device__ __forceinline__ CullMask make_cull_mask(ModelPtr M, float px, float py, float pz, bool enable) {
    CullMask cm{0ull, 0ull};
    if (!enable) return cm;
    float x0 = wave_min(px), x1 = wave_max(px);
    float y0 = wave_min(py), y1 = wave_max(py);
    float z0 = wave_min(pz), z1 = wave_max(pz);
    // any NaN coordinate (fminf/fmaxf would hide it) or a non-finite box disables culling
    if (ballot(!(px == px) || !(py == py) || !(pz == pz)) != 0ull) return cm;
    if (!(x1 - x0 < 1e30f && y1 - y0 < 1e30f && z1 - z0 < 1e30f)) return cm;
    float cx = 0.5f * (x0 + x1), cy = 0.5f * (y0 + y1), cz = 0.5f * (z0 + z1);
    float hx = 0.5f * (x1 - x0), hy = 0.5f * (y1 - y0), hz = 0.5f * (z1 - z0);
    float h = sqrtf(hx * hx + hy * hy + hz * hz) * 1.0001f + 1e-6f;
    const int n = (int)M->ctPrims;
#pragma unroll
    for (int half = 0; half < 2; ++half) {
        int i = half * 64 + lane_id();
        bool cull = false;
        if (i < n) {
            CPrim& P = M->prims[i];
            if (P.cullable) {
                float ad;
                float d = cull_dist(P, cx, cy, cz, &ad) - h;
                cull = d > 0.0f && d * d >= 1.02f;
                if (P.type == 0) cull = cull && (ad - h > 0.05f);
            } else if (P.type == 7) {
                cull = true;  // Triangle stub: dist2 = FLT_MAX -> field +0 at every point
            }
        }
        uint64_t b = ballot(cull);
        if (half == 0) cm.lo = b; else cm.hi = b;
    }
    return cm;
}

__device__ __forceinline__ bool culled(const CullMask& cm, uint32_t i) {
    return i < 64 ? ((cm.lo >> i) & 1ull) : ((cm.hi >> (i - 64)) & 1ull);
}

// ---------------------------------------------------------------------------
// FieldComputer::fieldValue (:1184-1376) over the flattened walk program.
//   GROUP 4: pruning decided per 4-lane group (S1/S2 quads, S4 edge samples)
//   GROUP 1: per lane (S5: the reference evaluates 4 identical lanes)
//   COLOR  : also fieldValueAndColor's colour walk (:1378-1551).  No subtree is
//            skipped; lanes inside a pruned subtree see field 0 for every prim and
//            op there (the reference's never-written arrays, defined as zero).
// `sl` is this lane's value stack in LDS (stride 64 floats); colour mode stores
// 4 floats per slot (field, r, g, b).
template <int GROUP, bool COLOR>
__device__ __forceinline__ float walk(ModelPtr M, float px, float py, float pz, float* __restrict__ sl,
                      const CullMask& cm, float* colOut) {
    const int n = (int)M->nInstr;
    const bool noOps = M->ctOps == 0;
    int resume = 0;
    float last = 0.0f, acc = 0.0f;
    float lc0 = 0.0f, lc1 = 0.0f, lc2 = 0.0f;
    constexpr int SW = COLOR ? 4 : 1;  // floats per slot
    for (int pc = 0; pc < n; ++pc) {
        const Instr I = load_instr(M, pc);
        const bool act = pc >= resume;
        if (I.kind == kEnter) {
            COp& O = M->ops[I.idx];
            bool in = ((px >= O.lo[0]) & (O.hi[0] >= px)) | ((py >= O.lo[1]) & (O.hi[1] >= py)) |
                      ((pz >= O.lo[2]) & (O.hi[2] >= pz));
            bool anyIn = (GROUP == 4) ? quad_any(act && in) : (act && in);
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
                float v;
                switch (I.type) {
                case 18: v = lf + rf; break;                       // Blend
                case 19: {                                          // RicciBlend: fast_pow
                    const float base = lf + rf, e = M->ops[I.idx].resY;
                    float den = e * base;
                    den = e - den;
                    den = base + den;
                    v = base * (1.0f / den);
                } break;
                case 14: v = max_ref(lf, rf); break;                // Union
                case 15: v = min_ref(lf, rf); break;                // Intersect
                case 16: v = min_ref(lf, 1.0f - rf); break;         // Dif
                case 17: v = lf * (1.0f - rf); break;               // SmoothDif
                case 22: case 23: case 24: case 25: v = lf; break;  // warps: identity
                default: v = last; break;                           // stale outField
                }
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
                    float wl = 0.0f, wr = 0.0f;
                    bool mix = true;
                    switch (I.type) {
                    case 18: case 19:
                        wl = 2.0f * (0.5f + lf) - 1.0f;
                        wr = 2.0f * (0.5f + rf) - 1.0f;
                        break;
                    case 14: case 15:
                        wl = m01((v - lf) == 0.0f);
                        wr = m01((v - rf) == 0.0f);
                        break;
                    case 16: case 17:
                        wl = m01(lf == v);
                        wr = m01((1.0f - rf) == v);
                        break;
                    case 22: case 23: case 24: case 25:
                        lc0 = cl0; lc1 = cl1; lc2 = cl2;
                        mix = false;
                        break;
                    default:
                        mix = false;
                        break;
                    }
                    if (mix) {
                        lc0 = wl * cl0 + wr * cr0;
                        lc1 = wl * cl1 + wr * cr1;
                        lc2 = wl * cl2 + wr * cr2;
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

__device__ __forceinline__ void mpu_origin(const Params& p, uint32_t m, float o[3]) {
    const uint32_t k = m % p.dims[2];
    const uint32_t j = (m / p.dims[2]) % p.dims[1];
    const uint32_t i = m / (p.dims[2] * p.dims[1]);
    o[0] = p.lo[0] + (float)i * p.side;
    o[1] = p.lo[1] + (float)j * p.side;
    o[2] = p.lo[2] + (float)k * p.side;
}

// ---------------------------------------------------------------------------
// S1: 8 corners per MPU, lanes 0-3 z = lo, lanes 4-7 z = lo + side; (x,y) lanes
// (0,0),(1,0),(0,1),(1,1) (PS_Polygonizer.cpp:488-519).  256 threads = 32 MPUs.
__global__ void __launch_bounds__(256) k_precheck(Params p) {
    extern __shared__ float lds[];
    const int wave = threadIdx.x >> 6;
    float* sl = lds + wave * p.slotsPerLane * 64 + lane_id();
    __shared__ uint32_t waveMask[4];
    const uint32_t local = (blockIdx.x * 256 + threadIdx.x) >> 3;
    const bool valid = local < p.mpuCount;
    const uint32_t m = p.mpuBegin + (valid ? local : 0);
    float o[3];
    mpu_origin(p, m, o);
    const int c = threadIdx.x & 7;
    const float X = (float)(c & 1), Y = (float)((c >> 1) & 1), Z = (float)(c >> 2);
    const float px = X * p.side + o[0];
    const float py = Y * p.side + o[1];
    const float pz = Z * p.side + o[2];
    CullMask cm = make_cull_mask(as_const(p.model), px, py, pz, false);
    float f = walk<4, false>(as_const(p.model), px, py, pz, sl, cm, nullptr);
    uint64_t b = ballot(valid && f > 0.0f);
    if (lane_id() == 0) {
        uint32_t mk = 0;
#pragma unroll
        for (int g = 0; g < 8; ++g) mk |= (((b >> (8 * g)) & 0xffull) != 0ull ? 1u : 0u) << g;
        waveMask[wave] = mk;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        p.passMask[blockIdx.x] = waveMask[0] | (waveMask[1] << 8) | (waveMask[2] << 16) | (waveMask[3] << 24);
    }
}

// Ordered compaction of the S1 survivors (single workgroup of 1024 threads).
__global__ void __launch_bounds__(1024) k_compact(Params p) {
    __shared__ uint32_t part[1024];
    const uint32_t nWords = (p.mpuCount + 31) / 32;
    const uint32_t per = (nWords + 1023) / 1024;
    const uint32_t w0 = threadIdx.x * per;
    uint32_t cnt = 0;
    for (uint32_t w = w0; w < w0 + per && w < nWords; ++w) cnt += __popc(p.passMask[w]);
    part[threadIdx.x] = cnt;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
        uint32_t v = threadIdx.x >= (uint32_t)off ? part[threadIdx.x - off] : 0u;
        __syncthreads();
        part[threadIdx.x] += v;
        __syncthreads();
    }
    uint32_t base = part[threadIdx.x] - cnt;
    for (uint32_t w = w0; w < w0 + per && w < nWords; ++w) {
        uint32_t mk = p.passMask[w];
        while (mk) {
            int b = __ffs(mk) - 1;
            mk &= mk - 1;
            p.passList[base++] = p.mpuBegin + w * 32 + (uint32_t)b;
        }
    }
    if (threadIdx.x == 1023) p.ctr->passCount = part[1023];
}

// ---------------------------------------------------------------------------
// Per-MPU kernel: one wavefront per MPU that passed S1, 4 wavefronts per block.
// LDS per wave: fv[512] f32 | edgeVid[1536] u16 | cfg[344] u8 | vbase[344] u16 |
//               tbase[344] u16 | value slots
constexpr int kLdsFv = 0;
constexpr int kLdsEdge = 2048;
constexpr int kLdsCfg = kLdsEdge + 1536 * 2;
constexpr int kLdsVbase = kLdsCfg + 344;
constexpr int kLdsTbase = kLdsVbase + 344 * 2;
constexpr int kLdsSlots = ((kLdsTbase + 344 * 2) + 15) & ~15;

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    const int l = lane_id();
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t t = __shfl_up(v, o);
        if (l >= o) v += t;
    }
    return v;
}

__global__ void __launch_bounds__(256) k_mpu(Params p) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int wave = threadIdx.x >> 6;
    const int lane = lane_id();
    const uint32_t w = blockIdx.x * 4 + wave;
    const uint32_t passCount = p.ctr->passCount;
    if (w >= passCount) return;
    unsigned char* base = smem + wave * (kLdsSlots + p.slotsPerLane * 64 * 4);
    float* fv = reinterpret_cast<float*>(base + kLdsFv);
    uint16_t* edgeVid = reinterpret_cast<uint16_t*>(base + kLdsEdge);
    uint8_t* cellCfg = base + kLdsCfg;
    uint16_t* cellV = reinterpret_cast<uint16_t*>(base + kLdsVbase);
    uint16_t* cellT = reinterpret_cast<uint16_t*>(base + kLdsTbase);
    float* sl = reinterpret_cast<float*>(base + kLdsSlots) + lane;

    const uint32_t m = __builtin_amdgcn_readfirstlane(p.passList[w]);
    float o[3];
    mpu_origin(p, m, o);
    const float cs = p.cs;

    // S2: fv[x][y][z], lane = y*8 + z, x loops (x-major like the reference cache)
    const int y = lane >> 3, z = lane & 7;
    const float py = o[1] + (float)y * cs;
    const float pz = o[2] + (float)z * cs;
    uint32_t inside = 0;
    for (int x = 0; x < 8; ++x) {
        const float px = o[0] + (float)x * cs;
        CullMask cm = make_cull_mask(as_const(p.model), px, py, pz, p.cull != 0);
        float f = walk<4, false>(as_const(p.model), px, py, pz, sl, cm, nullptr);
        fv[x * 64 + lane] = f;
        inside += __popcll(ballot(f >= 0.5f));
    }
    if (inside == 0 || inside == 512) {
        if (lane == 0) p.counts[w] = make_uint2(0u, 0u);
        return;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();

    // S3 pass 1: configs, owned (new) vertices and triangles per cell
    uint32_t carryV = 0, carryT = 0;
    for (int q = 0; q < 6; ++q) {
        const int c = q * 64 + lane;
        const int i = c / 49, j = (c / 7) % 7, k = c % 7;
        uint32_t cfg = 0;
        if (c < 343) {
#pragma unroll
            for (int cc = 0; cc < 8; ++cc) {
                const int xx = i + ((cc >> 2) & 1), yy = j + ((cc >> 1) & 1), zz = k + (cc & 1);
                cfg |= (fv[xx * 64 + yy * 8 + zz] >= 0.5f ? 1u : 0u) << cc;
            }
        }
        uint32_t nv = 0, nt = 0;
        if (cfg != 0 && cfg != 255) {
            uint32_t seen = 0;
            for (int e = 0; e < 16; ++e) {
                const int ed = c_tri[cfg][e];
                if (ed < 0) break;
                if ((seen >> ed) & 1u) continue;
                seen |= 1u << ed;
                const int c1 = c_corner1[ed], ax = c_axis[ed];
                const int sx = i + ((c1 >> 2) & 1), sy = j + ((c1 >> 1) & 1), sz = k + (c1 & 1);
                const int ox = ax == 0 ? sx : max(sx - 1, 0);
                const int oy = ax == 1 ? sy : max(sy - 1, 0);
                const int oz = ax == 2 ? sz : max(sz - 1, 0);
                nv += (ox == i && oy == j && oz == k) ? 1u : 0u;
            }
            nt = c_ntri[cfg];
        }
        const uint32_t sv = wave_incl_scan(nv);
        const uint32_t st = wave_incl_scan(nt);
        if (c < 343) {
            cellCfg[c] = (uint8_t)cfg;
            cellV[c] = (uint16_t)(carryV + sv - nv);
            cellT[c] = (uint16_t)(carryT + st - nt);
        }
        carryV += __shfl(sv, 63);
        carryT += __shfl(st, 63);
    }
    const uint32_t V = carryV, T = carryT;
    uint32_t qv = 0, qt = 0;
    if (lane == 0) {
        qv = atomicAdd(&p.ctr->vCount, V);
        qt = atomicAdd(&p.ctr->tCount, T);
        p.counts[w] = make_uint2(V, T);
    }
    qv = __shfl(qv, 0);
    qt = __shfl(qt, 0);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();

    // S4 ownership pass 2: vertex ids in discovery order, vertex records
    for (int q = 0; q < 6; ++q) {
        const int c = q * 64 + lane;
        if (c >= 343) break;
        const uint32_t cfg = cellCfg[c];
        if (cfg == 0 || cfg == 255) continue;
        const int i = c / 49, j = (c / 7) % 7, k = c % 7;
        uint32_t vid = cellV[c];
        uint32_t seen = 0;
        for (int e = 0; e < 16; ++e) {
            const int ed = c_tri[cfg][e];
            if (ed < 0) break;
            if ((seen >> ed) & 1u) continue;
            seen |= 1u << ed;
            const int c1 = c_corner1[ed], ax = c_axis[ed];
            const int sx = i + ((c1 >> 2) & 1), sy = j + ((c1 >> 1) & 1), sz = k + (c1 & 1);
            const int ox = ax == 0 ? sx : max(sx - 1, 0);
            const int oy = ax == 1 ? sy : max(sy - 1, 0);
            const int oz = ax == 2 ? sz : max(sz - 1, 0);
            if (ox == i && oy == j && oz == k) {
                edgeVid[((sx * 8 + sy) * 8 + sz) * 3 + ax] = (uint16_t)vid;
                const uint32_t key = (uint32_t)sx | ((uint32_t)sy << 3) | ((uint32_t)sz << 6) | ((uint32_t)ax << 9);
                const uint32_t g = qv + vid;
                if (g < p.vcap) p.vq[g] = VertexRec{w, vid | (key << 16)};
                ++vid;
            }
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();

    // S6 pass 3: triangles in table order
    for (int q = 0; q < 6; ++q) {
        const int c = q * 64 + lane;
        if (c >= 343) break;
        const uint32_t cfg = cellCfg[c];
        if (cfg == 0 || cfg == 255) continue;
        const int i = c / 49, j = (c / 7) % 7, k = c % 7;
        const uint32_t tb = cellT[c];
        const uint32_t nt = c_ntri[cfg];
        for (uint32_t t = 0; t < nt; ++t) {
            uint32_t v[3];
#pragma unroll
            for (int s = 0; s < 3; ++s) {
                const int ed = c_tri[cfg][t * 3 + s];
                const int c1 = c_corner1[ed], ax = c_axis[ed];
                const int sx = i + ((c1 >> 2) & 1), sy = j + ((c1 >> 1) & 1), sz = k + (c1 & 1);
                v[s] = edgeVid[((sx * 8 + sy) * 8 + sz) * 3 + ax];
            }
            const uint32_t g = qt + tb + t;
            if (g < p.tcap) p.tq[g] = TriRec{w, tb + t, v[0] | (v[1] << 16), v[2]};
        }
    }
}

// Exclusive scan of per-MPU (V,T) into mesh offsets (single workgroup).
__global__ void __launch_bounds__(1024) k_scan(Params p) {
    __shared__ uint32_t sv[1024], st[1024];
    __shared__ uint32_t surf[1024];
    const uint32_t n = p.ctr->passCount;
    const uint32_t per = (n + 1023) / 1024;
    const uint32_t s0 = threadIdx.x * per;
    uint32_t a = 0, b = 0, sc = 0;
    int firstOv = 0x7fffffff;
    for (uint32_t w = s0; w < s0 + per && w < n; ++w) {
        const uint2 c = p.counts[w];
        a += c.x;
        b += c.y;
        sc += c.y > 0 ? 1u : 0u;
        if ((c.x > 512u || c.y > 512u) && firstOv == 0x7fffffff) firstOv = (int)p.passList[w];
    }
    if (firstOv != 0x7fffffff) atomicMin(&p.ctr->firstOverflow, firstOv);
    sv[threadIdx.x] = a;
    st[threadIdx.x] = b;
    surf[threadIdx.x] = sc;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
        uint32_t x = threadIdx.x >= (uint32_t)off ? sv[threadIdx.x - off] : 0u;
        uint32_t y = threadIdx.x >= (uint32_t)off ? st[threadIdx.x - off] : 0u;
        uint32_t z = threadIdx.x >= (uint32_t)off ? surf[threadIdx.x - off] : 0u;
        __syncthreads();
        sv[threadIdx.x] += x;
        st[threadIdx.x] += y;
        surf[threadIdx.x] += z;
        __syncthreads();
    }
    uint32_t va = sv[threadIdx.x] - a, ta = st[threadIdx.x] - b;
    for (uint32_t w = s0; w < s0 + per && w < n; ++w) {
        const uint2 c = p.counts[w];
        p.voff[w] = va;
        p.toff[w] = ta;
        va += c.x;
        ta += c.y;
    }
    if (threadIdx.x == 1023) {
        p.voff[n] = sv[1023];
        p.toff[n] = st[1023];
        p.ctr->surfaceCount = surf[1023];
    }
}

// ---------------------------------------------------------------------------
// Vertices: batches of 16 vertices per wavefront iteration, one quad per vertex.
// Phase A (quad pruning): the 4 edge samples e1 + (e2-e1)*(l/3), l = 0..3 (:733-741)
// Phase B (per-lane pruning): lane 0 = p with colour, lanes 1..3 = p + delta*e_a.
__global__ void __launch_bounds__(256) k_vertex(Params p) {
    extern __shared__ __attribute__((aligned(16))) float vlds[];
    const int wave = threadIdx.x >> 6;
    const int lane = lane_id();
    float* sl = vlds + wave * (p.slotsPerLane * 4 * 64) + lane;
    const uint32_t nV = min(p.ctr->vCount, p.vcap);
    const int j = lane & 3;
    const float third = 1.0f / 3.0f;
    const float r = (float)j * third;
    const float delta = 0.001f;
    const float inv = -1.0f / delta;
    for (;;) {
        uint32_t batch = 0;
        if (lane == 0) batch = atomicAdd(&p.dequeue[0], 1u);
        batch = __shfl(batch, 0);
        const uint32_t v0 = batch * 16;
        if (v0 >= nV) break;
        uint32_t rec = v0 + (lane >> 2);
        const bool valid = rec < nV;
        if (!valid) rec = v0;
        const VertexRec R = p.vq[rec];
        const uint32_t m = p.passList[R.w];
        float o[3];
        mpu_origin(p, m, o);
        const uint32_t key = R.vidKey >> 16;
        const int sx = key & 7, sy = (key >> 3) & 7, sz = (key >> 6) & 7, ax = (key >> 9) & 3;
        const float cs = p.cs;
        float e1[3] = {o[0] + cs * (float)sx, o[1] + cs * (float)sy, o[2] + cs * (float)sz};
        float e2[3] = {e1[0], e1[1], e1[2]};
        e2[ax] = e1[ax] + cs;
        const float dX = e2[0] - e1[0], dY = e2[1] - e1[1], dZ = e2[2] - e1[2];
        const float qx = e1[0] + dX * r, qy = e1[1] + dY * r, qz = e1[2] + dZ * r;
        CullMask cm = make_cull_mask(as_const(p.model), qx, qy, qz, p.cull != 0);
        const float f = walk<4, false>(as_const(p.model), qx, qy, qz, sl, cm, nullptr);
        // gather the quad's 4 samples
        const int qb = lane & ~3;
        float fs[4], xs[4], ys[4], zs[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            fs[s] = __shfl(f, qb + s);
            const float rs = (float)s * third;
            xs[s] = e1[0] + dX * rs;
            ys[s] = e1[1] + dY * rs;
            zs[s] = e1[2] + dZ * rs;
        }
        const bool st0 = fs[0] >= 0.5f;
        int iv = 3;
        if ((fs[1] >= 0.5f) != st0) iv = 1;
        else if ((fs[2] >= 0.5f) != st0) iv = 2;
        float ax_[3], bx_[3], fa, fb;
        // iv in 1..3: select samples iv-1, iv
        fa = iv == 1 ? fs[0] : (iv == 2 ? fs[1] : fs[2]);
        fb = iv == 1 ? fs[1] : (iv == 2 ? fs[2] : fs[3]);
        ax_[0] = iv == 1 ? xs[0] : (iv == 2 ? xs[1] : xs[2]);
        ax_[1] = iv == 1 ? ys[0] : (iv == 2 ? ys[1] : ys[2]);
        ax_[2] = iv == 1 ? zs[0] : (iv == 2 ? zs[1] : zs[2]);
        bx_[0] = iv == 1 ? xs[1] : (iv == 2 ? xs[2] : xs[3]);
        bx_[1] = iv == 1 ? ys[1] : (iv == 2 ? ys[2] : ys[3]);
        bx_[2] = iv == 1 ? zs[1] : (iv == 2 ? zs[2] : zs[3]);
        const float scale = (0.5f - fa) / (fb - fa);
        const float P0 = ax_[0] + scale * (bx_[0] - ax_[0]);
        const float P1 = ax_[1] + scale * (bx_[1] - ax_[1]);
        const float P2 = ax_[2] + scale * (bx_[2] - ax_[2]);
        // Phase B
        float qx2 = j == 1 ? P0 + delta : P0;
        float qy2 = j == 2 ? P1 + delta : P1;
        float qz2 = j == 3 ? P2 + delta : P2;
        CullMask cm2 = make_cull_mask(as_const(p.model), qx2, qy2, qz2, p.cull != 0);
        float colr[3];
        const float g = walk<1, true>(as_const(p.model), qx2, qy2, qz2, sl, cm2, colr);
        const float vtx = __shfl(g, qb);
        const float gx = __shfl(g, qb + 1), gy = __shfl(g, qb + 2), gz = __shfl(g, qb + 3);
        float nx = (gx - vtx) * inv, ny = (gy - vtx) * inv, nz = (gz - vtx) * inv;
        const float im = 1.0f / __fsqrt_rn((nx * nx + ny * ny) + nz * nz);
        nx = nx * im;
        ny = ny * im;
        nz = nz * im;
        if (valid && j == 0) {
            const uint32_t gi = p.voff[R.w] + (R.vidKey & 0xffffu);
            p.pos[gi * 3 + 0] = P0; p.pos[gi * 3 + 1] = P1; p.pos[gi * 3 + 2] = P2;
            p.nrm[gi * 3 + 0] = nx; p.nrm[gi * 3 + 1] = ny; p.nrm[gi * 3 + 2] = nz;
            p.col[gi * 3 + 0] = colr[0]; p.col[gi * 3 + 1] = colr[1]; p.col[gi * 3 + 2] = colr[2];
        }
    }
}

__global__ void __launch_bounds__(256) k_tris(Params p) {
    const uint32_t nT = min(p.ctr->tCount, p.tcap);
    for (uint32_t t = blockIdx.x * 256 + threadIdx.x; t < nT; t += gridDim.x * 256) {
        const TriRec R = p.tq[t];
        const uint32_t g = p.toff[R.w] + R.tlocal;
        const uint32_t b = p.voff[R.w];
        p.tris[g * 3 + 0] = b + (R.v01 & 0xffffu);
        p.tris[g * 3 + 1] = b + (R.v01 >> 16);
        p.tris[g * 3 + 2] = b + R.v2;
    }
}

// Single-point field probe for tests: n points, grouped in quads (GROUP 4) or not.
__global__ void __launch_bounds__(256) k_probe(Params p, const float* __restrict__ xyz, float* __restrict__ out,
                                               float* __restrict__ colOut, uint32_t n, int mode) {
    extern __shared__ __attribute__((aligned(16))) float plds[];
    const int wave = threadIdx.x >> 6;
    float* sl = plds + wave * (p.slotsPerLane * 4 * 64) + lane_id();
    uint32_t i = blockIdx.x * 256 + threadIdx.x;
    const bool valid = i < n;
    if (!valid) i = (n ? n - 1 : 0);
    const float x = xyz[3 * i], y = xyz[3 * i + 1], z = xyz[3 * i + 2];
    CullMask cm = make_cull_mask(as_const(p.model), x, y, z, p.cull != 0);
    float c[3] = {0.0f, 0.0f, 0.0f};
    float f;
    if (mode == 0) f = walk<4, false>(as_const(p.model), x, y, z, sl, cm, nullptr);
    else if (mode == 1) f = walk<1, false>(as_const(p.model), x, y, z, sl, cm, nullptr);
    else f = walk<1, true>(as_const(p.model), x, y, z, sl, cm, c);
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

// ---------------------------------------------------------------------------
// Host-side launch helpers (called from psgpu_host.cpp).
namespace psgpu {

hipError_t upload_tables(const int8_t tri[256][16], const uint8_t ntri[256], const uint8_t corner1[12],
                         const uint8_t axis[12]) {
    hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(c_tri), tri, 256 * 16);
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(c_ntri), ntri, 256);
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(c_corner1), corner1, 12);
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(c_axis), axis, 12);
    return e;
}

size_t mpu_lds_bytes(uint32_t slots) { return 4 * (kLdsSlots + (size_t)slots * 64 * 4); }
size_t walk_lds_bytes(uint32_t slots) { return 4 * ((size_t)slots * 4 * 64 * 4); }
size_t precheck_lds_bytes(uint32_t slots) { return 4 * ((size_t)slots * 64 * 4); }

hipError_t launch_precheck(const Params& p, hipStream_t s) {
    const uint32_t blocks = (p.mpuCount + 31) / 32;
    hipLaunchKernelGGL(k_precheck, dim3(blocks), dim3(256), precheck_lds_bytes(p.slotsPerLane), s, p);
    return hipGetLastError();
}
hipError_t launch_compact(const Params& p, hipStream_t s) {
    hipLaunchKernelGGL(k_compact, dim3(1), dim3(1024), 0, s, p);
    return hipGetLastError();
}
hipError_t launch_mpu(const Params& p, hipStream_t s) {
    const uint32_t blocks = (p.mpuCount + 3) / 4;
    hipLaunchKernelGGL(k_mpu, dim3(blocks), dim3(256), mpu_lds_bytes(p.slotsPerLane), s, p);
    return hipGetLastError();
}
hipError_t launch_scan(const Params& p, hipStream_t s) {
    hipLaunchKernelGGL(k_scan, dim3(1), dim3(1024), 0, s, p);
    return hipGetLastError();
}
hipError_t launch_vertex(const Params& p, hipStream_t s, uint32_t blocks) {
    hipLaunchKernelGGL(k_vertex, dim3(blocks), dim3(256), walk_lds_bytes(p.slotsPerLane), s, p);
    return hipGetLastError();
}
hipError_t launch_tris(const Params& p, hipStream_t s, uint32_t blocks) {
    hipLaunchKernelGGL(k_tris, dim3(blocks), dim3(256), 0, s, p);
    return hipGetLastError();
}
hipError_t launch_probe(const Params& p, hipStream_t s, const float* xyz, float* out, float* col, uint32_t n,
                        int mode) {
    const uint32_t blocks = (n + 255) / 256;
    hipLaunchKernelGGL(k_probe, dim3(blocks ? blocks : 1), dim3(256), walk_lds_bytes(p.slotsPerLane), s, p, xyz,
                       out, col, n, mode);
    return hipGetLastError();
}

}  // namespace psgpu

/*
 * psoracle.c — TEST INFRASTRUCTURE ONLY.  CPU restatement of Parsip's PS_SimdPoly
 * polygonizer (Parsip100/PS_SimdPoly/include/PS_Polygonizer.cpp) used as the parity
 * checker for the HIP path and as the `cpu_baseline` leg of bench.py.  Nothing in
 * the product (parsip_amd/, include/) links, loads or calls this file.
 *
 * PARITY STATUS: the reference path is UNBUILDABLE in this image (PS_Polygonizer.h
 * includes the legacy TBB headers tbb/blocked_range.h, tbb/parallel_for.h,
 * tbb/enumerable_thread_specific.h, tbb/task_scheduler_observer.h and uses
 * tbb_thread; none are installed, and stand-ins are not permitted), and the
 * reference ships no tests, fixtures or golden vectors for this path.  The
 * restatement is pinned (tests/test_oracle.py) by (1) the outputs the compiled
 * reference produced in the survey (MPU / S1 / vertex /
 * triangle counts and per-MPU maxima for C1, C2 and C3 on std::mt19937(42) inputs,
 * tests/golden/reference_probe.json), which it reproduces exactly, and (2) the
 * marching-cubes table digest of _CellConfigTable.h (tests/golden/tritable.json).
 * Bits of positions / normals / colours beyond those counts were never recorded
 * from the reference: for them the restatement is "parity unpinned".
 *
 * Semantics are restated literally, 4 SSE lanes at a time, so the op-box pruning
 * that the reference decides per 4-lane group (PS_Polygonizer.cpp:1228-1252) is
 * reproduced.  Two defined deviations from the reference (documented in DESIGN.md):
 *   1. arrPrimFields / arrOpFields / arrOpColor* start zeroed.  The reference
 *      leaves them uninitialised and reads them for pruned subtrees in
 *      fieldValueAndColor (PS_Polygonizer.cpp:1194-1195, 1385-1400, 1451, 1466);
 *      zero matches the reference built with -ftrivial-auto-var-init=zero.
 *   2. _mm_rsqrt_ps / _mm_rcp_ps (PS_SIMDVecN.h:411, 122-128, 435-442) are
 *      replaced by correctly rounded 1/sqrt(x) and 1/x, because the SSE
 *      approximations are CPU-vendor specific.  Build with -DPSOR_SSE_APPROX to get
 *      the reference's approximate instructions instead.
 * Build flags must keep -ffp-contract=off and no fast-math.
 */
#include <immintrin.h>
#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/parsip_gpu.h"
#include "psoracle.h"

typedef __m128 V4;

/* Work counters (lane-evaluations, 4 per SIMD call) of the reference algorithm as
 * executed, per phase: 0 S1, 1 S2, 2 S4 root samples, 3 S5 value/normal samples,
 * 4 fieldValueAndColor.  Slots: [type] primitive evaluations by skeletType (0..15),
 * [16] primitive matrices applied, [17] depth>3 op-box tests, [18] colour op steps,
 * [32 + opType] op evaluations by type.  For the algorithmic-work figure of bench.py
 * (tests/golden/make_workload_ops.py); they do not affect any result. */
#define PSOR_NCNT 64
static __thread int t_phase;
static __thread uint64_t t_cnt[5][PSOR_NCNT];
static uint64_t g_cnt[5][PSOR_NCNT];
static pthread_mutex_t g_cnt_mu = PTHREAD_MUTEX_INITIALIZER;
#ifdef PSOR_COUNT
#define CNT(slot) (t_cnt[t_phase][(slot)] += 4)
#else
#define CNT(slot) ((void)0)
#endif

#define V(a) _mm_set1_ps(a)
#define ADD _mm_add_ps
#define SUB _mm_sub_ps
#define MUL _mm_mul_ps
#define DIV _mm_div_ps
/* _mm_max_ps(a,b) == a > b ? a : b, _mm_min_ps(a,b) == a < b ? a : b (NaN/-0 exact) */
#define VMAX _mm_max_ps
#define VMIN _mm_min_ps
#define ONE01(m) _mm_and_ps((m), V(1.0f)) /* SimdAnd(mask, one) -> {0, 1.0f} */

static inline V4 v_rsqrt(V4 x) {
#ifdef PSOR_SSE_APPROX
    return _mm_rsqrt_ps(x);
#else
    return DIV(V(1.0f), _mm_sqrt_ps(x));
#endif
}
static inline V4 v_rcp(V4 x) {
#ifdef PSOR_SSE_APPROX
    return _mm_rcp_ps(x);
#else
    return DIV(V(1.0f), x);
#endif
}
static inline float lane(V4 v, int i) {
    float t[4];
    _mm_storeu_ps(t, v);
    return t[i];
}

/* ------------------------------------------------------------------------- */
/* Marching cubes table: Bloomenthal, "An Implicit Surface Polygonizer",       */
/* Graphics Gems IV (1994), makecubetable(); polygons kept in discovery order, */
/* each polygon's edge list head-inserted, then fan-triangulated about its last */
/* edge.  Corner numbering bit2 = x, bit1 = y, bit0 = z (_CellConfigTable.h:30-49).*/
enum { LB, LT, LN, LF, RB, RT, RN, RF, BN, BF, TN, TF };
enum { FL, FR, FB, FT, FN, FF };
static const int k_corner1[12] = {0, 2, 0, 1, 4, 6, 4, 5, 0, 1, 2, 3};
static const int k_corner2[12] = {1, 3, 2, 3, 5, 7, 6, 7, 4, 5, 6, 7};
static const int k_axis[12] = {2, 2, 1, 1, 2, 2, 1, 1, 0, 0, 0, 0};
static const int k_leftface[12] = {FB, FL, FL, FF, FR, FT, FN, FR, FN, FB, FT, FF};
static const int k_rightface[12] = {FL, FT, FN, FL, FB, FR, FR, FF, FB, FF, FN, FT};

static int next_cw_edge(int e, int f) {
    switch (e) {
    case LB: return f == FL ? LF : BN;
    case LT: return f == FL ? LN : TF;
    case LN: return f == FL ? LB : TN;
    case LF: return f == FL ? LT : BF;
    case RB: return f == FR ? RN : BF;
    case RT: return f == FR ? RF : TN;
    case RN: return f == FR ? RT : BN;
    case RF: return f == FR ? RB : TF;
    case BN: return f == FB ? RB : LN;
    case BF: return f == FB ? LB : RF;
    case TN: return f == FT ? LT : RN;
    default: return f == FT ? RT : LF; /* TF */
    }
}

static int g_tri[256][16];
static pthread_once_t g_tri_once = PTHREAD_ONCE_INIT;

static void build_tritable(void) {
    for (int cfg = 0; cfg < 256; ++cfg) {
        int done[12] = {0}, n = 0;
        for (int i = 0; i < 16; ++i) g_tri[cfg][i] = -1;
        for (int e = 0; e < 12; ++e) {
            int in1 = (cfg >> k_corner1[e]) & 1, in2 = (cfg >> k_corner2[e]) & 1;
            if (done[e] || in1 == in2) continue;
            int poly[12], np = 0, edge = e;
            int face = in1 ? k_rightface[e] : k_leftface[e];
            for (;;) {
                edge = next_cw_edge(edge, face);
                done[edge] = 1;
                if (((cfg >> k_corner1[edge]) & 1) != ((cfg >> k_corner2[edge]) & 1)) {
                    memmove(poly + 1, poly, (size_t)np * sizeof(int));
                    poly[0] = edge;
                    ++np;
                    if (edge == e) break;
                    face = (face == k_leftface[edge]) ? k_rightface[edge] : k_leftface[edge];
                }
            }
            for (int t = np - 3; t >= 0; --t) {
                g_tri[cfg][n++] = poly[t];
                g_tri[cfg][n++] = poly[t + 1];
                g_tri[cfg][n++] = poly[np - 1];
            }
        }
    }
}

void psor_tritable(int32_t out[256 * 16]) {
    pthread_once(&g_tri_once, build_tritable);
    memcpy(out, g_tri, sizeof(g_tri));
}

/* ------------------------------------------------------------------------- */
/* computePrimitiveField, PS_Polygonizer.cpp:934-1179 + Wyvill h:397-407      */
static V4 prim_field(const PsModelRef* m, uint32_t idx, V4 pX, V4 pY, V4 pZ) {
    const PsSoaBlobPrims* P = m->prims;
    V4 d2 = _mm_setzero_ps();
    V4 x = pX, y = pY, z = pZ;
    uint32_t im = P->idxMatrix[idx];
    CNT(P->skeletType[idx] & 15);
    if (im != 0) CNT(16);
    if (im != 0) { /* :948-970, rows ((m0*x + m1*y) + m2*z) + m3 */
        const float* M = &m->mats->matrix[im * PSGPU_PRIM_MATRIX_STRIDE];
        x = ADD(ADD(ADD(MUL(V(M[0]), pX), MUL(V(M[1]), pY)), MUL(V(M[2]), pZ)), V(M[3]));
        y = ADD(ADD(ADD(MUL(V(M[4]), pX), MUL(V(M[5]), pY)), MUL(V(M[6]), pZ)), V(M[7]));
        z = ADD(ADD(ADD(MUL(V(M[8]), pX), MUL(V(M[9]), pY)), MUL(V(M[10]), pZ)), V(M[11]));
    }
    switch (P->skeletType[idx]) {
    case PSGPU_PRIM_POINT: { /* :975-983 */
        V4 dx = SUB(V(P->posX[idx]), x), dy = SUB(V(P->posY[idx]), y), dz = SUB(V(P->posZ[idx]), z);
        d2 = ADD(ADD(MUL(dx, dx), MUL(dy, dy)), MUL(dz, dz));
    } break;
    case PSGPU_PRIM_LINE: { /* :984-1011, projection not clamped */
        V4 l0x = V(P->posX[idx]), l0y = V(P->posY[idx]), l0z = V(P->posZ[idx]);
        V4 ldx = SUB(V(P->dirX[idx]), l0x), ldy = SUB(V(P->dirY[idx]), l0y), ldz = SUB(V(P->dirZ[idx]), l0z);
        V4 ldd = ADD(ADD(MUL(ldx, ldx), MUL(ldy, ldy)), MUL(ldz, ldz));
        V4 dx = SUB(x, l0x), dy = SUB(y, l0y), dz = SUB(z, l0z);
        V4 t = ADD(ADD(MUL(dx, ldx), MUL(dy, ldy)), MUL(dz, ldz));
        t = DIV(t, ldd);
        dx = SUB(x, ADD(l0x, MUL(t, ldx)));
        dy = SUB(y, ADD(l0y, MUL(t, ldy)));
        dz = SUB(z, ADD(l0z, MUL(t, ldz)));
        d2 = ADD(ADD(MUL(dx, dx), MUL(dy, dy)), MUL(dz, dz));
    } break;
    case PSGPU_PRIM_CYLINDER: { /* :1012-1039 */
        V4 px = SUB(x, V(P->posX[idx])), py = SUB(y, V(P->posY[idx])), pz = SUB(z, V(P->posZ[idx]));
        V4 ax = V(P->dirX[idx]), ay = V(P->dirY[idx]), az = V(P->dirZ[idx]);
        V4 radius = V(P->resX[idx]), height = V(P->resY[idx]);
        V4 zero = _mm_setzero_ps(), one = V(1.0f);
        V4 yy = ADD(ADD(MUL(px, ax), MUL(py, ay)), MUL(pz, az));
        V4 rr = SUB(ADD(ADD(MUL(px, px), MUL(py, py)), MUL(pz, pz)), MUL(yy, yy));
        V4 xx = VMAX(zero, SUB(_mm_sqrt_ps(rr), radius));
        V4 mask = ONE01(_mm_cmpgt_ps(yy, zero));
        yy = ADD(MUL(mask, VMAX(zero, SUB(yy, height))), MUL(SUB(one, mask), yy));
        d2 = ADD(MUL(xx, xx), MUL(yy, yy));
    } break;
    case PSGPU_PRIM_TRIANGLE: /* :1040-1057, distance stub */
        d2 = V(FLT_MAX);
        break;
    case PSGPU_PRIM_CUBE: { /* :1059-1097 */
        V4 side = V(P->resX[idx]), mside = V(-1.0f * P->resX[idx]);
        V4 dif[3] = {SUB(x, V(P->posX[idx])), SUB(y, V(P->posY[idx])), SUB(z, V(P->posZ[idx]))};
        for (int a = 0; a < 3; ++a) {
            V4 mm = ONE01(_mm_cmpgt_ps(mside, dif[a]));
            V4 mp = ONE01(_mm_cmpgt_ps(dif[a], side));
            V4 dl = ADD(MUL(ADD(dif[a], side), mm), MUL(SUB(dif[a], side), mp));
            d2 = (a == 0) ? MUL(dl, dl) : ADD(d2, MUL(dl, dl));
        }
    } break;
    case PSGPU_PRIM_DISC: { /* :1099-1132 */
        V4 dX = SUB(x, V(P->posX[idx])), dY = SUB(y, V(P->posY[idx])), dZ = SUB(z, V(P->posZ[idx]));
        V4 nX = V(P->dirX[idx]), nY = V(P->dirY[idx]), nZ = V(P->dirZ[idx]);
        V4 radius = V(P->resX[idx]), one = V(1.0f);
        V4 dot = ADD(ADD(MUL(nX, dX), MUL(nY, dY)), MUL(nZ, dZ));
        V4 rX = SUB(dX, MUL(nX, dot)), rY = SUB(dY, MUL(nY, dot)), rZ = SUB(dZ, MUL(nZ, dot));
        dot = ADD(ADD(MUL(rX, rX), MUL(rY, rY)), MUL(rZ, rZ));
        V4 rs = v_rsqrt(dot);
        rX = MUL(rX, rs); rY = MUL(rY, rs); rZ = MUL(rZ, rs);
        nX = SUB(MUL(radius, rX), dX); nY = SUB(MUL(radius, rY), dY); nZ = SUB(MUL(radius, rZ), dZ);
        V4 mask = ONE01(_mm_cmpge_ps(MUL(radius, radius), dot));
        d2 = ADD(MUL(mask, SUB(ADD(ADD(MUL(dX, dX), MUL(dY, dY)), MUL(dZ, dZ)), dot)),
                 MUL(SUB(one, mask), ADD(ADD(MUL(nX, nX), MUL(nY, nY)), MUL(nZ, nZ))));
    } break;
    case PSGPU_PRIM_RING: { /* :1134-1173 */
        V4 dX = SUB(x, V(P->posX[idx])), dY = SUB(y, V(P->posY[idx])), dZ = SUB(z, V(P->posZ[idx]));
        V4 nX = V(P->dirX[idx]), nY = V(P->dirY[idx]), nZ = V(P->dirZ[idx]);
        V4 radius = V(P->resX[idx]), one = V(1.0f), zero = _mm_setzero_ps();
        V4 dot = ADD(ADD(MUL(nX, dX), MUL(nY, dY)), MUL(nZ, dZ));
        V4 rX = SUB(dX, MUL(nX, dot)), rY = SUB(dY, MUL(nY, dot)), rZ = SUB(dZ, MUL(nZ, dot));
        dot = ADD(ADD(MUL(rX, rX), MUL(rY, rY)), MUL(rZ, rZ));
        V4 mask = ONE01(_mm_cmpeq_ps(dot, zero));
        dot = v_rsqrt(dot);
        rX = MUL(rX, dot); rY = MUL(rY, dot); rZ = MUL(rZ, dot);
        nX = SUB(MUL(radius, rX), dX); nY = SUB(MUL(radius, rY), dY); nZ = SUB(MUL(radius, rZ), dZ);
        d2 = ADD(MUL(mask, ADD(ADD(ADD(MUL(radius, radius), MUL(dX, dX)), MUL(dY, dY)), MUL(dZ, dZ))),
                 MUL(SUB(one, mask), ADD(ADD(MUL(nX, nX), MUL(nY, nY)), MUL(nZ, nZ))));
    } break;
    default: /* no case: dist2 stays zero, field 1 (:937-939) */
        break;
    }
    V4 t = SUB(V(1.0f), d2);
    V4 f = MUL(MUL(t, t), t);
    return VMAX(_mm_setzero_ps(), f);
}

float psor_prim_field1(const PsModelRef* m, uint32_t idx, float x, float y, float z) {
    return lane(prim_field(m, idx, V(x), V(y), V(z)), 0);
}

/* ------------------------------------------------------------------------- */
/* FieldComputer::fieldValue, PS_Polygonizer.cpp:1184-1376.  primF/opF are    */
/* 128*4-float arrays that the caller zeroes (deviation 1 above).             */
#define STACK_CAP 1024
static V4 field_value(const PsModelRef* m, V4 pX, V4 pY, V4 pZ, float* primF, float* opF) {
    const PsSoaBlobOps* O = m->ops;
    V4 out = _mm_setzero_ps();
    if (O->ctOps > 0) {
        uint8_t computed[256];
        memset(computed, 0, sizeof(computed));
        uint32_t sid[STACK_CAP], sdepth[STACK_CAP];
        int top = 0;
        sid[0] = 0;
        sdepth[0] = 0;
        while (top >= 0) {
            uint32_t op = sid[top], depth = sdepth[top];
            uint32_t L = O->opLeftChild[op], R = O->opRightChild[op];
            uint32_t kind = O->opChildKind[op];
            int lop = (kind & 2) >> 1, rop = kind & 1;
            if (depth > 3 && !computed[op]) CNT(17);
            if (depth > 3) { /* :1228-1252, OR of the three axis slabs, per 4 lanes */
                V4 in = _mm_and_ps(_mm_cmpge_ps(pX, V(O->vBoxLoX[op])), _mm_cmpge_ps(V(O->vBoxHiX[op]), pX));
                in = _mm_or_ps(in, _mm_and_ps(_mm_cmpge_ps(pY, V(O->vBoxLoY[op])), _mm_cmpge_ps(V(O->vBoxHiY[op]), pY)));
                in = _mm_or_ps(in, _mm_and_ps(_mm_cmpge_ps(pZ, V(O->vBoxLoZ[op])), _mm_cmpge_ps(V(O->vBoxHiZ[op]), pZ)));
                if (_mm_movemask_ps(in) == 0) {
                    --top;
                    out = _mm_setzero_ps();
                    _mm_storeu_ps(&opF[op * 4], out);
                    computed[op] = 1;
                    continue;
                }
            }
            int ready = !((lop && !computed[L]) || (rop && !computed[R]));
            if (ready) {
                --top;
                V4 lf, rf;
                if (lop) lf = _mm_loadu_ps(&opF[L * 4]);
                else { lf = prim_field(m, L, pX, pY, pZ); _mm_storeu_ps(&primF[L * 4], lf); }
                if (rop) rf = _mm_loadu_ps(&opF[R * 4]);
                else { rf = prim_field(m, R, pX, pY, pZ); _mm_storeu_ps(&primF[R * 4], rf); }
                CNT(32 + (O->opType[op] & 31));
                switch (O->opType[op]) { /* :1282-1338 */
                case PSGPU_OP_BLEND: out = ADD(lf, rf); break;
                case PSGPU_OP_RICCIBLEND: { /* fast_pow, PS_SIMDVecN.h:122-128 */
                    V4 base = ADD(lf, rf), e = V(O->resY[op]);
                    V4 den = MUL(e, base);
                    den = SUB(e, den);
                    den = ADD(base, den);
                    out = MUL(base, v_rcp(den));
                } break;
                case PSGPU_OP_UNION: out = VMAX(lf, rf); break;
                case PSGPU_OP_INTERSECT: out = VMIN(lf, rf); break;
                case PSGPU_OP_DIF: out = VMIN(lf, SUB(V(1.0f), rf)); break;
                case PSGPU_OP_SMOOTHDIF: out = MUL(lf, SUB(V(1.0f), rf)); break;
                case PSGPU_OP_WARPBEND: case PSGPU_OP_WARPTWIST:
                case PSGPU_OP_WARPTAPER: case PSGPU_OP_WARPSHEAR: out = lf; break;
                default: break; /* no case: previous op's field is kept */
                }
                computed[op] = 1;
                _mm_storeu_ps(&opF[op * 4], out);
            } else {
                if (lop && !computed[L] && top + 1 < STACK_CAP) { ++top; sid[top] = L; sdepth[top] = depth + 1; }
                if (rop && !computed[R] && top + 1 < STACK_CAP) { ++top; sid[top] = R; sdepth[top] = depth + 1; }
            }
        }
    } else { /* :1356-1368 */
        for (uint32_t i = 0; i < m->prims->ctPrims; ++i) {
            V4 f = prim_field(m, i, pX, pY, pZ);
            out = ADD(out, f);
            _mm_storeu_ps(&primF[i * 4], f);
        }
    }
    return out;
}

static V4 field_only(const PsModelRef* m, V4 x, V4 y, V4 z) {
    float primF[512], opF[512];
    memset(primF, 0, sizeof(primF));
    memset(opF, 0, sizeof(opF));
    return field_value(m, x, y, z, primF, opF);
}

/* FieldComputer::fieldValueAndColor, PS_Polygonizer.cpp:1378-1551 */
static V4 field_and_color(const PsModelRef* m, V4 pX, V4 pY, V4 pZ, V4* cX, V4* cY, V4* cZ) {
    const PsSoaBlobOps* O = m->ops;
    const PsSoaBlobPrims* P = m->prims;
    float primF[512], opF[512];
    memset(primF, 0, sizeof(primF));
    memset(opF, 0, sizeof(opF));
    V4 ox = _mm_setzero_ps(), oy = ox, oz = ox;
    V4 field = field_value(m, pX, pY, pZ, primF, opF);
    if (O->ctOps > 0) {
        float colX[512], colY[512], colZ[512];
        memset(colX, 0, sizeof(colX));
        memset(colY, 0, sizeof(colY));
        memset(colZ, 0, sizeof(colZ));
        uint8_t done[256];
        memset(done, 0, sizeof(done));
        uint32_t sid[STACK_CAP];
        int top = 0;
        sid[0] = 0;
        while (top >= 0) {
            uint32_t op = sid[top];
            uint32_t L = O->opLeftChild[op], R = O->opRightChild[op];
            int lop = (O->opChildKind[op] & 2) >> 1, rop = O->opChildKind[op] & 1;
            int ready = !((lop && !done[L]) || (rop && !done[R]));
            if (ready) {
                --top;
                CNT(18);
                V4 cur = _mm_loadu_ps(&opF[op * 4]);
                V4 lf, rf, lcx, lcy, lcz, rcx, rcy, rcz;
                if (lop) { lf = _mm_loadu_ps(&opF[L * 4]); lcx = V(colX[L * 4]); lcy = V(colY[L * 4]); lcz = V(colZ[L * 4]); }
                else { lf = _mm_loadu_ps(&primF[L * 4]); lcx = V(P->colorX[L]); lcy = V(P->colorY[L]); lcz = V(P->colorZ[L]); }
                if (rop) { rf = _mm_loadu_ps(&opF[R * 4]); rcx = V(colX[R * 4]); rcy = V(colY[R * 4]); rcz = V(colZ[R * 4]); }
                else { rf = _mm_loadu_ps(&primF[R * 4]); rcx = V(P->colorX[R]); rcy = V(P->colorY[R]); rcz = V(P->colorZ[R]); }
                int has = 1;
                switch (O->opType[op]) { /* :1472-1522 */
                case PSGPU_OP_BLEND: case PSGPU_OP_RICCIBLEND:
                    lf = SUB(MUL(V(2.0f), ADD(V(0.5f), lf)), V(1.0f));
                    rf = SUB(MUL(V(2.0f), ADD(V(0.5f), rf)), V(1.0f));
                    break;
                case PSGPU_OP_UNION: case PSGPU_OP_INTERSECT:
                    lf = ONE01(_mm_cmpeq_ps(SUB(cur, lf), _mm_setzero_ps()));
                    rf = ONE01(_mm_cmpeq_ps(SUB(cur, rf), _mm_setzero_ps()));
                    break;
                case PSGPU_OP_DIF: case PSGPU_OP_SMOOTHDIF:
                    lf = ONE01(_mm_cmpeq_ps(lf, cur));
                    rf = ONE01(_mm_cmpeq_ps(SUB(V(1.0f), rf), cur));
                    break;
                case PSGPU_OP_WARPTWIST: case PSGPU_OP_WARPTAPER:
                case PSGPU_OP_WARPBEND: case PSGPU_OP_WARPSHEAR:
                    ox = lcx; oy = lcy; oz = lcz;
                    has = 0;
                    break;
                default:
                    has = 0; /* colour of the previous op is kept */
                    break;
                }
                if (has) {
                    ox = ADD(MUL(lf, lcx), MUL(rf, rcx));
                    oy = ADD(MUL(lf, lcy), MUL(rf, rcy));
                    oz = ADD(MUL(lf, lcz), MUL(rf, rcz));
                }
                done[op] = 1;
                _mm_storeu_ps(&colX[op * 4], ox);
                _mm_storeu_ps(&colY[op * 4], oy);
                _mm_storeu_ps(&colZ[op * 4], oz);
            } else {
                if (lop && !done[L] && top + 1 < STACK_CAP) sid[++top] = L;
                if (rop && !done[R] && top + 1 < STACK_CAP) sid[++top] = R;
            }
        }
    } else {
        ox = V(P->colorX[0]); oy = V(P->colorY[0]); oz = V(P->colorZ[0]);
    }
    *cX = ox; *cY = oy; *cZ = oz;
    return field;
}

/* FieldComputer::normal + SimdNormalize, PS_Polygonizer.cpp:1598-1622, PS_SIMDVecN.h:435-442 */
static void normal_at(const PsModelRef* m, V4 pX, V4 pY, V4 pZ, V4 fv, V4* nX, V4* nY, V4* nZ) {
    const float delta = PSGPU_NORMAL_DELTA;
    V4 inv = V(-1.0f / delta);
    V4 dx = field_only(m, ADD(pX, V(delta)), pY, pZ);
    V4 dy = field_only(m, pX, ADD(pY, V(delta)), pZ);
    V4 dz = field_only(m, pX, pY, ADD(pZ, V(delta)));
    V4 x = MUL(SUB(dx, fv), inv), y = MUL(SUB(dy, fv), inv), z = MUL(SUB(dz, fv), inv);
    V4 im = v_rsqrt(ADD(ADD(MUL(x, x), MUL(y, y)), MUL(z, z)));
    *nX = MUL(x, im); *nY = MUL(y, im); *nZ = MUL(z, im);
}

void psor_field_value(const PsModelRef* m, const float* x4, const float* y4, const float* z4, float* out4) {
    _mm_storeu_ps(out4, field_only(m, _mm_loadu_ps(x4), _mm_loadu_ps(y4), _mm_loadu_ps(z4)));
}

void psor_field_value_and_color(const PsModelRef* m, const float* x4, const float* y4, const float* z4,
                                float* f4, float* cx4, float* cy4, float* cz4) {
    V4 cx, cy, cz;
    V4 f = field_and_color(m, _mm_loadu_ps(x4), _mm_loadu_ps(y4), _mm_loadu_ps(z4), &cx, &cy, &cz);
    _mm_storeu_ps(f4, f);
    _mm_storeu_ps(cx4, cx);
    _mm_storeu_ps(cy4, cy);
    _mm_storeu_ps(cz4, cz);
}

/* ------------------------------------------------------------------------- */
/* MPU lattice, Polygonize PS_Polygonizer.cpp:325-371 / CountMPUNeeded :388-412 */
static void mpu_dims(float cs, PsVec3f lo, PsVec3f hi, int d[3]) {
    const float ext[3] = {hi.x - lo.x, hi.y - lo.y, hi.z - lo.z};
    for (int a = 0; a < 3; ++a) {
        int cells = (int)ceilf(ext[a] / cs);
        d[a] = cells / PSGPU_CELLS_PER_MPU + ((cells % PSGPU_CELLS_PER_MPU) != 0);
    }
}

uint32_t psor_count_mpus(float cs, const float lo[3], const float hi[3]) {
    PsVec3f l = {lo[0], lo[1], lo[2]}, h = {hi[0], hi[1], hi[2]};
    int d[3];
    mpu_dims(cs, l, h, d);
    return (uint32_t)(d[0] * d[1] * d[2]);
}

static PsVec3f mpu_origin(float cs, PsVec3f lo, const int d[3], uint32_t idx) {
    const float side = cs * (float)PSGPU_CELLS_PER_MPU;
    int k = (int)(idx % (uint32_t)d[2]);
    int j = (int)((idx / (uint32_t)d[2]) % (uint32_t)d[1]);
    int i = (int)(idx / ((uint32_t)d[2] * (uint32_t)d[1]));
    PsVec3f o = {lo.x + (float)i * side, lo.y + (float)j * side, lo.z + (float)k * side};
    return o;
}

/* One MPU: process_cells_simd, PS_Polygonizer.cpp:475-829.  Returns 0 if the MPU
 * exited at the S1 precheck (counts untouched in the reference; zero here). */
typedef struct MpuOut {
    uint16_t ctV, ctT;
    uint8_t passed, overflow;
    uint32_t evals;
    float* vdata;  /* ctV * 9: pos(3) nrm(3) col(3) */
    uint16_t* tri; /* ctT * 3 */
} MpuOut;

static void process_mpu(const PsModelRef* m, float cs, PsVec3f lo, MpuOut* o, float* vbuf, uint16_t* tbuf) {
    memset(o, 0, sizeof(*o));
    t_phase = 0;
    /* S1: 8 MPU corners as two quads (:483-540) */
    {
        const float side = 7.0f * cs;
        V4 X = _mm_setr_ps(0, 1, 0, 1), Y = _mm_setr_ps(0, 0, 1, 1);
        V4 px = ADD(MUL(X, V(side)), V(lo.x)), py = ADD(MUL(Y, V(side)), V(lo.y));
        V4 z1 = ADD(MUL(V(0.0f), V(side)), V(lo.z)), z2 = ADD(MUL(V(1.0f), V(side)), V(lo.z));
        V4 f1 = field_only(m, px, py, z1), f2 = field_only(m, px, py, z2);
        int m1 = _mm_movemask_ps(_mm_cmpgt_ps(f1, _mm_setzero_ps()));
        int m2 = _mm_movemask_ps(_mm_cmpgt_ps(f2, _mm_setzero_ps()));
        if (m1 == 0 && m2 == 0) return;
    }
    o->passed = 1;
    t_phase = 1;
    /* S2: 8^3 field cache, z in quads of 4 (:550-610); fv[x][y][z] */
    float fv[8][8][8];
    int ctIn = 0, ctOut = 0;
    const V4 lanes = _mm_setr_ps(0, 1, 2, 3);
    for (int i = 0; i < 8; ++i)
        for (int j = 0; j < 8; ++j)
            for (int k = 0; k < 2; ++k) {
                V4 px = V(lo.x + (float)i * cs);
                V4 py = V(lo.y + (float)j * cs);
                V4 pz = ADD(V(lo.z), MUL(ADD(V((float)k * 4.0f), lanes), V(cs)));
                V4 f = field_only(m, px, py, pz);
                _mm_storeu_ps(&fv[i][j][k * 4], f);
                o->evals++;
                int in = _mm_movemask_ps(_mm_cmpge_ps(f, V(PSGPU_ISO_VALUE)));
                ctIn += __builtin_popcount((unsigned)in);
                ctOut += 4 - __builtin_popcount((unsigned)in);
            }
    if (ctIn == 0 || ctOut == 0) return;

    /* S3-S6 (:647-825) */
    int16_t edgeVid[8][8][8][3];
    memset(edgeVid, 0xff, sizeof(edgeVid));
    const float oneThird = 1.0f / 3.0f;
    const V4 rootRes = MUL(lanes, V(oneThird));
    uint32_t ctV = 0, ctT = 0;
    for (int i = 0; i < 7; ++i)
        for (int j = 0; j < 7; ++j)
            for (int k = 0; k < 7; ++k) {
                int cfg = 0;
                for (int c = 0; c < 8; ++c) {
                    int x = i + ((c >> 2) & 1), y = j + ((c >> 1) & 1), z = k + (c & 1);
                    cfg |= (fv[x][y][z] >= PSGPU_ISO_VALUE) << c;
                }
                if (cfg == 0 || cfg == 255) continue;
                const int* row = g_tri[cfg];
                int vid[16], ctE = 0;
                for (int ic = 0; ic < 16 && row[ic] != -1; ++ic) {
                    int e = row[ic], c1 = k_corner1[e], ax = k_axis[e];
                    int sx = i + ((c1 & 4) >> 2), sy = j + ((c1 & 2) >> 1), sz = k + (c1 & 1);
                    int v = edgeVid[sx][sy][sz][ax];
                    if (v < 0) {
                        /* S4: root bracketing with 4 samples (:722-762) */
                        float e1[3] = {lo.x + cs * (float)sx, lo.y + cs * (float)sy, lo.z + cs * (float)sz};
                        float e2[3] = {e1[0], e1[1], e1[2]};
                        e2[ax] = e1[ax] + cs;
                        V4 qx = ADD(V(e1[0]), MUL(V(e2[0] - e1[0]), rootRes));
                        V4 qy = ADD(V(e1[1]), MUL(V(e2[1] - e1[1]), rootRes));
                        V4 qz = ADD(V(e1[2]), MUL(V(e2[2] - e1[2]), rootRes));
                        t_phase = 2;
                        V4 rf = field_only(m, qx, qy, qz);
                        int in = _mm_movemask_ps(_mm_cmpge_ps(rf, V(PSGPU_ISO_VALUE)));
                        int state = in & 1, iv = 0;
                        for (int q = 1; q < 4; ++q) {
                            iv = q;
                            if (((in >> q) & 1) != state) break;
                        }
                        float a[3] = {lane(qx, iv - 1), lane(qy, iv - 1), lane(qz, iv - 1)};
                        float b[3] = {lane(qx, iv), lane(qy, iv), lane(qz, iv)};
                        float fa = lane(rf, iv - 1), fb = lane(rf, iv);
                        float scale = (PSGPU_ISO_VALUE - fa) / (fb - fa);
                        float p[3];
                        for (int c = 0; c < 3; ++c) p[c] = a[c] + scale * (b[c] - a[c]);
                        /* S5: field + colour + normal (:764-807) */
                        V4 cx, cy, cz, nx, ny, nz;
                        t_phase = 4;
                        V4 vf = field_and_color(m, V(p[0]), V(p[1]), V(p[2]), &cx, &cy, &cz);
                        t_phase = 3;
                        normal_at(m, V(p[0]), V(p[1]), V(p[2]), vf, &nx, &ny, &nz);
                        if (ctV >= PSGPU_MAX_MPU_VERTEX_COUNT * 4) { o->overflow = 1; v = 0; }
                        else {
                            float* d = &vbuf[ctV * 9];
                            d[0] = p[0]; d[1] = p[1]; d[2] = p[2];
                            d[3] = lane(nx, 0); d[4] = lane(ny, 0); d[5] = lane(nz, 0);
                            d[6] = lane(cx, 0); d[7] = lane(cy, 0); d[8] = lane(cz, 0);
                            v = (int)ctV++;
                            edgeVid[sx][sy][sz][ax] = (int16_t)v;
                        }
                    }
                    vid[ic] = v;
                    ++ctE;
                }
                for (int t = 0; t < ctE / 3; ++t) {
                    if (ctT >= PSGPU_MAX_MPU_TRIANGLE_COUNT * 4) { o->overflow = 1; break; }
                    tbuf[ctT * 3 + 0] = (uint16_t)vid[t * 3 + 0];
                    tbuf[ctT * 3 + 1] = (uint16_t)vid[t * 3 + 1];
                    tbuf[ctT * 3 + 2] = (uint16_t)vid[t * 3 + 2];
                    ++ctT;
                }
            }
    if (ctV > PSGPU_MAX_MPU_VERTEX_COUNT || ctT > PSGPU_MAX_MPU_TRIANGLE_COUNT) o->overflow = 1;
    o->ctV = (uint16_t)ctV;
    o->ctT = (uint16_t)ctT;
    if (ctV) {
        o->vdata = (float*)malloc((size_t)ctV * 9 * sizeof(float));
        memcpy(o->vdata, vbuf, (size_t)ctV * 9 * sizeof(float));
    }
    if (ctT) {
        o->tri = (uint16_t*)malloc((size_t)ctT * 3 * sizeof(uint16_t));
        memcpy(o->tri, tbuf, (size_t)ctT * 3 * sizeof(uint16_t));
    }
}

/* ------------------------------------------------------------------------- */
struct psor_result {
    uint32_t ctMPUs, begin;
    MpuOut* mpus;
    uint32_t ctV, ctT;
};

typedef struct Job {
    const PsModelRef* m;
    float cs;
    PsVec3f lo;
    int dims[3];
    uint32_t begin, count;
    MpuOut* out;
    volatile uint32_t next;
    int keep;
} Job;

static void* worker(void* arg) {
    Job* J = (Job*)arg;
    memset(t_cnt, 0, sizeof(t_cnt));
    float* vbuf = (float*)malloc((size_t)PSGPU_MAX_MPU_VERTEX_COUNT * 4 * 9 * sizeof(float));
    uint16_t* tbuf = (uint16_t*)malloc((size_t)PSGPU_MAX_MPU_TRIANGLE_COUNT * 4 * 3 * sizeof(uint16_t));
    for (;;) {
        uint32_t s = __sync_fetch_and_add(&J->next, 8u);
        if (s >= J->count) break;
        uint32_t e = s + 8 < J->count ? s + 8 : J->count;
        for (uint32_t w = s; w < e; ++w) {
            PsVec3f o = mpu_origin(J->cs, J->lo, J->dims, J->begin + w);
            process_mpu(J->m, J->cs, o, &J->out[w], vbuf, tbuf);
            if (!J->keep) {
                free(J->out[w].vdata);
                free(J->out[w].tri);
                J->out[w].vdata = NULL;
                J->out[w].tri = NULL;
            }
        }
    }
    free(vbuf);
    free(tbuf);
    pthread_mutex_lock(&g_cnt_mu);
    for (int ph = 0; ph < 5; ++ph)
        for (int k = 0; k < PSOR_NCNT; ++k) g_cnt[ph][k] += t_cnt[ph][k];
    pthread_mutex_unlock(&g_cnt_mu);
    return NULL;
}

/* Work counters of the last psor_polygonize (see t_cnt). */
void psor_work_counts(uint64_t out[5 * PSOR_NCNT]) {
    pthread_mutex_lock(&g_cnt_mu);
    memcpy(out, g_cnt, sizeof(g_cnt));
    pthread_mutex_unlock(&g_cnt_mu);
}

int psor_polygonize(float cellsize, const PsModelRef* m, uint32_t mpuBegin, uint32_t mpuEnd, int nthreads,
                    int keepMesh, psor_result** out) {
    *out = NULL;
    if (m->prims->ctPrims == 0 || !(cellsize > 0.0f)) return PSGPU_RET_PARAM_ERROR;
    pthread_once(&g_tri_once, build_tritable);
    Job J;
    memset(&J, 0, sizeof(J));
    J.m = m;
    J.cs = cellsize;
    J.lo = m->prims->bboxLo;
    mpu_dims(cellsize, m->prims->bboxLo, m->prims->bboxHi, J.dims);
    uint32_t total = (uint32_t)(J.dims[0] * J.dims[1] * J.dims[2]);
    if (mpuEnd > total) mpuEnd = total;
    if (mpuBegin > mpuEnd) mpuBegin = mpuEnd;
    J.begin = mpuBegin;
    J.count = mpuEnd - mpuBegin;
    J.out = (MpuOut*)calloc(J.count ? J.count : 1, sizeof(MpuOut));
    J.keep = keepMesh;
    pthread_mutex_lock(&g_cnt_mu);
    memset(g_cnt, 0, sizeof(g_cnt));
    pthread_mutex_unlock(&g_cnt_mu);
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    for (int t = 1; t < nthreads; ++t) pthread_create(&th[t], NULL, worker, &J);
    worker(&J);
    for (int t = 1; t < nthreads; ++t) pthread_join(th[t], NULL);
    psor_result* r = (psor_result*)calloc(1, sizeof(psor_result));
    r->ctMPUs = J.count;
    r->begin = mpuBegin;
    r->mpus = J.out;
    for (uint32_t w = 0; w < J.count; ++w) {
        r->ctV += J.out[w].ctV;
        r->ctT += J.out[w].ctT;
    }
    *out = r;
    return PSGPU_RET_SUCCESS;
}

void psor_result_info(const psor_result* r, uint32_t* ctMPUs, uint32_t* ctV, uint32_t* ctT) {
    *ctMPUs = r->ctMPUs;
    *ctV = r->ctV;
    *ctT = r->ctT;
}

/* Per-MPU arrays: stats[w] = {passed, evals, ctV, ctT, overflow}; pos/nrm/col/tri
 * concatenated in MPU order (triangles keep MPU-local ids, as in PolyMPUs). */
void psor_result_copy(const psor_result* r, uint32_t* stats5, float* pos, float* nrm, float* col, uint16_t* tri) {
    size_t v = 0, t = 0;
    for (uint32_t w = 0; w < r->ctMPUs; ++w) {
        const MpuOut* o = &r->mpus[w];
        if (stats5) {
            stats5[w * 5 + 0] = o->passed;
            stats5[w * 5 + 1] = o->evals;
            stats5[w * 5 + 2] = o->ctV;
            stats5[w * 5 + 3] = o->ctT;
            stats5[w * 5 + 4] = o->overflow;
        }
        for (uint32_t i = 0; i < o->ctV && o->vdata; ++i, ++v) {
            for (int c = 0; c < 3; ++c) {
                if (pos) pos[v * 3 + c] = o->vdata[i * 9 + c];
                if (nrm) nrm[v * 3 + c] = o->vdata[i * 9 + 3 + c];
                if (col) col[v * 3 + c] = o->vdata[i * 9 + 6 + c];
            }
        }
        if (tri && o->tri) memcpy(&tri[t * 3], o->tri, (size_t)o->ctT * 3 * sizeof(uint16_t));
        t += o->ctT;
    }
}

void psor_result_free(psor_result* r) {
    if (!r) return;
    for (uint32_t w = 0; w < r->ctMPUs; ++w) {
        free(r->mpus[w].vdata);
        free(r->mpus[w].tri);
    }
    free(r->mpus);
    free(r);
}

/* ------------------------------------------------------------------------- */
/* PrepareBBoxes (PS_Polygonizer.cpp:55-309) with isoDist = ISO_DIST + 5*MIN_CELL */
int psor_prepare_bboxes(PsSoaBlobPrims* P, const PsSoaBoxMatrices* BM, PsSoaBlobOps* O) {
    if (P->ctPrims == 0) return PSGPU_RET_PARAM_ERROR;
    const float iso = PSGPU_ISO_DIST + 5.0f * PSGPU_MIN_CELL_SIZE;
    PsVec3f blo = {0, 0, 0}, bhi = {0, 0, 0};
    for (uint32_t i = 0; i < P->ctPrims; ++i) {
        float lo[3], hi[3];
        int have = 1;
        float p[3] = {P->posX[i], P->posY[i], P->posZ[i]};
        float d[3] = {P->dirX[i], P->dirY[i], P->dirZ[i]};
        switch (P->skeletType[i]) {
        case PSGPU_PRIM_POINT:
            for (int a = 0; a < 3; ++a) { lo[a] = p[a] - iso; hi[a] = p[a] + iso; }
            break;
        case PSGPU_PRIM_LINE:
            for (int a = 0; a < 3; ++a) {
                float ex = iso * 1.0f + (3.0f * iso) * (d[a] - p[a]);
                lo[a] = p[a] - ex; hi[a] = d[a] + ex;
            }
            break;
        case PSGPU_PRIM_RING: case PSGPU_PRIM_DISC: {
            float r = P->resX[i] + iso;
            for (int a = 0; a < 3; ++a) {
                float ex = (r + iso) * (1.0f - d[a]) + iso * d[a];
                lo[a] = p[a] - ex; hi[a] = p[a] + ex;
            }
        } break;
        case PSGPU_PRIM_CYLINDER: {
            float r = P->resX[i], h = P->resY[i];
            for (int a = 0; a < 3; ++a) {
                float s1 = p[a] + h * d[a];
                float ex = (iso + r) * 1.0f + (0.5f * iso) * d[a];
                lo[a] = p[a] - ex; hi[a] = s1 + ex;
            }
        } break;
        case PSGPU_PRIM_CUBE: {
            float s = P->resX[i] + iso;
            for (int a = 0; a < 3; ++a) { lo[a] = p[a] - s; hi[a] = p[a] + s; }
        } break;
        case PSGPU_PRIM_TRIANGLE: {
            float r[3] = {P->resX[i], P->resY[i], P->resZ[i]};
            for (int a = 0; a < 3; ++a) {
                float mn = p[a] < d[a] ? p[a] : d[a];
                mn = mn < r[a] ? mn : r[a];
                float mx = p[a] > d[a] ? p[a] : d[a];
                mx = mx > r[a] ? mx : r[a];
                lo[a] = mn - iso; hi[a] = mx + iso;
            }
        } break;
        default:
            have = 0;
            lo[0] = P->vPrimBoxLoX[i]; lo[1] = P->vPrimBoxLoY[i]; lo[2] = P->vPrimBoxLoZ[i];
            hi[0] = P->vPrimBoxHiX[i]; hi[1] = P->vPrimBoxHiY[i]; hi[2] = P->vPrimBoxHiZ[i];
            break;
        }
        (void)have;
        uint32_t im = P->idxMatrix[i];
        if (im != 0 && BM && im < BM->count) { /* mat4Transform, PS_MATRIX4.h:199-209 */
            const float* M = &BM->matrix[im * PSGPU_BOX_MATRIX_STRIDE];
            float tl[3], th[3];
            for (int r = 0; r < 3; ++r) {
                tl[r] = ((M[0 + r] * lo[0] + M[4 + r] * lo[1]) + M[8 + r] * lo[2]) + M[12 + r];
                th[r] = ((M[0 + r] * hi[0] + M[4 + r] * hi[1]) + M[8 + r] * hi[2]) + M[12 + r];
            }
            memcpy(lo, tl, sizeof(lo));
            memcpy(hi, th, sizeof(hi));
        }
        P->vPrimBoxLoX[i] = lo[0]; P->vPrimBoxLoY[i] = lo[1]; P->vPrimBoxLoZ[i] = lo[2];
        P->vPrimBoxHiX[i] = hi[0]; P->vPrimBoxHiY[i] = hi[1]; P->vPrimBoxHiZ[i] = hi[2];
        if (i == 0) {
            blo.x = lo[0]; blo.y = lo[1]; blo.z = lo[2];
            bhi.x = hi[0]; bhi.y = hi[1]; bhi.z = hi[2];
        } else {
            blo.x = blo.x < lo[0] ? blo.x : lo[0]; blo.y = blo.y < lo[1] ? blo.y : lo[1]; blo.z = blo.z < lo[2] ? blo.z : lo[2];
            bhi.x = bhi.x > hi[0] ? bhi.x : hi[0]; bhi.y = bhi.y > hi[1] ? bhi.y : hi[1]; bhi.z = bhi.z > hi[2] ? bhi.z : hi[2];
        }
    }
    P->bboxLo = blo;
    P->bboxHi = bhi;
    /* op boxes bottom-up (:238-307): a post-order walk gives the same result */
    if (O->ctOps > 0) {
        uint8_t doneOp[256];
        memset(doneOp, 0, sizeof(doneOp));
        uint32_t st[STACK_CAP];
        int top = 0;
        st[0] = 0;
        while (top >= 0) {
            uint32_t op = st[top], L = O->opLeftChild[op], R = O->opRightChild[op];
            int lop = (O->opChildKind[op] & 2) >> 1, rop = O->opChildKind[op] & 1;
            if (!((lop && !doneOp[L]) || (rop && !doneOp[R]))) {
                --top;
                float l[6], r[6];
                if (lop) { l[0] = O->vBoxLoX[L]; l[1] = O->vBoxLoY[L]; l[2] = O->vBoxLoZ[L]; l[3] = O->vBoxHiX[L]; l[4] = O->vBoxHiY[L]; l[5] = O->vBoxHiZ[L]; }
                else { l[0] = P->vPrimBoxLoX[L]; l[1] = P->vPrimBoxLoY[L]; l[2] = P->vPrimBoxLoZ[L]; l[3] = P->vPrimBoxHiX[L]; l[4] = P->vPrimBoxHiY[L]; l[5] = P->vPrimBoxHiZ[L]; }
                if (rop) { r[0] = O->vBoxLoX[R]; r[1] = O->vBoxLoY[R]; r[2] = O->vBoxLoZ[R]; r[3] = O->vBoxHiX[R]; r[4] = O->vBoxHiY[R]; r[5] = O->vBoxHiZ[R]; }
                else { r[0] = P->vPrimBoxLoX[R]; r[1] = P->vPrimBoxLoY[R]; r[2] = P->vPrimBoxLoZ[R]; r[3] = P->vPrimBoxHiX[R]; r[4] = P->vPrimBoxHiY[R]; r[5] = P->vPrimBoxHiZ[R]; }
                O->vBoxLoX[op] = l[0] < r[0] ? l[0] : r[0];
                O->vBoxLoY[op] = l[1] < r[1] ? l[1] : r[1];
                O->vBoxLoZ[op] = l[2] < r[2] ? l[2] : r[2];
                O->vBoxHiX[op] = l[3] > r[3] ? l[3] : r[3];
                O->vBoxHiY[op] = l[4] > r[4] ? l[4] : r[4];
                O->vBoxHiZ[op] = l[5] > r[5] ? l[5] : r[5];
                doneOp[op] = 1;
            } else {
                if (lop && !doneOp[L] && top + 1 < STACK_CAP) st[++top] = L;
                if (rop && !doneOp[R] && top + 1 < STACK_CAP) st[++top] = R;
            }
        }
    }
    return PSGPU_RET_SUCCESS;
}

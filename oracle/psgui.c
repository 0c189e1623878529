/* TEST INFRASTRUCTURE ONLY -- the CPU restatement of ParsipHaptics' own polygonizer (the
 * "GUI path") used as the parity checker of psgpu_gui_* (the HIP compat
 * mode).  Never linked into the product.
 *
 * Restated, function by function, from
 *   ParsipHaptics/include/CompactBlobTree.cpp   (COMPACTBLOBTREE field, colour, normal, Newton)
 *   ParsipHaptics/include/CPolyParsipOptimized.cpp (CParsipOptimized::setup/run,
 *                                                 CSIMDMPURunBody::doMarchingCubes, getEdge/setEdge)
 *   PS_FrameWork/include/PS_Vector.h            (vec3f / vec4f arithmetic order)
 *   PS_FrameWork/include/PS_GeometryFuncs.cpp   (NearestPointInLineSegment)
 *   PS_BlobTree/include/CSkeletonTriangle.cpp   (ComputeTriangleSquareDist)
 *   PS_BlobTree/include/CFieldFunction.h:104    (ComputeWyvillFieldValueSquare)
 * in fp32 with the reference's operation order (-ffp-contract=off, no fast-math).
 *
 * Deliberate deviation (also in the device code): the reference calls powf (Ricci) and
 * cos/sin (warps) from the host libm; here they are the correctly rounded fp32 results,
 * computed as (float)pow((double), (double)) etc., so that the oracle and the GPU agree
 * bit for bit on every platform.  The reference's own results depend on its C runtime:
 * glibc 2.35's powf / cosf / sinf differ from the correctly rounded value by 1 ulp on about
 * 0.4 % / 1 % of arguments (tests/test_gui.py measures it on the scene's own arguments).
 *
 * PCM (precise contact modelling, CompactBlobTree.cpp:490-614) keeps a contact state, the
 * PCMCONTEXT maxima, that the reference updates as a running maximum in each TBB body's
 * copy of the tree, so its propagation fields depend on the body split.  The defined order
 * restated here (and on the device, include/parsip_gpu_gui.h): a run reads the state it
 * started with (cur*) and raises the state to the largest compression its evaluations met
 * when it ends (max*); probes read it and never change it.  marchTowardNode stops after
 * PSGUI_PCM_MARCH_MAX steps (the reference loops until it converges, forever if it never
 * does).
 *
 * Parity status: no output of this path is recorded in the reference beyond
 * Distrib/ParsipHaptics_Release.csv, which came from a different build and scene (see
 * DESIGN.md §6): "parity unpinned" beyond the restatement, the shared MC table digest and
 * the reference scene's structure.
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/parsip_gpu_gui.h"

/* GRID_DIM: 8 in this snapshot (CPolyParsipOptimized.h:23, GRID_DIM_8); 16 and 32 are the
 * header's other settings (:25-39).  The oracle takes it at run time (psgui_set_grid_dim). */
static int GRID_DIM = 8;
static int CELLID_SHIFT = 3;
#define CELLS (GRID_DIM - 1)
#define MAX_GRID 32
#define ISO_VALUE 0.5f
#define FIELD_VALUE_EPSILON 0.001f
#define NORMAL_DELTA 0.001f
#define MAX_FIELD_VALUE 1.0f
#define EPSILON 0.0001f
#define EDGETABLE_DEPTH 8
#define CELLID_HASHSIZE (MAX_GRID * MAX_GRID * MAX_GRID)
#define MAX_KIDS 1024

typedef struct { float x, y, z, w; } v4;
typedef struct { float x, y, z; } v3;

typedef struct {
    float curL, curR;  /* maxCompressionLeft / Right as the run started (read)             */
    float maxL, maxR;  /* the running maxima (written when `update`)                       */
    int update;
} PcmCtx;

typedef struct {
    const PsGuiPrim* P;
    uint32_t nP;
    const PsGuiOp* O;
    uint32_t nO;
    const uint32_t* K;
    const PsGuiMatrix* M;
    PcmCtx* pcm;
} Tree;

#define ISO_DISTANCE 0.454202f  /* _constSettings.h:11 */
static float field_op(const Tree* T, v4 p, int id, float* storeOp, float* storePrim);

static float cr_powf(float x, float y) { return (float)pow((double)x, (double)y); }
static float cr_cosf(float x) { return (float)cos((double)x); }
static float cr_sinf(float x) { return (float)sin((double)x); }

static int FLOAT_EQ(float x, float v) { return ((v - EPSILON) < x) && (x < (v + EPSILON)); }  /* mathHelper.h:95 */
static float maxf(float a, float b) { return (a > b) ? a : b; }
static float Absolutef(float n) { return n < 0 ? (0 - n) : n; }

static v3 v3sub(v3 a, v3 b) { v3 r = {a.x - b.x, a.y - b.y, a.z - b.z}; return r; }
static v3 v3add(v3 a, v3 b) { v3 r = {a.x + b.x, a.y + b.y, a.z + b.z}; return r; }
static v3 v3scale(v3 a, float s) { v3 r = {a.x * s, a.y * s, a.z * s}; return r; }
static float v3dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static float v3len2(v3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
static float v3dist2(v3 self, v3 a) {  /* Vector3d::dist2 (PS_Vector.h:888-894) */
    float dx = a.x - self.x, dy = a.y - self.y, dz = a.z - self.z;
    return dx * dx + dy * dy + dz * dz;
}
static void v3normalize(v3* a) {  /* PS_Vector.h:910-925 */
    float d = sqrtf(a->x * a->x + a->y * a->y + a->z * a->z);
    if (d > 0) {
        float r = 1.0f / d;
        a->x *= r; a->y *= r; a->z *= r;
    } else {
        a->x = a->y = a->z = 1;
    }
}
static v3 xyz(const float* f) { v3 r = {f[0], f[1], f[2]}; return r; }
static float v4dot(const float* r, v4 p) { return r[0] * p.x + r[1] * p.y + r[2] * p.z + r[3] * p.w; }

static float wyvill(float dd) {  /* CFieldFunction.h:104-114 */
    if (dd >= 1.0f) return 0.0f;
    float t = (1.0f - dd);
    return t * t * t;
}

/* PS_GeometryFuncs.cpp:156-179 */
static v3 nearest_point_on_segment(v3 point, v3 line0, v3 line1) {
    v3 d = v3sub(line1, line0);
    if (FLOAT_EQ(0.0f, d.x) && FLOAT_EQ(0.0f, d.y) && FLOAT_EQ(0.0f, d.z)) return line0;  /* operator== */
    float delta = v3dot(v3sub(point, line0), d) / v3dot(d, d);
    if (delta < 0) delta = 0;
    else if (delta > 1) delta = 1;
    return v3add(line0, v3scale(d, delta));
}

/* CSkeletonTriangle.cpp:19-254 */
static float triangle_sqr_dist(v3 v0, v3 v1, v3 v2, v3 p) {
    v3 dif = v3sub(v0, p), edge0 = v3sub(v1, v0), edge1 = v3sub(v2, v0);
    float a00 = v3len2(edge0), a01 = v3dot(edge0, edge1), a11 = v3len2(edge1);
    float b0 = v3dot(dif, edge0), b1 = v3dot(dif, edge1), c = v3len2(dif);
    float det = Absolutef(a00 * a11 - a01 * a01);
    float s = a01 * b1 - a11 * b0;
    float t = a01 * b0 - a00 * b1;
    float sq;
    if (s + t <= det) {
        if (s < 0.0f) {
            if (t < 0.0f) {  /* region 4 */
                if (b0 < 0.0f) {
                    t = 0.0f;
                    if (-b0 >= a00) { s = 1.0f; sq = a00 + 2.0f * b0 + c; }
                    else { s = -b0 / a00; sq = b0 * s + c; }
                } else {
                    s = 0.0f;
                    if (b1 >= 0.0f) { t = 0.0f; sq = c; }
                    else if (-b1 >= a11) { t = 1.0f; sq = a11 + 2.0f * b1 + c; }
                    else { t = -b1 / a11; sq = b1 * t + c; }
                }
            } else {  /* region 3 */
                s = 0.0f;
                if (b1 >= 0.0f) { t = 0.0f; sq = c; }
                else if (-b1 >= a11) { t = 1.0f; sq = a11 + 2.0f * b1 + c; }
                else { t = -b1 / a11; sq = b1 * t + c; }
            }
        } else if (t < 0.0f) {  /* region 5 */
            t = 0.0f;
            if (b0 >= 0.0f) { s = 0.0f; sq = c; }
            else if (-b0 >= a00) { s = 1.0f; sq = a00 + 2.0f * b0 + c; }
            else { s = -b0 / a00; sq = b0 * s + c; }
        } else {  /* region 0 */
            float invDet = 1.0f / det;
            s *= invDet;
            t *= invDet;
            sq = s * (a00 * s + a01 * t + 2.0f * b0) + t * (a01 * s + a11 * t + 2.0f * b1) + c;
        }
    } else {
        float tmp0, tmp1, numer, denom;
        if (s < 0.0f) {  /* region 2 */
            tmp0 = a01 + b0;
            tmp1 = a11 + b1;
            if (tmp1 > tmp0) {
                numer = tmp1 - tmp0;
                denom = a00 - 2.0f * a01 + a11;
                if (numer >= denom) { s = 1.0f; t = 0.0f; sq = a00 + 2.0f * b0 + c; }
                else {
                    s = numer / denom;
                    t = 1.0f - s;
                    sq = s * (a00 * s + a01 * t + 2.0f * b0) + t * (a01 * s + a11 * t + 2.0f * b1) + c;
                }
            } else {
                s = 0.0f;
                if (tmp1 <= 0.0f) { t = 1.0f; sq = a11 + 2.0f * b1 + c; }
                else if (b1 >= 0.0f) { t = 0.0f; sq = c; }
                else { t = -b1 / a11; sq = b1 * t + c; }
            }
        } else if (t < 0.0f) {  /* region 6 */
            tmp0 = a01 + b1;
            tmp1 = a00 + b0;
            if (tmp1 > tmp0) {
                numer = tmp1 - tmp0;
                denom = a00 - 2.0f * a01 + a11;
                if (numer >= denom) { t = 1.0f; s = 0.0f; sq = a11 + 2.0f * b1 + c; }
                else {
                    t = numer / denom;
                    s = 1.0f - t;
                    sq = s * (a00 * s + a01 * t + 2.0f * b0) + t * (a01 * s + a11 * t + 2.0f * b1) + c;
                }
            } else {
                t = 0.0f;
                if (tmp1 <= 0.0f) { s = 1.0f; sq = a00 + 2.0f * b0 + c; }
                else if (b0 >= 0.0f) { s = 0.0f; sq = c; }
                else { s = -b0 / a00; sq = b0 * s + c; }
            }
        } else {  /* region 1 */
            numer = a11 + b1 - a01 - b0;
            if (numer <= 0.0f) { s = 0.0f; t = 1.0f; sq = a11 + 2.0f * b1 + c; }
            else {
                denom = a00 - 2.0f * a01 + a11;
                if (numer >= denom) { s = 1.0f; t = 0.0f; sq = a00 + 2.0f * b0 + c; }
                else {
                    s = numer / denom;
                    t = 1.0f - s;
                    sq = s * (a00 * s + a01 * t + 2.0f * b0) + t * (a01 * s + a11 * t + 2.0f * b1) + c;
                }
            }
        }
    }
    (void)s;
    (void)t;
    if (sq < 0.0f) sq = 0.0f;
    return sq;
}

/* COMPACTBLOBTREE::fieldvaluePrim (CompactBlobTree.cpp:893-1092) */
static float field_prim(const Tree* T, v4 p, int id, float* storePrim) {
    const PsGuiPrim* P = &T->P[id];
    v3 pn = {p.x, p.y, p.z};
    if (P->idxMtx != 0) {
        const PsGuiMatrix* m = &T->M[P->idxMtx];
        v4 pp = {p.x, p.y, p.z, 1.0f};
        pn.x = v4dot(m->r[0], pp);
        pn.y = v4dot(m->r[1], pp);
        pn.z = v4dot(m->r[2], pp);
    }
    float fv = 0.0f;
    switch (P->type) {
    case PSGUI_PRIM_POINT:
        fv = wyvill(v3dist2(pn, xyz(P->pos)));
        break;
    case PSGUI_PRIM_CYLINDER: {
        v3 pos = v3sub(pn, xyz(P->pos));
        float y = v3dot(pos, xyz(P->dir));
        float x = maxf(0.0f, sqrtf(v3len2(pos) - y * y) - P->res1[0]);
        if (y > 0.0f) y = maxf(0.0f, y - P->res2[0]);
        fv = wyvill(x * x + y * y);
    } break;
    case PSGUI_PRIM_TRIANGLE:
        fv = wyvill(triangle_sqr_dist(xyz(P->pos), xyz(P->res1), xyz(P->res2), pn));
        break;
    case PSGUI_PRIM_CUBE: {
        v3 center = xyz(P->pos);
        float side = P->res1[0];
        v3 dif = v3sub(pn, center);
        float dist2 = 0.0f, delta, projected;
        const float axes[3][3] = {{1.0f, 0.0f, 0.0f}, {0.0f, 1.0f, 0.0f}, {0.0f, 0.0f, 1.0f}};
        for (int a = 0; a < 3; ++a) {
            projected = dif.x * axes[a][0] + dif.y * axes[a][1] + dif.z * axes[a][2];
            if (projected < -1.0f * side) {
                delta = projected + side;
                dist2 += delta * delta;
            } else if (projected > side) {
                delta = projected - side;
                dist2 += delta * delta;
            }
        }
        fv = wyvill(dist2);
    } break;
    case PSGUI_PRIM_DISC: {
        v3 n = xyz(P->dir), c = xyz(P->pos);
        float r = P->res1[0];
        v3 pc = v3sub(pn, c);
        v3 dir = v3sub(pc, v3scale(n, v3dot(n, pc)));
        float dd;
        if (sqrtf(v3len2(dir)) <= r) {
            dd = Absolutef(v3len2(pc) - v3len2(dir));
        } else {
            v3normalize(&dir);
            v3 x = v3add(c, v3scale(dir, r));
            dd = v3len2(v3sub(x, pn));
        }
        fv = wyvill(dd);
    } break;
    case PSGUI_PRIM_RING: {
        v3 n = xyz(P->dir), c = xyz(P->pos);
        float r = P->res1[0];
        v3 pc = v3sub(pn, c);
        v3 dir = v3sub(pc, v3scale(n, v3dot(n, pc)));
        float dd;
        if (FLOAT_EQ(0.0f, v3len2(dir))) {  /* isZero */
            dd = r * r + v3len2(pc);
        } else {
            v3normalize(&dir);
            v3 x = v3add(c, v3scale(dir, r));
            dd = v3len2(v3sub(x, pn));
        }
        fv = wyvill(dd);
    } break;
    case PSGUI_PRIM_LINE: {
        v3 np = nearest_point_on_segment(pn, xyz(P->res1), xyz(P->res2));
        fv = wyvill(v3dist2(np, pn));
    } break;
    case PSGUI_PRIM_QUADRICPOINT: {
        float d2 = v3len2(v3sub(pn, xyz(P->pos)));
        float R = P->res1[0];
        float f = (1.0f - (d2 / (R * R)));
        fv = (f <= 0.0f) ? 0.0f : P->res2[0] * f * f;
    } break;
    case PSGUI_PRIM_INSTANCE: {  /* :1069-1078 */
        int isOriginOp = P->res1[2] != 0.0f;
        int idxOrigin = (int)P->res1[0];
        v4 myp = {pn.x, pn.y, pn.z, 1.0f};
        fv = isOriginOp ? field_op(T, myp, idxOrigin, 0, 0) : field_prim(T, myp, idxOrigin, 0);
    } break;
    default:  /* Null */
        fv = 0.0f;
        break;
    }
    if (storePrim) storePrim[id] = fv;
    return fv;
}

/* warps (CompactBlobTree.cpp:1315-1536); the results are fresh vec4f (w = 0) */
static v4 warp_bend(v4 pin, float k, float y0, float left, float right) {
    v4 out = {0, 0, 0, 0};
    float kDiv = 1.0f / k;
    float yh = 0.0f;
    if (pin.y <= left) yh = left;
    else if ((pin.y > left) && (pin.y < right)) yh = pin.y;
    else if (pin.y >= right) yh = right;
    float theta = k * (yh - y0);
    float ct = cr_cosf(theta), st = cr_sinf(theta);
    int inside = (pin.y >= left) && (pin.y <= right);
    out.x = pin.x;
    if (inside) out.y = -st * (pin.z - kDiv) + y0;
    else if (pin.y < left) out.y = -st * (pin.z - kDiv) + y0 + ct * (pin.y - left);
    else if (pin.y > right) out.y = -st * (pin.z - kDiv) + y0 + ct * (pin.y - right);
    if (inside) out.z = ct * (pin.z - kDiv) + kDiv;
    else if (pin.y < left) out.z = ct * (pin.z - kDiv) + kDiv + st * (pin.y - left);
    else if (pin.y > right) out.z = ct * (pin.z - kDiv) + kDiv + st * (pin.y - right);
    return out;
}
static v4 warp_twist(v4 pin, float factor, int axis) {
    v4 out = {0, 0, 0, 0};
    float theta;
    switch (axis) {
    case 0:
        theta = pin.x * factor;
        out.x = pin.x;
        out.y = pin.y * cr_cosf(theta) - pin.z * cr_sinf(theta);
        out.z = pin.y * cr_sinf(theta) + pin.z * cr_cosf(theta);
        break;
    case 1:
        theta = pin.y * factor;
        out.x = pin.x * cr_cosf(theta) - pin.z * cr_sinf(theta);
        out.y = pin.y;
        out.z = pin.x * cr_sinf(theta) + pin.z * cr_cosf(theta);
        break;
    case 2:
        theta = pin.z * factor;
        out.x = pin.x * cr_cosf(theta) - pin.y * cr_sinf(theta);
        out.y = pin.x * cr_sinf(theta) + pin.y * cr_cosf(theta);
        out.z = pin.z;
        break;
    }
    return out;
}
static v4 warp_taper(v4 pin, float f, int along, int taper) {
    v4 out = {pin.x, pin.y, pin.z, 0.0f};
    if (along == 0) {  /* taperAlongX: y (default) or z scaled by 1 + x f */
        if (taper == 2) out.z = pin.z * (1 + pin.x * f);
        else out.y = pin.y * (1 + pin.x * f);
    } else if (along == 1) {  /* taperAlongY: x (default) or z */
        if (taper == 2) out.z = pin.z * (1 + pin.y * f);
        else out.x = pin.x * (1 + pin.y * f);
    } else if (along == 2) {  /* taperAlongZ: x (default) or, for zAxis, y */
        if (taper == 2) out.y = pin.y * (1 + pin.z * f);
        else out.x = pin.x * (1 + pin.z * f);
    }
    return out;
}
static v4 warp_shear(v4 pin, float f, int along, int dep) {
    v4 out = {pin.x, pin.y, pin.z, 0.0f};
    if (along == 1) {  /* shearAlongY: + f x (default) or + f z */
        out.y = (dep == 2) ? pin.y + f * pin.z : pin.y + f * pin.x;
    } else if (along == 2) {  /* shearAlongZ: + f x (default) or + f y */
        out.z = (dep == 1) ? pin.z + f * pin.y : pin.z + f * pin.x;
    } else {  /* shearAlongX (and the default): + f y (default) or + f z */
        out.x = (dep == 2) ? pin.x + f * pin.z : pin.x + f * pin.y;
    }
    return out;
}

/* fieldAtNode (:646-652) */
static float field_at_node(const Tree* T, int isOp, int id, v4 p) {
    return isOp ? field_op(T, p, id, 0, 0) : field_prim(T, p, id, 0);
}

/* gradientAtNode (:617-643) */
static v4 gradient_at_node(const Tree* T, int isOp, int id, v4 p, float fp, float delta) {
    float inv = 1.0f / delta;
    v4 a = {p.x + delta, p.y + 0.0f, p.z + 0.0f, p.w + 0.0f};
    v4 b = {p.x + 0.0f, p.y + delta, p.z + 0.0f, p.w + 0.0f};
    v4 c = {p.x + 0.0f, p.y + 0.0f, p.z + delta, p.w + 0.0f};
    v4 res = {field_at_node(T, isOp, id, a), field_at_node(T, isOp, id, b), field_at_node(T, isOp, id, c), 0.0f};
    res.x -= fp; res.y -= fp; res.z -= fp; res.w -= 0.0f;
    res.x *= inv; res.y *= inv; res.z *= inv; res.w *= inv;
    return res;
}

/* marchTowardNode (:572-592); fp is updated in place */
static v3 march_toward_node(const Tree* T, int isOp, int id, v3 p, v3 grad, float* fp) {
    int dir = (*fp < ISO_VALUE) ? 1 : -1;
    int dir2;
    float step = ISO_DISTANCE;
    v3 q = p;
    for (int it = 0; it < PSGUI_PCM_MARCH_MAX && !(((ISO_VALUE - FIELD_VALUE_EPSILON) < *fp) && (*fp < (ISO_VALUE + FIELD_VALUE_EPSILON)));
         ++it) {
        float s = step * (float)dir;
        q.x += grad.x * s; q.y += grad.y * s; q.z += grad.z * s;
        v4 q4 = {q.x, q.y, q.z, 0.0f};
        *fp = field_at_node(T, isOp, id, q4);
        dir2 = (*fp < ISO_VALUE) ? 1 : -1;
        if (dir != dir2) step *= 0.5f;
        dir = dir2;
    }
    return q;
}

/* computePropagationDeformation (:594-614) */
static float propagation_deformation(float dist, float k, float a0, float w) {
    float wh = 0.5f * w;
    float w2 = w * w;
    float w3 = w2 * w;
    if (dist >= 0 && dist < wh) {
        float p1 = (4.0f * (w * k - 4 * a0)) / w3;
        float p2 = (4.0f * (3.0f * a0 - w * k)) / w2;
        float d2 = dist * dist;
        float d3 = dist * d2;
        return p1 * d3 + p2 * d2 + k * dist;
    } else if (dist >= wh && dist < w) {
        return (4 * a0 + (dist - w) * (dist - w) * (4 * dist - w)) / w3;
    }
    return 0.0f;
}

static const float* oct_of(const Tree* T, int isOp, int id, int hi) {
    return isOp ? (hi ? T->O[id].octHi : T->O[id].octLo) : (hi ? T->P[id].octHi : T->P[id].octLo);
}

/* computePCM (:490-570) */
static float compute_pcm(const Tree* T, v4 p, const PsGuiOp* O, int id1, int id2, int isOp1, int isOp2, float fp1,
                         float fp2) {
    PcmCtx* C = T->pcm;
    const float *lo1 = oct_of(T, isOp1, id1, 0), *hi1 = oct_of(T, isOp1, id1, 1);
    const float *lo2 = oct_of(T, isOp2, id2, 0), *hi2 = oct_of(T, isOp2, id2, 1);
    int crossed = !((lo1[0] >= hi2[0]) || (hi1[0] <= lo2[0]) || (lo1[1] >= hi2[1]) || (hi1[1] <= lo2[1]) ||
                    (lo1[2] >= hi2[2]) || (hi1[2] <= lo2[2]));  /* intersects (_GlobalFunctions.h:34-44) */
    if (crossed) {
        if (fp1 >= ISO_VALUE && fp2 >= ISO_VALUE) {
            if (fp1 > fp2) {
                if (C->update && fp2 > C->maxL) C->maxL = fp2;
                return fp1 + (ISO_VALUE - fp2);
            } else {
                if (C->update && fp1 > C->maxR) C->maxR = fp1;
                return fp2 + (ISO_VALUE - fp1);
            }
        } else if (fp1 >= ISO_VALUE && fp2 > FIELD_VALUE_EPSILON) {
            v4 g = gradient_at_node(T, isOp2, id2, p, fp2, NORMAL_DELTA);
            v3 grad = {g.x, g.y, g.z};
            v3 pp = {p.x, p.y, p.z};
            v3 p0 = march_toward_node(T, isOp2, id2, pp, grad, &fp2);
            v4 p00 = {p0.x, p0.y, p0.z, 0.0f};
            v4 g0 = gradient_at_node(T, isOp2, id2, p00, fp2, NORMAL_DELTA);
            float k = sqrtf(g0.x * g0.x + g0.y * g0.y + g0.z * g0.z);
            float a0 = O->params[2] * C->curL;
            v3 d3 = {p0.x - pp.x, p0.y - pp.y, p0.z - pp.z};
            float d = sqrtf(d3.x * d3.x + d3.y * d3.y + d3.z * d3.z);
            return fp1 + propagation_deformation(d, k, a0, O->params[0]);
        } else if (fp2 >= ISO_VALUE && fp1 > FIELD_VALUE_EPSILON) {
            v4 g = gradient_at_node(T, isOp1, id1, p, fp1, NORMAL_DELTA);
            v3 grad = {g.x, g.y, g.z};
            v3 pp = {p.x, p.y, p.z};
            v3 p0 = march_toward_node(T, isOp1, id1, pp, grad, &fp1);
            v4 p00 = {p0.x, p0.y, p0.z, 0.0f};
            v4 g0 = gradient_at_node(T, isOp1, id1, p00, fp1, NORMAL_DELTA);
            float k = sqrtf(g0.x * g0.x + g0.y * g0.y + g0.z * g0.z);
            float a0 = O->params[3] * C->curR;
            v3 d3 = {p0.x - pp.x, p0.y - pp.y, p0.z - pp.z};
            float d = sqrtf(d3.x * d3.x + d3.y * d3.y + d3.z * d3.z);
            return fp2 + propagation_deformation(d, k, a0, O->params[1]);
        }
        return maxf(fp1, fp2);
    }
    return maxf(fp1, fp2);
}

/* COMPACTBLOBTREE::fieldvalueOp (CompactBlobTree.cpp:677-891) */
static float field_op(const Tree* T, v4 p, int id, float* storeOp, float* storePrim) {
    const PsGuiOp* O = &T->O[id];
    float kids[MAX_KIDS];
    float res = 0.0f;
    int n = O->ctKids;
    v4 pw = p;
    if (O->idxMtx != 0) {
        const PsGuiMatrix* m = &T->M[O->idxMtx];
        pw.x = v4dot(m->r[0], p);
        pw.y = v4dot(m->r[1], p);
        pw.z = v4dot(m->r[2], p);
        pw.w = 1.0f;
    }
    if (storeOp) storeOp[id] = 0.0f;
    switch (O->type) {
    case PSGUI_OP_WARPBEND: pw = warp_bend(pw, O->params[0], O->params[1], O->params[2], O->params[3]); break;
    case PSGUI_OP_WARPTWIST: pw = warp_twist(pw, O->params[0], (int)O->params[1]); break;
    case PSGUI_OP_WARPTAPER: pw = warp_taper(pw, O->params[0], (int)O->params[1], (int)O->params[2]); break;
    case PSGUI_OP_WARPSHEAR: pw = warp_shear(pw, O->params[0], (int)O->params[1], (int)O->params[2]); break;
    default: break;
    }
    for (int i = 0; i < n; ++i) {
        uint32_t k = T->K[O->kidStart + i];
        kids[i] = (k >> 16) ? field_op(T, pw, (int)(k & 0xffffu), storeOp, storePrim)
                            : field_prim(T, pw, (int)(k & 0xffffu), storePrim);
    }
    switch (O->type) {
    case PSGUI_OP_PCM:
        if (n == 2) {
            uint32_t k1 = T->K[O->kidStart], k2 = T->K[O->kidStart + 1];
            res = compute_pcm(T, pw, O, (int)(k1 & 0xffffu), (int)(k2 & 0xffffu), (int)(k1 >> 16), (int)(k2 >> 16),
                              kids[0], kids[1]);
        } else {
            return 0.0f;  /* before storing res: the store keeps the 0 written above */
        }
        break;
    case PSGUI_OP_BLEND:
        for (int i = 0; i < n; ++i) res += kids[i];
        break;
    case PSGUI_OP_RICCIBLEND:
        for (int i = 0; i < n; ++i) res += cr_powf(kids[i], O->params[0]);
        res = cr_powf(res, O->params[1]);
        break;
    case PSGUI_OP_UNION:
        res = kids[0];
        for (int i = 1; i < n; ++i)
            if (kids[i] > res) res = kids[i];
        break;
    case PSGUI_OP_INTERSECT:
        res = kids[0];
        for (int i = 1; i < n; ++i)
            if (kids[i] < res) res = kids[i];
        break;
    case PSGUI_OP_DIF:
        res = kids[0];
        for (int i = 1; i < n; ++i) res = (res < (MAX_FIELD_VALUE - kids[i])) ? res : (MAX_FIELD_VALUE - kids[i]);
        break;
    case PSGUI_OP_SMOOTHDIF:
        res = kids[0];
        for (int i = 1; i < n; ++i) res *= (MAX_FIELD_VALUE - kids[i]);
        break;
    default:  /* warps */
        res = kids[0];
        break;
    }
    if (storeOp) storeOp[id] = res;
    return res;
}

/* COMPACTBLOBTREE::fieldvalue (:476-487) */
static float fieldvalue(const Tree* T, v4 p, float* so, float* sp) {
    p.w = 0.0f;
    if (T->nO > 0) return field_op(T, p, 0, so, sp);
    if (T->nP > 0) return field_prim(T, p, 0, sp);
    return 0.0f;
}

/* baseColorOp / baseColorPrim with the stored field values (:1108-1294) */
static v4 color_op(const Tree* T, int id, const float* so, const float* sp);
static v4 color_prim(const Tree* T, int id, const float* so, const float* sp) {
    if (T->P[id].type == PSGUI_PRIM_INSTANCE) {  /* :1110-1118 */
        int idxOrigin = (int)T->P[id].res1[0];
        int isOriginOp = (int)T->P[id].res1[2];
        return isOriginOp ? color_op(T, idxOrigin, so, sp) : color_prim(T, idxOrigin, so, sp);
    }
    v4 c = {T->P[id].color[0], T->P[id].color[1], T->P[id].color[2], T->P[id].color[3]};
    return c;
}
static v4 color_op(const Tree* T, int id, const float* so, const float* sp) {
    const PsGuiOp* O = &T->O[id];
    v4 cl[MAX_KIDS];
    float fv[MAX_KIDS];
    v4 res = {0, 0, 0, 0};
    int n = O->ctKids;
    if (n == 0) return res;
    for (int i = 0; i < n; ++i) {
        uint32_t k = T->K[O->kidStart + i];
        int kid = (int)(k & 0xffffu);
        if (k >> 16) {
            cl[i] = color_op(T, kid, so, sp);
            fv[i] = so[kid];
        } else {
            cl[i] = color_prim(T, kid, so, sp);
            fv[i] = sp[kid];
        }
    }
    int sel = 0;
    float temp;
    switch (O->type) {
    case PSGUI_OP_BLEND:
    case PSGUI_OP_RICCIBLEND: {
        float sum = 0.0f;
        for (int i = 0; i < n; ++i) {
            temp = fv[i];
            res.x += cl[i].x * temp; res.y += cl[i].y * temp; res.z += cl[i].z * temp; res.w += cl[i].w * temp;
            sum += temp;
        }
        if (sum == 0.0f) return cl[0];
        float r = 1.0f / sum;
        res.x *= r; res.y *= r; res.z *= r; res.w *= r;
        return res;
    }
    case PSGUI_OP_PCM:  /* :1191-1200 */
        return (fv[0] > fv[1]) ? cl[0] : cl[1];
    case PSGUI_OP_UNION:
        temp = fv[0];
        for (int i = 1; i < n; ++i)
            if (fv[i] > temp) { temp = fv[i]; sel = i; }
        return cl[sel];
    case PSGUI_OP_INTERSECT:
        temp = fv[0];
        for (int i = 1; i < n; ++i)
            if (fv[i] < temp) { temp = fv[i]; sel = i; }
        return cl[sel];
    case PSGUI_OP_DIF:
    case PSGUI_OP_SMOOTHDIF:
        temp = fv[0];
        for (int i = 1; i < n; ++i) {
            float cur = MAX_FIELD_VALUE - fv[i];
            if (cur < temp) { temp = cur; sel = i; }
        }
        return cl[sel];
    default:  /* warps */
        return cl[0];
    }
}
static v4 base_color(const Tree* T, const float* so, const float* sp) {
    if (T->nO > 0) return color_op(T, 0, so, sp);
    if (T->nP > 0) {  /* m_lpPrims[0].color (:1099-1100) */
        v4 c = {T->P[0].color[0], T->P[0].color[1], T->P[0].color[2], T->P[0].color[3]};
        return c;
    }
    v4 z = {0, 0, 0, 0};
    return z;
}

/* COMPACTBLOBTREE::normal (:433-450) */
static v4 normal_at(const Tree* T, v4 p, float fp, float delta) {
    float inv = -1.0f / delta;
    v4 a = p, b = p, c = p;
    a.x = p.x + delta; a.y = p.y + 0.0f; a.z = p.z + 0.0f;
    b.x = p.x + 0.0f; b.y = p.y + delta; b.z = p.z + 0.0f;
    c.x = p.x + 0.0f; c.y = p.y + 0.0f; c.z = p.z + delta;
    v4 n = {fieldvalue(T, a, 0, 0), fieldvalue(T, b, 0, 0), fieldvalue(T, c, 0, 0), 0.0f};
    n.x -= fp; n.y -= fp; n.z -= fp;
    n.x *= inv; n.y *= inv; n.z *= inv;
    float d = sqrtf(n.x * n.x + n.y * n.y + n.z * n.z);  /* normalizeXYZ */
    if (d > 0) {
        float r = 1.0f / d;
        n.x *= r; n.y *= r; n.z *= r;
    } else {
        n.x = n.y = n.z = 1;
    }
    return n;
}

/* ComputeRootNewtonRaphsonVEC4 (:1581-1622) with fieldValueAndGradient (:452-474) */
static int newton(const Tree* T, float* so, float* sp, v4 p1, v4 p2, float fp1, float fp2, v4* out, float* outF,
                  float target, int iterations) {
    v4 x = (fabsf(fp1 - target) < fabsf(fp2 - target)) ? p1 : p2;
    const float delta = FIELD_VALUE_EPSILON, inv = 1.0f / delta;
    int i;
    for (i = 0; i < iterations; ++i) {
        float fp = fieldvalue(T, x, 0, 0);
        v4 a = x, b = x, c = x;
        a.x = x.x + delta; a.y = x.y + 0.0f; a.z = x.z + 0.0f; a.w = x.w + 0.0f;
        b.x = x.x + 0.0f; b.y = x.y + delta; b.z = x.z + 0.0f; b.w = x.w + 0.0f;
        c.x = x.x + 0.0f; c.y = x.y + 0.0f; c.z = x.z + delta; c.w = x.w + 0.0f;
        v4 g = {fieldvalue(T, a, 0, 0), fieldvalue(T, b, 0, 0), fieldvalue(T, c, 0, 0), 0.0f};
        g.x -= fp; g.y -= fp; g.z -= fp;
        g.x *= inv; g.y *= inv; g.z *= inv;
        g.w = fp;
        float d = target - g.w;
        float gi = 1.0f / (g.x * g.x + g.y * g.y + g.z * g.z + g.w * g.w);
        x.x = x.x + (d * g.x) * gi;
        x.y = x.y + (d * g.y) * gi;
        x.z = x.z + (d * g.z) * gi;
        x.w = x.w + (d * g.w) * gi;
        *outF = fieldvalue(T, x, so, sp);
        *out = x;
        if (fabsf(*outF - target) < FIELD_VALUE_EPSILON) break;
    }
    out->w = 0.0f;
    return (i + 1) * 4;
}

/* ---- CParsipOptimized ------------------------------------------------------ */
typedef struct {
    float* pos;
    float* nrm;
    float* col;
    uint32_t* tri;  /* local vertex ids */
    uint32_t nv, nt, capv, capt;
    PsGuiMpuStats st;
    int processed;
} MpuMesh;

typedef struct { int start[3]; int end[3]; int vid; } EdgeEl;

static int cellid(int i, int j, int k) {  /* CELLID_FROM_IDX (CPolyParsipOptimized.h:54) */
    const int m = GRID_DIM - 1;  /* CELLID_BITMASK */
    return ((k & m) << (2 * CELLID_SHIFT)) | ((j & m) << CELLID_SHIFT) | (i & m);
}

int psgui_set_grid_dim(int g) {
    if (g != 8 && g != 16 && g != 32) return -1;
    GRID_DIM = g;
    CELLID_SHIFT = g == 8 ? 3 : (g == 16 ? 4 : 5);
    return 1;
}

typedef struct {
    EdgeEl tab[2 * CELLID_HASHSIZE][EDGETABLE_DEPTH];
    int sizes[2 * CELLID_HASHSIZE];
} EdgeTable;

static void order_edge(int* s, int* e) {  /* getEdge/setEdge canonical order (:57-66) */
    if (s[0] > e[0] || (s[0] == e[0] && (s[1] > e[1] || (s[1] == e[1] && s[2] > e[2])))) {
        for (int a = 0; a < 3; ++a) { int t = s[a]; s[a] = e[a]; e[a] = t; }
    }
}
static int get_edge(const EdgeTable* E, const int* s0, const int* e0) {  /* :48-81 */
    int s[3] = {s0[0], s0[1], s0[2]}, e[3] = {e0[0], e0[1], e0[2]};
    order_edge(s, e);
    int h = cellid(s[0], s[1], s[2]) + cellid(e[0], e[1], e[2]);
    for (int q = 0; q < E->sizes[h]; ++q) {
        const EdgeEl* x = &E->tab[h][q];
        if (!memcmp(x->start, s, sizeof(s)) && !memcmp(x->end, e, sizeof(e))) return x->vid;
    }
    return -1;
}
static void set_edge(EdgeTable* E, const int* s0, const int* e0, int vid) {  /* :83-115 */
    int s[3] = {s0[0], s0[1], s0[2]}, e[3] = {e0[0], e0[1], e0[2]};
    order_edge(s, e);
    int h = cellid(s[0], s[1], s[2]) + cellid(e[0], e[1], e[2]);
    int q = E->sizes[h];
    if (q >= EDGETABLE_DEPTH) return;  /* "table is full" */
    E->sizes[h] = q + 1;
    memcpy(E->tab[h][q].start, s, sizeof(s));
    memcpy(E->tab[h][q].end, e, sizeof(e));
    E->tab[h][q].vid = vid;
}

static void push_vertex(MpuMesh* m, v4 p, v4 n, v4 c) {
    if (m->nv == m->capv) {
        m->capv = m->capv ? 2 * m->capv : 256;
        m->pos = realloc(m->pos, (size_t)m->capv * 12);
        m->nrm = realloc(m->nrm, (size_t)m->capv * 12);
        m->col = realloc(m->col, (size_t)m->capv * 16);
    }
    float* P = m->pos + 3 * m->nv;
    float* N = m->nrm + 3 * m->nv;
    float* C = m->col + 4 * m->nv;
    P[0] = p.x; P[1] = p.y; P[2] = p.z;
    N[0] = n.x; N[1] = n.y; N[2] = n.z;
    C[0] = c.x; C[1] = c.y; C[2] = c.z; C[3] = c.w;
    m->nv++;
}
static void push_tri(MpuMesh* m, int a, int b, int c) {
    if (m->nt == m->capt) {
        m->capt = m->capt ? 2 * m->capt : 256;
        m->tri = realloc(m->tri, (size_t)m->capt * 12);
    }
    m->tri[3 * m->nt] = (uint32_t)a;
    m->tri[3 * m->nt + 1] = (uint32_t)b;
    m->tri[3 * m->nt + 2] = (uint32_t)c;
    m->nt++;
}

static const int corner1[12] = {0, 2, 0, 1, 4, 6, 4, 5, 0, 1, 2, 3};  /* CCubeTable.h:43 */
static const int corner2[12] = {1, 3, 2, 3, 5, 7, 6, 7, 4, 5, 6, 7};  /* CCubeTable.h:44 */

/* CSIMDMPURunBody::doMarchingCubes (CPolyParsipOptimized.cpp:130-327) */
static void do_marching_cubes(const Tree* T, const int32_t* tri, v3 origin, float cs, float iso, MpuMesh* out,
                              EdgeTable* E, float* cache, float* so, float* sp) {
    memset(out, 0, sizeof(*out));
    const int nCache = GRID_DIM * GRID_DIM * GRID_DIM;
    memset(E->sizes, 0, sizeof(int) * 2 * (size_t)nCache);
    for (int i = 0; i < nCache; ++i) cache[i] = 1.17549435e-38f;  /* FLT_MIN: "not set" */
    v4 org = {origin.x, origin.y, origin.z, 0.0f};
    float side = (float)(GRID_DIM - 1) * cs;
    v4 hi = {org.x + side, org.y + side, org.z + side, org.w + side};
    int any = 0;
    for (uint32_t i = 0; i < T->nP && !any; ++i) {  /* intersects (:117-127) */
        const PsGuiPrim* P = &T->P[i];
        if ((P->octLo[0] >= hi.x) || (P->octHi[0] <= org.x)) continue;
        if ((P->octLo[1] >= hi.y) || (P->octHi[1] <= org.y)) continue;
        if ((P->octLo[2] >= hi.z) || (P->octHi[2] <= org.z)) continue;
        any = 1;
    }
    if (!any) return;
    out->processed = 1;
    uint32_t evals = 0, cells = 0;
    for (int i = 0; i < CELLS; ++i)
        for (int j = 0; j < CELLS; ++j)
            for (int k = 0; k < CELLS; ++k) {
                int idx[8][3];
                int key[8];
                v4 pos[8];
                float fld[8];
                int cfg = 0;
                for (int c = 0; c < 8; ++c) {
                    int ci = i + ((c >> 2) & 1), cj = j + ((c >> 1) & 1), ck = k + (c & 1);
                    idx[c][0] = ci; idx[c][1] = cj; idx[c][2] = ck;
                    key[c] = cellid(ci, cj, ck);
                    pos[c].x = org.x + cs * (float)ci;
                    pos[c].y = org.y + cs * (float)cj;
                    pos[c].z = org.z + cs * (float)ck;
                    pos[c].w = org.w + 0.0f;
                    float f = cache[key[c]];
                    if (f == 1.17549435e-38f) {
                        evals++;
                        f = fieldvalue(T, pos[c], 0, 0);
                        cache[key[c]] = f;
                    }
                    fld[c] = f;
                    if (f > iso) cfg += (1 << c);
                }
                (void)fld;
                if (cfg == 0 || cfg == 255) continue;
                cells++;
                int cand[16], vids[16], ct = 0;
                for (int q = 0; q < 16; ++q) {
                    cand[q] = tri[cfg * 16 + q];
                    if (cand[q] != -1) ct++;
                }
                for (int q = 0; q < ct; ++q) {
                    int a = corner1[cand[q]], b = corner2[cand[q]];
                    vids[q] = get_edge(E, idx[a], idx[b]);
                    if (vids[q] == -1) {
                        v4 p;
                        float fp = 0.0f;
                        evals += (uint32_t)newton(T, so, sp, pos[a], pos[b], cache[key[a]], cache[key[b]], &p, &fp, iso,
                                                  PSGUI_ITERATIONS);
                        evals += 3;
                        v4 n = normal_at(T, p, fp, NORMAL_DELTA);
                        v4 col = base_color(T, so, sp);
                        push_vertex(out, p, n, col);
                        vids[q] = (int)out->nv - 1;
                        set_edge(E, idx[a], idx[b], vids[q]);
                    }
                }
                for (int q = 0; q < ct / 3; ++q) push_tri(out, vids[3 * q], vids[3 * q + 1], vids[3 * q + 2]);
            }
    out->st.fieldEvals = evals;
    out->st.intersectedCells = cells;
    out->st.ctVertices = out->nv;
    out->st.ctTriangles = out->nt;
}

typedef struct {
    PsGuiInfo info;
    MpuMesh* mpus;
} Result;

typedef struct {
    const Tree* T;
    PcmCtx pcm;  /* this thread's copy of the contact state */
    const int32_t* tri;
    const float* lo;
    float cs, iso, side;
    uint32_t dims[3];
    Result* R;
    uint32_t begin, end;
} Job;

static void* run_job(void* arg) {
    Job* J = (Job*)arg;
    Tree TT = *J->T;
    TT.pcm = &J->pcm;
    EdgeTable* E = malloc(sizeof(EdgeTable));
    float* cache = malloc(sizeof(float) * MAX_GRID * MAX_GRID * MAX_GRID);
    float* so = calloc(J->T->nO + 1, sizeof(float));
    float* sp = calloc(J->T->nP + 1, sizeof(float));
    for (uint32_t m = J->begin; m < J->end; ++m) {
        uint32_t k = m % J->dims[2], j = (m / J->dims[2]) % J->dims[1], i = m / (J->dims[2] * J->dims[1]);
        v3 o = {J->lo[0] + (float)i * J->side, J->lo[1] + (float)j * J->side, J->lo[2] + (float)k * J->side};
        do_marching_cubes(&TT, J->tri, o, J->cs, J->iso, &J->R->mpus[m], E, cache, so, sp);
    }
    free(so);
    free(sp);
    free(E);
    free(cache);
    return NULL;
}

/* CParsipOptimized::setup + run (:330-410).  *out: a Result for psgui_result_*.  pcmState
 * (may be NULL: ISO_VALUE, not returned): the contact state the run reads, replaced by the
 * state it leaves. */
int psgui_polygonize(const PsGuiPrim* prims, uint32_t nP, const PsGuiOp* ops, uint32_t nO, const uint32_t* kids,
                     const PsGuiMatrix* mtx, const float lo[3], const float hi[3], float cs, float iso,
                     const int32_t* tri, int threads, void** out, float* pcmState) {
    Tree T = {prims, nP, ops, nO, kids, mtx, 0};
    const float curL = pcmState ? pcmState[0] : ISO_VALUE, curR = pcmState ? pcmState[1] : ISO_VALUE;
    Result* R = calloc(1, sizeof(Result));
    int cells[3];
    for (int a = 0; a < 3; ++a) {
        float sideA = hi[a] - lo[a];
        cells[a] = (int)ceilf(sideA / cs);
        R->info.dims[a] = (uint32_t)(cells[a] / CELLS + (cells[a] % CELLS != 0 ? 1 : 0));
    }
    uint32_t N = R->info.dims[0] * R->info.dims[1] * R->info.dims[2];
    R->info.ctLatticeMPUs = N;
    R->mpus = calloc(N ? N : 1, sizeof(MpuMesh));
    if (threads < 1) threads = 1;
    pthread_t th[64];
    Job jobs[64];
    if (threads > 64) threads = 64;
    for (int t = 0; t < threads; ++t) {
        Job J = {&T, {curL, curR, curL, curR, 1}, tri, lo, cs, iso, (float)CELLS * cs,
                 {R->info.dims[0], R->info.dims[1], R->info.dims[2]}, R,
                 (uint32_t)((uint64_t)N * t / threads), (uint32_t)((uint64_t)N * (t + 1) / threads)};
        jobs[t] = J;
        pthread_create(&th[t], NULL, run_job, &jobs[t]);
    }
    for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
    if (pcmState) {  /* maxima: the thread split does not matter */
        float mL = curL, mR = curR;
        for (int t = 0; t < threads; ++t) {
            if (jobs[t].pcm.maxL > mL) mL = jobs[t].pcm.maxL;
            if (jobs[t].pcm.maxR > mR) mR = jobs[t].pcm.maxR;
        }
        pcmState[0] = mL;
        pcmState[1] = mR;
    }
    for (uint32_t m = 0; m < N; ++m) {
        MpuMesh* M = &R->mpus[m];
        R->info.ctFieldEvals += M->st.fieldEvals;
        R->info.ctIntersectedCells += M->st.intersectedCells;
        R->info.ctVertices += M->nv;
        R->info.ctTriangles += M->nt;
        R->info.ctProcessedMPUs += (uint32_t)M->processed;
        if (M->nt > 0) R->info.ctIntersectedMPUs++;
    }
    /* removeExtraPUs (:573-592): MPUs without faces go whenever run() counted any */
    R->info.ctMPUs = R->info.ctIntersectedMPUs < N ? R->info.ctIntersectedMPUs : N;
    R->info.ctCellsInIntersectedMPUs = (uint64_t)CELLS * CELLS * CELLS * R->info.ctIntersectedMPUs;
    *out = R;
    return 1;
}

void psgui_result_info(void* r, PsGuiInfo* info) { *info = ((Result*)r)->info; }

/* exportMesh order: lattice order, triangle ids made mesh-wide */
void psgui_result_copy(void* r, float* pos, float* nrm, float* col, uint32_t* tris, uint64_t* offs,
                       PsGuiMpuStats* stats) {
    Result* R = (Result*)r;
    uint32_t V = 0, T = 0;
    for (uint32_t m = 0; m < R->info.ctLatticeMPUs; ++m) {
        MpuMesh* M = &R->mpus[m];
        if (offs) offs[m] = (uint64_t)V | ((uint64_t)T << 32);
        if (stats) stats[m] = M->st;
        if (pos) memcpy(pos + 3 * (size_t)V, M->pos, (size_t)M->nv * 12);
        if (nrm) memcpy(nrm + 3 * (size_t)V, M->nrm, (size_t)M->nv * 12);
        if (col) memcpy(col + 4 * (size_t)V, M->col, (size_t)M->nv * 16);
        if (tris)
            for (uint32_t t = 0; t < 3 * M->nt; ++t) tris[3 * (size_t)T + t] = M->tri[t] + V;
        V += M->nv;
        T += M->nt;
    }
    if (offs) offs[R->info.ctLatticeMPUs] = (uint64_t)V | ((uint64_t)T << 32);
}

void psgui_result_free(void* r) {
    Result* R = (Result*)r;
    for (uint32_t m = 0; m < R->info.ctLatticeMPUs; ++m) {
        free(R->mpus[m].pos);
        free(R->mpus[m].nrm);
        free(R->mpus[m].col);
        free(R->mpus[m].tri);
    }
    free(R->mpus);
    free(R);
}

/* fieldvalue + baseColor at n points (baseColor over the values stored by that walk) */
void psgui_field_values(const PsGuiPrim* prims, uint32_t nP, const PsGuiOp* ops, uint32_t nO, const uint32_t* kids,
                        const PsGuiMatrix* mtx, const float* xyz3, uint32_t n, float* out, float* col4,
                        const float* pcmState) {
    PcmCtx C = {pcmState ? pcmState[0] : ISO_VALUE, pcmState ? pcmState[1] : ISO_VALUE, 0.0f, 0.0f, 0};
    Tree T = {prims, nP, ops, nO, kids, mtx, &C};
    float* so = calloc(nO + 1, sizeof(float));
    float* sp = calloc(nP + 1, sizeof(float));
    for (uint32_t i = 0; i < n; ++i) {
        v4 p = {xyz3[3 * i], xyz3[3 * i + 1], xyz3[3 * i + 2], 0.0f};
        out[i] = fieldvalue(&T, p, so, sp);
        if (col4) {
            v4 c = base_color(&T, so, sp);
            col4[4 * i] = c.x; col4[4 * i + 1] = c.y; col4[4 * i + 2] = c.z; col4[4 * i + 3] = c.w;
        }
    }
    free(so);
    free(sp);
}

/* glibc's own powf / cosf / sinf against cr_*: counts of differing results and the largest
 * difference in ulps (tests only) */
static uint32_t ulps(float a, float b) {
    int32_t ia, ib;
    memcpy(&ia, &a, 4);
    memcpy(&ib, &b, 4);
    if (ia < 0) ia = (int32_t)0x80000000 - ia;
    if (ib < 0) ib = (int32_t)0x80000000 - ib;
    return (uint32_t)(ia > ib ? ia - ib : ib - ia);
}
void psgui_libm_agreement(const float* x, const float* y, uint32_t n, uint32_t* diff, uint32_t* maxUlp) {
    for (int k = 0; k < 3; ++k) diff[k] = maxUlp[k] = 0;
    for (uint32_t i = 0; i < n; ++i) {
        float a[3] = {powf(x[i], y[i]), cosf(x[i]), sinf(x[i])};
        float b[3] = {cr_powf(x[i], y[i]), cr_cosf(x[i]), cr_sinf(x[i])};
        for (int k = 0; k < 3; ++k) {
            uint32_t u = ulps(a[k], b[k]);
            if (u) diff[k]++;
            if (u > maxUlp[k]) maxUlp[k] = u;
        }
    }
}

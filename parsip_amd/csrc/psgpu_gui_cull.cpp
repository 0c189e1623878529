// psgpu_gui_cull.cpp -- compat mode: world-space boxes outside which a primitive's field, and
// an operator subtree's value, is exactly +0 (exact culling of the compact walk).
//
// A primitive sees the point through the operator matrices above it and its own matrix
// (psgpu_gui_device.h: op_point_k -- the first operator matrix from the root acts on w = 0,
// so only its linear part applies; later ones act on w = 1 -- and prim_field_k with w = 1).
// Its field is non-zero only inside a local support box (Wyvill: squared distance < 1 to the
// skeleton; QuadricPoint: d^2 < R^2; Null: nowhere); the world box is that box mapped back
// through the composed affine map (double precision), widened by a margin far above the
// float rounding of the device's transform chain.  Anything the bound cannot cover exactly
// (warps above the primitive, singular or ill-conditioned maps, non-unit axes, non-finite
// parameters) gets an infinite box: always evaluated.
//
// An operator's box is the union of its kids' boxes.  Its value with every kid at +0 is +0
// for Union, Intersect, Dif, SmoothDif, Blend and Ricci with positive exponents
// (pow(+0, y > 0) = +0), and its colour then is its first kid's (first-kid chain down to a
// primitive): the generated walk substitutes both when no lane of the wave is in the box.
#include <cmath>
#include <limits>
#include <vector>

#include "psgpu_gui_jit.h"

namespace psgui {
namespace {

constexpr double kInf = std::numeric_limits<double>::infinity();

struct Affine {  // q = L p + t
    double L[3][3], t[3];
};

Affine identity() {
    Affine a{};
    for (int i = 0; i < 3; ++i) a.L[i][i] = 1.0;
    return a;
}

// m applied after a (rows of the backward matrix; `linear`: the w = 0 case, no translation)
Affine compose(const PsGuiMatrix& m, const Affine& a, bool linear) {
    Affine r{};
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) {
            double s = 0.0;
            for (int k = 0; k < 3; ++k) s += (double)m.r[i][k] * a.L[k][j];
            r.L[i][j] = s;
        }
        double s = linear ? 0.0 : (double)m.r[i][3];
        for (int k = 0; k < 3; ++k) s += (double)m.r[i][k] * a.t[k];
        r.t[i] = s;
    }
    return r;
}

struct Box {
    double lo[3], hi[3];
};

Box infinite() { return Box{{-kInf, -kInf, -kInf}, {kInf, kInf, kInf}}; }
Box empty() { return Box{{kInf, kInf, kInf}, {-kInf, -kInf, -kInf}}; }
bool is_infinite(const Box& b) { return std::isinf(b.lo[0]) && b.lo[0] < 0; }

Box around(const double c[3], double r) {
    return Box{{c[0] - r, c[1] - r, c[2] - r}, {c[0] + r, c[1] + r, c[2] + r}};
}
Box segment(const double a[3], const double b[3], double r) {
    Box x;
    for (int i = 0; i < 3; ++i) {
        x.lo[i] = std::fmin(a[i], b[i]) - r;
        x.hi[i] = std::fmax(a[i], b[i]) + r;
    }
    return x;
}
void join(Box& a, const Box& b) {
    for (int i = 0; i < 3; ++i) {
        a.lo[i] = std::fmin(a.lo[i], b.lo[i]);
        a.hi[i] = std::fmax(a.hi[i], b.hi[i]);
    }
}

bool finite4(const float* v) {
    return std::isfinite(v[0]) && std::isfinite(v[1]) && std::isfinite(v[2]) && std::isfinite(v[3]);
}
bool unit(const float* d) {
    const double n = std::sqrt((double)d[0] * d[0] + (double)d[1] * d[1] + (double)d[2] * d[2]);
    return std::fabs(n - 1.0) < 1e-5;
}

// local support box of prim_field_k (psgpu_gui_device.h), margin included
bool local_box(const PsGuiPrim& P, Box& b) {
    if (P.type == PSGUI_PRIM_NULL) {  // the default case: 0 everywhere
        b = empty();
        return true;
    }
    if (!finite4(P.pos) || !finite4(P.dir) || !finite4(P.res1) || !finite4(P.res2)) return false;
    const double pos[3] = {P.pos[0], P.pos[1], P.pos[2]};
    const double r1[3] = {P.res1[0], P.res1[1], P.res1[2]};
    const double r2[3] = {P.res2[0], P.res2[1], P.res2[2]};
    switch (P.type) {
    case PSGUI_PRIM_POINT:
        b = around(pos, 1.0);
        break;
    case PSGUI_PRIM_CYLINDER: {  // radial < r + 1, axial in (-1, h + 1), unit axis
        if (!unit(P.dir) || !(r1[0] >= 0.0)) return false;
        const double h = std::fmax(r2[0], 0.0);
        const double a[3] = {pos[0] - P.dir[0], pos[1] - P.dir[1], pos[2] - P.dir[2]};
        const double e[3] = {pos[0] + (h + 1.0) * P.dir[0], pos[1] + (h + 1.0) * P.dir[1], pos[2] + (h + 1.0) * P.dir[2]};
        b = segment(a, e, r1[0] + 1.0);
        break;
    }
    case PSGUI_PRIM_TRIANGLE:
        b = segment(pos, r1, 1.0);
        join(b, segment(r2, r2, 1.0));
        break;
    case PSGUI_PRIM_CUBE:
        b = around(pos, std::fabs(r1[0]) + 1.0);
        break;
    case PSGUI_PRIM_DISC:
    case PSGUI_PRIM_RING:  // within r + 1 of the centre (unit normal; an in-plane direction
        // of length 0 normalises to (1, 1, 1): within |r| sqrt(3) + 1)
        if (!unit(P.dir)) return false;
        b = around(pos, std::fabs(r1[0]) * 1.7320508075688772 + 1.0);
        break;
    case PSGUI_PRIM_LINE:
        b = segment(r1, r2, 1.0);
        break;
    case PSGUI_PRIM_QUADRICPOINT:  // f = 1 - d^2 / R^2 > 0
        if (!(std::fabs(r1[0]) > 1e-6)) return false;
        b = around(pos, std::fabs(r1[0]));
        break;
    default:
        return false;
    }
    for (int i = 0; i < 3; ++i) {  // relative + absolute margin over the float evaluation
        const double m = 1e-3 * (1.0 + std::fmax(std::fabs(b.lo[i]), std::fabs(b.hi[i])));
        b.lo[i] -= m;
        b.hi[i] += m;
    }
    return true;
}

// the world points p with a.L p + a.t inside the local box
bool world_box(const Affine& a, const Box& local, Box& out) {
    if (std::isinf(local.lo[0]) && local.lo[0] > 0) {  // empty: nowhere non-zero
        out = empty();
        return true;
    }
    const double (*L)[3] = a.L;
    const double det = L[0][0] * (L[1][1] * L[2][2] - L[1][2] * L[2][1]) - L[0][1] * (L[1][0] * L[2][2] - L[1][2] * L[2][0]) +
                       L[0][2] * (L[1][0] * L[2][1] - L[1][1] * L[2][0]);
    double nrm = 0.0;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) nrm = std::fmax(nrm, std::fabs(L[i][j]));
    if (!std::isfinite(det) || std::fabs(det) < 1e-9 * nrm * nrm * nrm || nrm == 0.0) return false;
    double inv[3][3];
    inv[0][0] = (L[1][1] * L[2][2] - L[1][2] * L[2][1]) / det;
    inv[0][1] = (L[0][2] * L[2][1] - L[0][1] * L[2][2]) / det;
    inv[0][2] = (L[0][1] * L[1][2] - L[0][2] * L[1][1]) / det;
    inv[1][0] = (L[1][2] * L[2][0] - L[1][0] * L[2][2]) / det;
    inv[1][1] = (L[0][0] * L[2][2] - L[0][2] * L[2][0]) / det;
    inv[1][2] = (L[0][2] * L[1][0] - L[0][0] * L[1][2]) / det;
    inv[2][0] = (L[1][0] * L[2][1] - L[1][1] * L[2][0]) / det;
    inv[2][1] = (L[0][1] * L[2][0] - L[0][0] * L[2][1]) / det;
    inv[2][2] = (L[0][0] * L[1][1] - L[0][1] * L[1][0]) / det;
    double inorm = 0.0;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) inorm = std::fmax(inorm, std::fabs(inv[i][j]));
    if (nrm * inorm > 1e6) return false;  // ill-conditioned: rounding could move the boundary
    out = empty();
    for (int c = 0; c < 8; ++c) {
        const double q[3] = {(c & 1) ? local.hi[0] : local.lo[0], (c & 2) ? local.hi[1] : local.lo[1],
                             (c & 4) ? local.hi[2] : local.lo[2]};
        double p[3];
        for (int i = 0; i < 3; ++i)
            p[i] = inv[i][0] * (q[0] - a.t[0]) + inv[i][1] * (q[1] - a.t[1]) + inv[i][2] * (q[2] - a.t[2]);
        join(out, Box{{p[0], p[1], p[2]}, {p[0], p[1], p[2]}});
    }
    for (int i = 0; i < 3; ++i) {
        const double m = 1e-3 * (1.0 + std::fmax(std::fabs(out.lo[i]), std::fabs(out.hi[i])));
        out.lo[i] -= m;
        out.hi[i] += m;
    }
    return std::isfinite(out.lo[0]) && std::isfinite(out.hi[0]) && std::isfinite(out.lo[1]) &&
           std::isfinite(out.hi[1]) && std::isfinite(out.lo[2]) && std::isfinite(out.hi[2]);
}

bool zero_preserving(const PsGuiOp& O) {
    switch (O.type) {
    case PSGUI_OP_UNION:
    case PSGUI_OP_INTERSECT:
    case PSGUI_OP_DIF:
    case PSGUI_OP_SMOOTHDIF:
    case PSGUI_OP_BLEND:
        return true;
    case PSGUI_OP_RICCIBLEND:
        return O.params[0] > 0.0f && O.params[1] > 0.0f;
    default:
        return false;  // warps: the point changes below them
    }
}

struct Walker {
    const PsGuiPrim* P;
    const PsGuiOp* O;
    const uint32_t* K;
    const PsGuiMatrix* M;
    uint32_t nM;
    std::vector<Box> prim, op;

    Box visit(uint32_t o, const Affine& a, bool w1, bool warped) {
        const PsGuiOp& Op = O[o];
        Affine here = a;
        bool hereW1 = w1;
        if (Op.idxMtx != 0 && Op.idxMtx < nM) {
            here = compose(M[Op.idxMtx], a, !w1);
            hereW1 = true;
        }
        const bool isWarp = !zero_preserving(Op) && Op.type != PSGUI_OP_RICCIBLEND;
        const bool below = warped || isWarp;
        Box u = empty();
        bool anyInf = false;
        for (int i = 0; i < Op.ctKids; ++i) {
            const uint32_t k = K[Op.kidStart + i];
            const uint32_t id = k & 0xffffu;
            Box b;
            if (k >> 16) {
                b = visit(id, here, hereW1, below);
            } else {
                const PsGuiPrim& Pr = P[id];
                Box local;
                bool ok = !below && local_box(Pr, local);
                if (ok) {
                    const Affine full = (Pr.idxMtx != 0 && Pr.idxMtx < nM) ? compose(M[Pr.idxMtx], here, false) : here;
                    ok = world_box(full, local, b);
                }
                if (!ok) b = infinite();
                prim[id] = b;
            }
            if (is_infinite(b)) anyInf = true;
            else join(u, b);
        }
        Box ob = (anyInf || below || !zero_preserving(Op)) ? infinite() : u;
        op[o] = ob;
        return ob;
    }
};

void put(float* out, const Box& b) {
    for (int i = 0; i < 3; ++i) {
        out[i] = (float)b.lo[i];
        out[4 + i] = (float)b.hi[i];
        // rounding to float must not shrink the box
        if ((double)out[i] > b.lo[i]) out[i] = std::nextafter(out[i], -std::numeric_limits<float>::infinity());
        if ((double)out[4 + i] < b.hi[i]) out[4 + i] = std::nextafter(out[4 + i], std::numeric_limits<float>::infinity());
    }
    out[3] = out[7] = 0.0f;
}

}  // namespace

void cull_boxes(const PsGuiPrim* P, uint32_t nP, const PsGuiOp* O, uint32_t nO, const uint32_t* K,
                const PsGuiMatrix* M, uint32_t nM, std::vector<float>& primBoxes, std::vector<float>& opBoxes) {
    Walker w{P, O, K, M, nM, std::vector<Box>(nP, infinite()), std::vector<Box>(nO, infinite())};
    if (nO == 0) {
        for (uint32_t i = 0; i < nP; ++i) {  // a lone primitive: the root point, w = 0 (prim matrix: w = 1)
            Box local, b;
            bool ok = local_box(P[i], local);
            if (ok) ok = world_box(P[i].idxMtx != 0 && P[i].idxMtx < nM ? compose(M[P[i].idxMtx], identity(), false)
                                                                        : identity(),
                                   local, b);
            w.prim[i] = ok ? b : infinite();
        }
    } else {
        w.visit(0, identity(), false, false);
    }
    primBoxes.assign(8 * (size_t)std::max<uint32_t>(nP, 1), 0.0f);
    opBoxes.assign(8 * (size_t)std::max<uint32_t>(nO, 1), 0.0f);
    for (uint32_t i = 0; i < nP; ++i) put(&primBoxes[8 * i], w.prim[i]);
    for (uint32_t i = 0; i < nO; ++i) put(&opBoxes[8 * i], w.op[i]);
}

}  // namespace psgui

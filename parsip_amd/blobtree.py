"""BlobTree model API and its linearizer into the polygonizer's SoA.

Mirrors the reference's PS_BlobTree node classes (Parsip100/PS_BlobTree/include/*.h:
node types from _constSettings.h:26-38, skeletons with their loadScript fields,
CAffineTransformation from PS_FrameWork/include/PS_AffineTransformation.h) and
``SimdPoly::linearizeBlobTree`` (Parsip100/ParsipHaptics/include/
PS_HighPerformanceRender.cpp:42-371):

* pre-order ids: an operator takes the next op id before its children are visited,
  primitives are numbered in visiting order, the root op is 0 (:68-96, :163-166);
* ``opChildKind = isOpLeft * 2 + isOpRight`` (:93);
* only binary operators (-3, PS_ERROR_NON_BINARY_OP), at most 128 prims (-1) / ops (-2);
* node boxes from the node's octree (:47-50, :97-107, :176-187);
* a non-identity backward matrix goes to the next SOABlobPrimMatrices slot, rows 0-2
  in the 12-float stride (:194-214); identity -> idxMatrix 0;
* per-type parameter packing (:218-349) including RicciBlend resY = 1/n and the
  Triangle adapter bug (p2.z overwrites resX; ``triangle_compat=True`` keeps it).

Node type codes: the reference writes raw ``getNodeType()`` (BlobTree enum) into the
SoA although the SIMD path switches on the PS_Polygonizer.h enum;
``linearize_blobtree`` translates by default (``raw_types=True`` reproduces the
reference's bytes).

Matrices are restated in fp32 exactly as CMatrix does them (PS_Matrix.h:124-145,
416-446, 548-604; CQuaternion::toMatrix PS_Quaternion.h:368-394).  Node boxes are the
octrees ParsipHaptics computes after loading a model (CLayer::recursive_RecomputeAllOctrees,
CLayerManager.cpp:629-646: skeleton bounds, two corners through the accumulated forward
matrix, per-operator union / first child / intersection / warp growth), restated in fp32
(``compute_octrees_reference``); ``octrees="aabb"`` uses conservative world AABBs instead.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from enum import IntEnum

import numpy as np

from . import soa
from .soa import NodeType

_F = np.float32
PS_ERROR_PRIM_OVERFLOW = -1
PS_ERROR_OPERATOR_OVERFLOW = -2
PS_ERROR_NON_BINARY_OP = -3
EPSILON = _F(0.0001)  # mathHelper.h:28


class BlobNodeType(IntEnum):
    """_constSettings.h:26-38 (the caller-side BlobTree enum)."""

    PRIM_POINT = 0
    PRIM_LINE = 1
    PRIM_CYLINDER = 2
    PRIM_DISC = 3
    PRIM_RING = 4
    PRIM_POLYGON = 5
    PRIM_CUBE = 6
    PRIM_TRIANGLE = 7
    PRIM_CATMULLROM = 8
    PRIM_SKELETON = 9
    PRIM_QUADRICPOINT = 10
    PRIM_HALFPLANE = 11
    PRIM_NULL = 12
    PRIM_INSTANCE = 13
    OP_UNION = 14
    OP_INTERSECT = 15
    OP_DIF = 16
    OP_SMOOTHDIF = 17
    OP_BLEND = 18
    OP_RICCIBLEND = 19
    OP_GRADIENTBLEND = 20
    OP_FASTQPS = 21
    OP_PCM = 22
    OP_CACHE = 23
    OP_WARPTWIST = 24
    OP_WARPTAPER = 25
    OP_WARPBEND = 26
    OP_WARPSHEAR = 27
    OP_TEXTURE = 28


# ---------------------------------------------------------------------------
# CMatrix (mElement[col][row], row vectors: p' = p * M) in fp32
class Matrix:
    def __init__(self, m=None):
        self.e = np.eye(4, dtype=np.float32) if m is None else np.array(m, np.float32).reshape(4, 4)

    def copy(self) -> "Matrix":
        return Matrix(self.e.copy())

    @staticmethod
    def product(a: "Matrix", b: "Matrix") -> "Matrix":
        """CMatrix::multiply(t1, t2) (PS_Matrix.h:132-145): M[i][j] = sum_k A[i][k] B[k][j]."""
        out = np.zeros((4, 4), np.float32)
        for i in range(4):
            for j in range(4):
                acc = _F(0.0)
                for k in range(4):
                    acc = _F(acc + _F(a.e[i, k] * b.e[k, j]))
                out[i, j] = acc
        return Matrix(out)

    def set_scale(self, s) -> None:  # :421-433
        w = Matrix()
        w.e[0, 0], w.e[1, 1], w.e[2, 2] = _F(s[0]), _F(s[1]), _F(s[2])
        self.e = Matrix.product(self, w).e

    def set_translate(self, t) -> None:  # :441-446
        self.e[3, 0], self.e[3, 1], self.e[3, 2] = _F(t[0]), _F(t[1]), _F(t[2])

    def multiply(self, rhs: "Matrix") -> None:  # :124-129
        self.e = Matrix.product(self, rhs).e

    def is_identity(self) -> bool:
        return bool(np.array_equal(self.e, np.eye(4, dtype=np.float32)))

    def determinant(self) -> np.float32:
        """getDeterminant (:573-584): p0 . (p1 x p2) over the upper 3x3."""
        p0, p1, p2 = self.e[0, :3], self.e[1, :3], self.e[2, :3]
        cx = _F(_F(p1[1] * p2[2]) - _F(p1[2] * p2[1]))
        cy = _F(_F(p1[2] * p2[0]) - _F(p1[0] * p2[2]))
        cz = _F(_F(p1[0] * p2[1]) - _F(p1[1] * p2[0]))
        return _F(_F(_F(p0[0] * cx) + _F(p0[1] * cy)) + _F(p0[2] * cz))

    def submatrix(self, ki: int, kj: int) -> "Matrix":  # :548-570
        dst = Matrix()
        dc = 0
        for col in range(4):
            if col == kj:
                continue
            dr = 0
            for row in range(4):
                if row == ki:
                    continue
                dst.e[dc, dr] = self.e[col, row]
                dr += 1
            dc += 1
        return dst

    def inverted(self) -> "Matrix":  # :586-604
        det = self.determinant()
        det = _F(1.0) if (_F(0.0) - EPSILON) < det < (_F(0.0) + EPSILON) else _F(_F(1.0) / det)
        out = Matrix()
        for i in range(4):
            for j in range(4):
                sign = _F(1 - ((i + j) % 2) * 2)
                sub = self.submatrix(i, j).determinant()
                out.e[i, j] = _F(_F(sub * sign) * det)
        return out

    def transform(self, v) -> np.ndarray:  # :170-188
        x, y, z = (_F(c) for c in v)
        e = self.e
        return np.array([_F(_F(_F(_F(e[0, a] * x) + _F(e[1, a] * y)) + _F(e[2, a] * z)) + e[3, a]) for a in range(3)],
                        np.float32)

    def row(self, r: int) -> np.ndarray:  # getRow (:786-795)
        return np.array([self.e[0, r], self.e[1, r], self.e[2, r], self.e[3, r]], np.float32)


def quat_to_matrix(q) -> Matrix:
    """CQuaternion::toMatrix (PS_Quaternion.h:368-394); q = (x, y, z, w)."""
    x, y, z, w = (_F(c) for c in q)
    xx, yy, zz = _F(x * x), _F(y * y), _F(z * z)
    xy, xz, yz = _F(x * y), _F(x * z), _F(y * z)
    wx, wy, wz = _F(w * x), _F(w * y), _F(w * z)
    one, two = _F(1.0), _F(2.0)
    t = Matrix()
    t.e[0, 0] = _F(one - _F(two * _F(yy + zz)))
    t.e[1, 0] = _F(two * _F(xy - wz))
    t.e[2, 0] = _F(two * _F(xz + wy))
    t.e[0, 1] = _F(two * _F(xy + wz))
    t.e[1, 1] = _F(one - _F(two * _F(xx + zz)))
    t.e[2, 1] = _F(two * _F(yz - wx))
    t.e[0, 2] = _F(two * _F(xz - wy))
    t.e[1, 2] = _F(two * _F(yz + wx))
    t.e[2, 2] = _F(one - _F(two * _F(xx + yy)))
    t.e[3, :3] = 0.0
    t.e[:3, 3] = 0.0
    t.e[3, 3] = 1.0
    return t


@dataclass
class Affine:
    """CAffineTransformation (PS_AffineTransformation.h:62-68, 159-181)."""

    scale: tuple = (1.0, 1.0, 1.0)
    rotate: tuple = (0.0, 0.0, 0.0, 1.0)  # quaternion x, y, z, w
    translate: tuple = (0.0, 0.0, 0.0)

    def forward(self) -> Matrix:
        m = Matrix()
        t = np.asarray(self.translate, np.float32)
        m.set_translate(_F(-1.0) * t)
        m.set_scale(self.scale)
        m.multiply(quat_to_matrix(self.rotate))
        m.set_translate(t)
        return m

    def backward(self) -> Matrix:
        return self.forward().inverted()


@dataclass
class Material:
    ambient: tuple = (0.2, 0.2, 0.2, 0.5)
    diffused: tuple = (0.6, 0.6, 0.6, 1.0)
    specular: tuple = (0.9, 0.9, 0.9, 1.0)
    shininess: float = 32.0


# ---------------------------------------------------------------------------
@dataclass
class BlobNode:
    """CBlobNode: type, children, transform, material, id and (optional) octree box."""

    node_type: BlobNodeType
    children: list = field(default_factory=list)
    transform: Affine = field(default_factory=Affine)
    material: Material = field(default_factory=Material)
    node_id: int = -1
    octree: tuple | None = None  # (lo[3], hi[3]) world box; computed if None
    params: dict = field(default_factory=dict)

    def is_operator(self) -> bool:
        return self.node_type >= BlobNodeType.OP_UNION

    def add_child(self, n: "BlobNode") -> "BlobNode":
        self.children.append(n)
        return n


def Point(position, **kw):  # CSkeletonPoint
    return BlobNode(BlobNodeType.PRIM_POINT, params={"position": position}, **kw)


def Line(start, end, **kw):  # CSkeletonLine
    return BlobNode(BlobNodeType.PRIM_LINE, params={"start": start, "end": end}, **kw)


def Cylinder(position, direction, radius, height, **kw):  # CSkeletonCylinder
    return BlobNode(BlobNodeType.PRIM_CYLINDER,
                    params={"position": position, "direction": direction, "radius": radius, "height": height}, **kw)


def Disc(position, direction, radius, **kw):  # CSkeletonDisc
    return BlobNode(BlobNodeType.PRIM_DISC, params={"position": position, "direction": direction, "radius": radius},
                    **kw)


def Ring(position, direction, radius, **kw):  # CSkeletonRing
    return BlobNode(BlobNodeType.PRIM_RING, params={"position": position, "direction": direction, "radius": radius},
                    **kw)


def Cube(position, side, **kw):  # CSkeletonCube
    return BlobNode(BlobNodeType.PRIM_CUBE, params={"position": position, "side": side}, **kw)


def Triangle(c0, c1, c2, **kw):  # CSkeletonTriangle
    return BlobNode(BlobNodeType.PRIM_TRIANGLE, params={"corners": (c0, c1, c2)}, **kw)


def Null(**kw):  # CNullPrimitive
    return BlobNode(BlobNodeType.PRIM_NULL, **kw)


def Instance(origin: "BlobNode", **kw):  # CInstance (PS_BlobTree/include/CInstance.h): origin's field
    return BlobNode(BlobNodeType.PRIM_INSTANCE, params={"origin": origin}, **kw)


def Op(kind: BlobNodeType, *children, **params) -> BlobNode:
    """An operator node; RicciBlend takes n=..., warps their factors (resX..resW)."""
    return BlobNode(BlobNodeType(kind), children=list(children), params=params)


# ---------------------------------------------------------------------------
ISO_BOX = _F(soa.ISO_DIST + _F(_F(5.0) * soa.MIN_CELL_SIZE))


def _local_support_box(n: BlobNode):
    """Skeleton support box in local coordinates (PrepareBBoxes' extents,
    PS_Polygonizer.cpp:71-195), used for the node's octree box."""
    p = n.params
    iso = float(ISO_BOX)
    t = n.node_type
    if t == BlobNodeType.PRIM_POINT:
        c = np.asarray(p["position"], np.float64)
        return c - iso, c + iso
    if t == BlobNodeType.PRIM_LINE:
        a, b = np.asarray(p["start"], np.float64), np.asarray(p["end"], np.float64)
        return np.minimum(a, b) - iso, np.maximum(a, b) + iso
    if t == BlobNodeType.PRIM_CYLINDER:
        a = np.asarray(p["position"], np.float64)
        b = a + float(p["height"]) * np.asarray(p["direction"], np.float64)
        r = float(p["radius"]) + iso
        return np.minimum(a, b) - r, np.maximum(a, b) + r
    if t in (BlobNodeType.PRIM_DISC, BlobNodeType.PRIM_RING):
        c = np.asarray(p["position"], np.float64)
        r = float(p["radius"]) + iso
        return c - r, c + r
    if t == BlobNodeType.PRIM_CUBE:
        c = np.asarray(p["position"], np.float64)
        s = float(p["side"]) + iso
        return c - s, c + s
    if t == BlobNodeType.PRIM_TRIANGLE:
        cs = np.asarray(p["corners"], np.float64)
        return cs.min(axis=0) - iso, cs.max(axis=0) + iso
    return np.zeros(3) - iso, np.zeros(3) + iso


def compute_octrees(n: BlobNode, method: str = "reference"):
    """Fill every node's octree box: "reference" (default) as ParsipHaptics computes them
    for SimdPoly (compute_octrees_reference), or "aabb", conservative world AABBs of each
    skeleton's support (8 transformed corners; an operator's box is the union)."""
    if method == "reference":
        fn = compute_octrees_reference
    elif method == "aabb":
        fn = compute_octrees_aabb
    else:
        raise ValueError(f"unknown octree method {method!r}")
    box = fn(n)
    if _has_instance(n):  # an Instance takes its origin's box: a second pass once every origin has one
        box = fn(n)
    return box


def _has_instance(n: BlobNode) -> bool:
    return n.node_type == BlobNodeType.PRIM_INSTANCE or any(_has_instance(c) for c in n.children)


def _instance_box(n: BlobNode, fwd: "Matrix"):
    """CInstance::computeOctree (CInstance.h:43-53): the origin's box (zero before the origin
    has one), mapped like a primitive's by the accumulated forward matrix."""
    o = n.params["origin"].octree
    blo, bhi = (np.zeros(3, np.float32), np.zeros(3, np.float32)) if o is None else o
    lt, ht = fwd.transform(blo), fwd.transform(bhi)
    return np.minimum(lt, ht), np.maximum(lt, ht)


def compute_octrees_aabb(n: BlobNode):
    if n.is_operator():
        boxes = [compute_octrees_aabb(c) for c in n.children]
        lo = np.min([b[0] for b in boxes], axis=0)
        hi = np.max([b[1] for b in boxes], axis=0)
    elif n.node_type == BlobNodeType.PRIM_INSTANCE:
        lo, hi = _instance_box(n, n.transform.forward())
    else:
        llo, lhi = _local_support_box(n)
        fwd = n.transform.forward()
        corners = [fwd.transform([(llo, lhi)[i >> 2 & 1][0], (llo, lhi)[i >> 1 & 1][1], (llo, lhi)[i & 1][2]])
                   for i in range(8)]
        lo = np.min(corners, axis=0).astype(np.float64)
        hi = np.max(corners, axis=0).astype(np.float64)
    n.octree = (np.asarray(lo, np.float32), np.asarray(hi, np.float32))
    return n.octree


ISO_VALUE = _F(0.5)  # _constSettings.h:10
OCTREE_EXPANSION = _F(0.6)  # BOUNDING_OCTREE_EXPANSION_FACTOR, _constSettings.h:4


def _skeleton_bound(n: BlobNode):
    """CSkeleton*::bound() in local coordinates, fp32 in the reference's operation order
    (CSkeletonPoint.h:59-64, CSkeletonLine.h:80-85, CSkeletonCylinder.h:103-110,
    CSkeletonDisc.h:93-100, CSkeletonRing.h:107-114, CSkeletonCube.h:175-182,
    CSkeletonTriangle.h:326-333, CNullPrimitive.h:25-30).  BBOX keeps the corners as given
    (PS_BoundingBox.h:17): a Line or Cylinder along a negative direction gives lo > hi."""
    p = n.params
    t = n.node_type
    iso = ISO_VALUE
    v = lambda x: np.asarray(x, np.float32)  # noqa: E731
    if t == BlobNodeType.PRIM_POINT:
        c = v(p["position"])
        return c - iso, c + iso
    if t == BlobNodeType.PRIM_LINE:
        a, b = v(p["start"]), v(p["end"])
        e = iso + (_F(3.0) * iso) * (b - a)
        return a - e, b + e
    if t == BlobNodeType.PRIM_CYLINDER:
        s0, d = v(p["position"]), v(p["direction"])
        s1 = s0 + _F(p["height"]) * d
        e = (iso + _F(p["radius"])) * v((1.0, 1.0, 1.0)) + (_F(0.5) * iso) * d
        return s0 - e, s1 + e
    if t in (BlobNodeType.PRIM_DISC, BlobNodeType.PRIM_RING):
        c, d = v(p["position"]), v(p["direction"])
        r = _F(_F(p["radius"]) + iso)
        e = r * (v((1.0, 1.0, 1.0)) - d) + iso * d
        return c - e, c + e
    if t == BlobNodeType.PRIM_CUBE:
        c = v(p["position"])
        ss = _F(_F(p["side"]) + iso)
        return c - ss, c + ss
    if t == BlobNodeType.PRIM_TRIANGLE:
        cs = v(p["corners"])
        return cs.min(axis=0) - iso, cs.max(axis=0) + iso
    return v((0.0, 0.0, 0.0)), v((0.0, 0.0, 0.0))


def compute_octrees_reference(n: BlobNode, branch: "Matrix | None" = None):
    """The octrees ParsipHaptics hands SimdPoly after loading a model:
    CLayer::recursive_RecomputeAllOctrees (CLayerManager.cpp:629-646).  A primitive's box
    is its skeleton bound with only its two corners mapped by the accumulated forward
    matrix (COctree::transform, PS_Octree.cpp:342-348); an operator's box is the union of
    its children (Union, Blend, RicciBlend, GradientBlend, PCM), its first child
    (Difference, SmoothDifference), their csgIntersection (Intersection) or its first
    child grown by 0.6 (the warps) (the operators' computeOctree, PS_BlobTree/include)."""
    cur = (branch.copy() if branch is not None else Matrix())
    cur.multiply(n.transform.forward())
    if n.is_operator():
        boxes = [compute_octrees_reference(c, cur) for c in n.children]
        t = n.node_type
        lo, hi = boxes[0][0].copy(), boxes[0][1].copy()
        if t in (BlobNodeType.OP_DIF, BlobNodeType.OP_SMOOTHDIF):
            pass
        elif t == BlobNodeType.OP_INTERSECT:
            for blo, bhi in boxes[1:]:
                for a in range(3):  # COctree::csgIntersection (PS_Octree.cpp:362-380)
                    if lo[a] <= bhi[a] and hi[a] >= blo[a]:
                        lo[a] = max(lo[a], blo[a])
                        hi[a] = min(hi[a], bhi[a])
        elif t in (BlobNodeType.OP_WARPTWIST, BlobNodeType.OP_WARPTAPER, BlobNodeType.OP_WARPBEND,
                   BlobNodeType.OP_WARPSHEAR):
            lo, hi = lo - OCTREE_EXPANSION, hi + OCTREE_EXPANSION
        else:
            for blo, bhi in boxes[1:]:
                lo, hi = np.minimum(lo, blo), np.maximum(hi, bhi)
    elif n.node_type == BlobNodeType.PRIM_INSTANCE:
        lo, hi = _instance_box(n, cur)
    else:
        blo, bhi = _skeleton_bound(n)
        lt, ht = cur.transform(blo), cur.transform(bhi)
        lo, hi = np.minimum(lt, ht), np.maximum(lt, ht)
    n.octree = (np.asarray(lo, np.float32), np.asarray(hi, np.float32))
    return n.octree


def binarize(n: BlobNode) -> BlobNode:
    """Fold n-ary operators into left-nested binary ones in child order (an extension:
    the reference SIMD path rejects non-binary ops with -3, :81-86)."""
    kids = [binarize(c) for c in n.children]
    if not n.is_operator() or len(kids) <= 2:
        return BlobNode(n.node_type, kids, n.transform, n.material, n.node_id, n.octree, dict(n.params))
    acc = kids[0]
    for k in kids[1:]:
        acc = BlobNode(n.node_type, [acc, k], n.transform, n.material, n.node_id, None, dict(n.params))
    return acc


def _translate(code: int, raw: bool) -> int:
    return int(code) if raw else soa.translate_blobtree_type(int(code))


def linearize_blobtree(root: BlobNode, raw_types: bool = False, triangle_compat: bool = False,
                       octrees: str = "reference"):
    """SimdPoly::linearizeBlobTree (PS_HighPerformanceRender.cpp:42-371, 366-371).

    Node boxes are the nodes' octrees (getOctree(), :47-50, 97-107, 176-187); nodes without
    one get them from compute_octrees(root, octrees) first.
    Returns (code, Model): code is the root's id (0) or a negative PS_ERROR_* code."""
    model = soa.Model.empty("blobtree")
    P, O, PM, BM = model.prims, model.ops, model.mats, model.boxmats

    def missing(n):
        return n.octree is None or any(missing(c) for c in n.children)

    if missing(root):
        compute_octrees(root, octrees)
    lo, hi = root.octree
    P["bboxLo"][0] = lo
    P["bboxHi"][0] = hi
    PM["matrix"][0, :12] = np.eye(4, dtype=np.float32).reshape(-1)[:12]
    BM["matrix"][0, :16] = np.eye(4, dtype=np.float32).reshape(-1)
    PM["count"][0] = 1
    BM["count"][0] = 1

    def rec(n: BlobNode):
        nlo, nhi = n.octree
        if n.is_operator():
            if int(O["ctOps"][0]) >= soa.MAX_TREE_NODES:
                return PS_ERROR_OPERATOR_OVERFLOW, 1
            cur = int(O["ctOps"][0])
            O["ctOps"][0] = cur + 1
            O["opType"][0, cur] = _translate(n.node_type, raw_types)
            if len(n.children) != 2:
                return PS_ERROR_NON_BINARY_OP, 1
            kid, isop = [0, 0], [0, 0]
            for c in range(2):
                r, iop = rec(n.children[c])
                if r < 0:
                    return r, 1
                kid[c], isop[c] = r, iop
            O["opLeftChild"][0, cur] = kid[0]
            O["opRightChild"][0, cur] = kid[1]
            O["opChildKind"][0, cur] = isop[0] * 2 + isop[1]
            for a, cname in enumerate("XYZ"):
                O[f"vBoxLo{cname}"][0, cur] = nlo[a]
                O[f"vBoxHi{cname}"][0, cur] = nhi[a]
            pr = n.params
            t = n.node_type
            if t == BlobNodeType.OP_PCM:
                for k, key in zip("XYZW", ("propagate_left", "propagate_right", "alpha_left", "alpha_right")):
                    O[f"res{k}"][0, cur] = pr.get(key, 0.0)
            elif t == BlobNodeType.OP_RICCIBLEND:
                nn = _F(pr.get("n", 2.0))
                O["resX"][0, cur] = nn
                if nn != 0.0:
                    O["resY"][0, cur] = _F(_F(1.0) / nn)
            elif t in (BlobNodeType.OP_WARPTWIST, BlobNodeType.OP_WARPTAPER, BlobNodeType.OP_WARPBEND,
                       BlobNodeType.OP_WARPSHEAR):
                for k in "XYZW":
                    if f"res{k}" in pr:
                        O[f"res{k}"][0, cur] = pr[f"res{k}"]
            return cur, 1
        if int(P["ctPrims"][0]) >= soa.MAX_TREE_NODES:
            return PS_ERROR_PRIM_OVERFLOW, 0
        cur = int(P["ctPrims"][0])
        P["ctPrims"][0] = cur + 1
        d = n.material.diffused
        P["colorX"][0, cur], P["colorY"][0, cur], P["colorZ"][0, cur] = d[0], d[1], d[2]
        for a, cname in enumerate("XYZ"):
            P[f"vPrimBoxLo{cname}"][0, cur] = nlo[a]
            P[f"vPrimBoxHi{cname}"][0, cur] = nhi[a]
        back = n.transform.backward()
        if back.is_identity():
            P["idxMatrix"][0, cur] = 0
        else:
            k = int(PM["count"][0])
            if k >= soa.MAX_TREE_NODES:  # 128 slots, slot 0 the identity (the C++ face returns the same)
                return PS_ERROR_PRIM_OVERFLOW, 0
            P["idxMatrix"][0, cur] = k
            rows = np.concatenate([back.row(0), back.row(1), back.row(2)])
            PM["matrix"][0, k * 12:(k + 1) * 12] = rows
            PM["count"][0] = k + 1
        P["skeletType"][0, cur] = _translate(n.node_type, raw_types)
        p = n.params
        t = n.node_type

        def put(prefix, v):
            for a, cname in enumerate("XYZ"):
                P[f"{prefix}{cname}"][0, cur] = v[a]

        if t == BlobNodeType.PRIM_POINT:
            put("pos", p["position"])
        elif t == BlobNodeType.PRIM_LINE:
            put("pos", p["start"])
            put("dir", p["end"])
        elif t in (BlobNodeType.PRIM_RING, BlobNodeType.PRIM_DISC):
            put("pos", p["position"])
            put("dir", p["direction"])
            r = _F(p["radius"])
            P["resX"][0, cur] = r
            P["resY"][0, cur] = _F(r * r)
        elif t == BlobNodeType.PRIM_CYLINDER:
            put("pos", p["position"])
            put("dir", p["direction"])
            P["resX"][0, cur] = p["radius"]
            P["resY"][0, cur] = p["height"]
        elif t == BlobNodeType.PRIM_CUBE:
            put("pos", p["position"])
            P["resX"][0, cur] = p["side"]
        elif t == BlobNodeType.PRIM_TRIANGLE:
            c0, c1, c2 = p["corners"]
            put("pos", c0)
            put("dir", c1)
            P["resX"][0, cur] = c2[0]
            P["resY"][0, cur] = c2[1]
            if triangle_compat:
                P["resX"][0, cur] = c2[2]  # the adapter's bug (:342-344)
            else:
                P["resZ"][0, cur] = c2[2]
        elif t == BlobNodeType.PRIM_NULL:
            put("pos", (0.0, 0.0, 0.0))
        return cur, 0

    code, _ = rec(root)
    return code, model


class SimdPoly:
    """SimdPoly (PS_HighPerformanceRender.h:15-33) on the MI355X library."""

    def __init__(self, device: int = 0):
        from . import gpu

        self._gpu = gpu
        self.poly = gpu.Polygonizer(device)
        self.model = soa.Model.empty()

    def reset(self) -> None:
        self.model = soa.Model.empty()

    def linearizeBlobTree(self, root: BlobNode, **kw) -> int:  # noqa: N802 (reference name)
        self.reset()
        code, self.model = linearize_blobtree(root, **kw)
        if code >= 0:
            self.poly.set_model(self.model)
        return code

    def run(self, cellsize: float):
        """Polygonize (PS_HighPerformanceRender.cpp:373-376); returns PsMeshInfo."""
        return self.poly.run(cellsize)

    def mesh(self):
        return self.poly.download()

    def close(self) -> None:
        self.poly.close()

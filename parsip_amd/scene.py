"""Parsip `.scene` files -> BlobTree.

The format is the INI-style script CLayerManager writes and reads
(Parsip100/ParsipHaptics/include/CLayerManager.cpp:1456-1520 save/load,
CLayer::recursive_ReadBlobNode :683-791): a [Global] section (NumLayers, RootIDs) and
one [BLOBNODE id] section per node.  Operators: IsOperator=1, OperatorType (factory
names, e.g. "RICCI BLEND"), ChildrenCount + ChildrenIDs=(a, b, ...) or
ChildrenIDsUseRange + ChildrenIDsRange; RicciBlend reads `power`
(CRicciBlend.h:167-175).  Primitives: PrimitiveType (older files, like the reference's
Distrib/train_corrected.scene, say SkeletonType), the affine transform AffineScale /
AffineRotate (quaternion x, y, z, w) / AffineTranslate and the material
(CBlobNode::loadGenericInfoScript, CBlobTree.cpp:123-149), then the skeleton's own
fields (CSkeleton*.h loadScript: position, direction, radius, height, side, start,
end, corner0..2).  PCM reads its four widths / attenuations (CPcm.h:93-101); an
INSTANCE primitive names its origin by OriginalNodeIndex (CInstance.h:69-75, resolved with
findNodeByID, CLayerManager.cpp:782-793; here after the whole layer is read, so an origin
may also come later in the file).  Lines end in NUL CR LF in files the reference wrote.
"""
from __future__ import annotations

import re

from . import blobtree as bt
from .blobtree import BlobNodeType as B

OPERATOR_NAMES = {
    "UNION": B.OP_UNION, "INTERSECTION": B.OP_INTERSECT, "DIFFERENCE": B.OP_DIF,
    "SMOOTH DIFFERENCE": B.OP_SMOOTHDIF, "SMOOTHDIFFERENCE": B.OP_SMOOTHDIF, "BLEND": B.OP_BLEND,
    "RICCI BLEND": B.OP_RICCIBLEND, "GRADIENT BLEND": B.OP_GRADIENTBLEND, "PCM": B.OP_PCM,
    "WARP TWIST": B.OP_WARPTWIST, "WARPTWIST": B.OP_WARPTWIST, "WARP TAPER": B.OP_WARPTAPER,
    "WARPTAPER": B.OP_WARPTAPER, "WARP BEND": B.OP_WARPBEND, "WARPBEND": B.OP_WARPBEND,
    "WARP SHEAR": B.OP_WARPSHEAR, "WARPSHEAR": B.OP_WARPSHEAR, "CACHE": B.OP_CACHE,
}
PRIMITIVE_NAMES = {
    "POINT": B.PRIM_POINT, "LINE": B.PRIM_LINE, "CYLINDER": B.PRIM_CYLINDER, "DISC": B.PRIM_DISC,
    "RING": B.PRIM_RING, "CUBE": B.PRIM_CUBE, "TRIANGLE": B.PRIM_TRIANGLE, "NULL": B.PRIM_NULL,
    "INSTANCE": B.PRIM_INSTANCE,
}


class SceneError(ValueError):
    pass


def parse_ini(text: str) -> dict:
    """CSketchConfig's INI dialect: [section] headers, key=value lines."""
    sections: dict = {}
    cur = None
    for raw in text.replace("\r", "\n").split("\n"):
        line = raw.replace("\x00", "").strip()
        if not line or line.startswith(";") or line.startswith("#"):
            continue
        m = re.fullmatch(r"\[(.+)\]", line)
        if m:
            cur = sections.setdefault(m.group(1).strip(), {})
            continue
        if "=" in line and cur is not None:
            k, v = line.split("=", 1)
            cur[k.strip()] = v.strip()
    return sections


def _floats(s: str) -> list:
    return [float(x) for x in s.strip().strip("()").split(",") if x.strip()]


def _ints(s: str) -> list:
    return [int(float(x)) for x in s.strip().strip("()").split(",") if x.strip()]


class _Reader:
    def __init__(self, sections: dict):
        self.s = sections
        self.by_id: dict = {}
        self.instances: list = []  # (Instance node, origin id)

    def resolve_instances(self) -> None:
        for n, oid in self.instances:
            if oid not in self.by_id:
                raise SceneError(f"Instance BLOBNODE {n.node_id}: unable to find origin node id {oid}")
            n.params["origin"] = self.by_id[oid]
        self.instances = []

    def sec(self, nid: int) -> dict | None:
        return self.s.get(f"BLOBNODE {nid}")

    def node(self, nid: int, depth: int = 0) -> bt.BlobNode:
        if depth > 4096:
            raise SceneError("node graph too deep (cycle?)")
        sec = self.sec(nid)
        if sec is None:
            raise SceneError(f"missing [BLOBNODE {nid}]")
        if int(float(sec.get("IsOperator", "0"))):
            name = sec.get("OperatorType", "").upper()
            if name not in OPERATOR_NAMES:
                raise SceneError(f"BLOBNODE {nid}: unknown operator {name!r}")
            ids: list = []
            if int(float(sec.get("ChildrenIDsUseRange", "0"))) and "ChildrenIDsRange" in sec:
                r = _ints(sec["ChildrenIDsRange"])
                if len(r) == 2:
                    ids = list(range(r[0], r[1] + 1))
            if not ids:
                ids = _ints(sec.get("ChildrenIDs", "()"))
                ct = int(float(sec.get("ChildrenCount", len(ids))))
                ids = ids[:ct]
            params = {}
            if OPERATOR_NAMES[name] == B.OP_RICCIBLEND:
                params["n"] = float(sec.get("power", "2"))
            elif OPERATOR_NAMES[name] == B.OP_PCM:  # readFloat's default is 0 (PS_AppConfig.h:60)
                for key, k in (("Propagate Left", "propagate_left"), ("Propagate Right", "propagate_right"),
                               ("Attenuate Left", "alpha_left"), ("Attenuate Right", "alpha_right")):
                    params[k] = float(sec.get(key, "0"))
            n = bt.Op(OPERATOR_NAMES[name], *[self.node(i, depth + 1) for i in ids], **params)
            n.node_id = nid
            self.by_id[nid] = n
            return n
        name = (sec.get("PrimitiveType") or sec.get("SkeletonType") or "").upper()
        if name not in PRIMITIVE_NAMES:
            raise SceneError(f"BLOBNODE {nid}: unknown primitive {name!r}")
        t = PRIMITIVE_NAMES[name]

        def v3(key, default=(0.0, 0.0, 0.0)):
            return tuple(_floats(sec[key])[:3]) if key in sec else default

        def f1(key, default=0.0):
            return float(sec[key]) if key in sec else default

        kw = {
            "transform": bt.Affine(v3("AffineScale", (1.0, 1.0, 1.0)),
                                   tuple(_floats(sec["AffineRotate"])[:4]) if "AffineRotate" in sec
                                   else (0.0, 0.0, 0.0, 1.0),
                                   v3("AffineTranslate")),
            "material": bt.Material(diffused=tuple(_floats(sec["MtrlDiffused"])[:4]) if "MtrlDiffused" in sec
                                    else (0.6, 0.6, 0.6, 1.0)),
        }
        if t == B.PRIM_POINT:
            n = bt.Point(v3("position"), **kw)
        elif t == B.PRIM_LINE:
            n = bt.Line(v3("start"), v3("end"), **kw)
        elif t == B.PRIM_CYLINDER:
            n = bt.Cylinder(v3("position"), v3("direction", (0.0, 1.0, 0.0)), f1("radius"), f1("height"), **kw)
        elif t == B.PRIM_DISC:
            n = bt.Disc(v3("position"), v3("direction", (0.0, 1.0, 0.0)), f1("radius"), **kw)
        elif t == B.PRIM_RING:
            n = bt.Ring(v3("position"), v3("direction", (0.0, 1.0, 0.0)), f1("radius"), **kw)
        elif t == B.PRIM_CUBE:
            n = bt.Cube(v3("position"), f1("side"), **kw)
        elif t == B.PRIM_TRIANGLE:
            n = bt.Triangle(v3("corner0"), v3("corner1"), v3("corner2"), **kw)
        elif t == B.PRIM_INSTANCE:
            n = bt.Instance(None, **kw)
            self.instances.append((n, int(float(sec.get("OriginalNodeIndex", "-1")))))
        else:
            n = bt.Null(**kw)
        n.node_id = nid
        self.by_id[nid] = n
        return n


def load_scene(path_or_text: str, from_text: bool = False) -> list:
    """Parse a .scene file; returns one BlobTree root per layer (RootIDs order)."""
    if from_text:
        text = path_or_text
    else:
        with open(path_or_text, "rb") as f:
            text = f.read().decode("latin-1")
    sections = parse_ini(text)
    g = sections.get("Global", {})
    roots = _ints(g.get("RootIDs", "()"))
    n_layers = int(float(g.get("NumLayers", len(roots))))
    rd = _Reader(sections)
    layers = []
    for r in roots[:n_layers]:
        if r >= 0:
            layers.append(rd.node(r))
            rd.resolve_instances()
    return layers


def count_nodes(n: bt.BlobNode) -> tuple:
    """(primitives, operators) of a tree."""
    if not n.is_operator():
        return 1, 0
    p, o = 0, 1
    for c in n.children:
        cp, co = count_nodes(c)
        p += cp
        o += co
    return p, o

"""Compat mode: ParsipHaptics' own polygonizer (the "GUI path") on the
MI355X library (include/parsip_gpu_gui.h).

Reference interface mirrored (Parsip100/ParsipHaptics/include/):

    int COMPACTBLOBTREE::convert(CBlobNode* root);               CompactBlobTree.cpp:25-408
    void CParsipOptimized::setup(COMPACTBLOBTREE*, const COctree&, int id,
                                 float cellsize, float isovalue);  CPolyParsipOptimized.cpp:330-390
    void CParsipOptimized::run();                                  :392-410
    countMPUs / statsIntersectedMPUs / statsMeshInfo / statsTotalFieldEvals /
    statsIntersectedCellsCount / statsTotalCellsInIntersectedMPUs / exportMesh
    CParsipOptimized* Run_Polygonizer(CBlobNode*, float cellSize, float isovalue);  :615-628

``compact_blobtree`` restates ``COMPACTBLOBTREE::convert`` (pre-order op ids, DFS prim
ids, a matrix slot per non-identity backward matrix, the operator parameters of :159-240
and primitive fields of :287-400, its error codes).  The polygonization itself runs on
the device; there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from . import blobtree as bt
from . import gpu

B = bt.BlobNodeType
_F = np.float32

PS_SUCCESS = 1  # convert() returns the root's id (0) on success
ERR_OPS_OVERFLOW = -1
ERR_PRIMS_OVERFLOW = -2
ERR_KIDS_OVERFLOW = -3
ERR_PARAM_ERROR = -4
ERR_NODE_NOT_RECOGNIZED = -5
RET_UNSUPPORTED = -7  # PSGUI_RET_UNSUPPORTED (parsip_gpu_gui.h: empty operators, depth, PCM / Instance limits)
MAX_COMPACT_KIDS_COUNT = 1024
MIN_BLOB_NODES = 32
ISO_VALUE = 0.5
GRID_DIM = 8

PRIM_DTYPE = np.dtype([("type", "<i4"), ("orgID", "<i4"), ("idxMtx", "<u4"), ("reserved", "<u4"),
                       ("color", "<f4", 4), ("pos", "<f4", 4), ("dir", "<f4", 4), ("res1", "<f4", 4),
                       ("res2", "<f4", 4), ("octLo", "<f4", 4), ("octHi", "<f4", 4)])
OP_DTYPE = np.dtype([("type", "<i4"), ("orgID", "<i4"), ("ctKids", "<i4"), ("kidStart", "<u4"),
                     ("idxMtx", "<u4"), ("reserved", "<u4", 3), ("params", "<f4", 4), ("octLo", "<f4", 4),
                     ("octHi", "<f4", 4)])
MTX_DTYPE = np.dtype([("r", "<f4", (4, 4))])
STATS_DTYPE = np.dtype([("fieldEvals", "<u4"), ("intersectedCells", "<u4"), ("ctVertices", "<u4"),
                        ("ctTriangles", "<u4")])
assert PRIM_DTYPE.itemsize == 128 and OP_DTYPE.itemsize == 80 and MTX_DTYPE.itemsize == 64

_OPS = {B.OP_UNION, B.OP_BLEND, B.OP_DIF, B.OP_SMOOTHDIF, B.OP_INTERSECT, B.OP_PCM, B.OP_RICCIBLEND,
        B.OP_WARPTWIST, B.OP_WARPTAPER, B.OP_WARPBEND, B.OP_WARPSHEAR}
_PRIMS = {B.PRIM_POINT, B.PRIM_LINE, B.PRIM_RING, B.PRIM_DISC, B.PRIM_CYLINDER, B.PRIM_CUBE, B.PRIM_TRIANGLE,
          B.PRIM_QUADRICPOINT, B.PRIM_NULL, B.PRIM_INSTANCE}


class PsGuiInfo(ctypes.Structure):
    _fields_ = [("dims", ctypes.c_uint32 * 3), ("ctLatticeMPUs", ctypes.c_uint32), ("ctMPUs", ctypes.c_uint32),
                ("ctIntersectedMPUs", ctypes.c_uint32), ("ctProcessedMPUs", ctypes.c_uint32),
                ("ctVertices", ctypes.c_uint32), ("ctTriangles", ctypes.c_uint32),
                ("ctIntersectedCells", ctypes.c_uint32), ("ctFieldEvals", ctypes.c_uint64),
                ("ctCellsInIntersectedMPUs", ctypes.c_uint64)]


assert ctypes.sizeof(PsGuiInfo) == 56


def QuadricPoint(position, radius, scale, **kw):  # CQuadricPoint (getFieldRadius, getFieldScale)
    return bt.BlobNode(B.PRIM_QUADRICPOINT, params={"position": position, "radius": radius, "scale": scale},
                       **kw)


def Pcm(left, right, propagate_left=None, propagate_right=None, alpha_left=0.5, alpha_right=0.5, **kw):
    """CPcm (PS_BlobTree/include/CPcm.h): precise contact between two kids; the defaults are
    resetParams' PCM_PROPAGATION_WIDTH = 0.5 * ISO_DISTANCE and PCM_ATTENUATION = 0.5
    (_constSettings.h:14-15)."""
    w = float(np.float32(0.5) * np.float32(0.454202))
    return bt.Op(B.OP_PCM, left, right, propagate_left=w if propagate_left is None else propagate_left,
                 propagate_right=w if propagate_right is None else propagate_right, alpha_left=alpha_left,
                 alpha_right=alpha_right, **kw)


@dataclass
class CompactTree:
    """COMPACTBLOBTREE's arrays (CompactBlobTree.h:26-61), kid lists flattened."""

    prims: np.ndarray  # PRIM_DTYPE[ctPrims]
    ops: np.ndarray    # OP_DTYPE[ctOps]
    kids: np.ndarray   # uint32: kid id | isOp << 16
    mtx: np.ndarray    # MTX_DTYPE[ctMtx], entry 0 the identity
    root_octree: tuple  # the root's (lo, hi): CParsipOptimized::setup's COctree

    @property
    def ct_prims(self) -> int:
        return len(self.prims)

    @property
    def ct_ops(self) -> int:
        return len(self.ops)

    def ptrs(self):
        def p(a):
            return a.ctypes.data if len(a) else None
        return (p(self.prims), len(self.prims), p(self.ops), len(self.ops), p(self.kids), len(self.kids),
                p(self.mtx), len(self.mtx))


def _v4(v, w=0.0):
    return (_F(v[0]), _F(v[1]), _F(v[2]), _F(w))


def compact_blobtree(root: bt.BlobNode | None, octrees: str = "reference"):
    """COMPACTBLOBTREE::convert (CompactBlobTree.cpp:25-408).  Returns (code, CompactTree):
    code is the root's id (0) or a negative ERR_* code."""
    if root is None:
        return ERR_PARAM_ERROR, None

    def missing(n):
        return n.octree is None or any(missing(c) for c in n.children)

    if missing(root):
        bt.compute_octrees(root, octrees)
    prims, ops, kids = [], [], []
    mtx = [np.eye(4, dtype=np.float32)]
    converted = []  # m_lstConvertedIds: (node, compact id) in conversion order
    instances = []  # (prim index, origin node)

    def matrix_index(n) -> int:  # :118-135 / :266-283
        back = n.transform.backward()
        if back.is_identity():
            return 0
        mtx.append(np.stack([back.row(r) for r in range(4)]))
        return len(mtx) - 1

    def convert_node(n: bt.BlobNode):  # convert(CBlobNode*, parentID) (:93-408)
        lo, hi = n.octree
        if n.is_operator():
            cur = len(ops)
            o = np.zeros((), OP_DTYPE)
            o["type"], o["orgID"] = int(n.node_type), n.node_id
            o["octLo"], o["octHi"] = _v4(lo), _v4(hi)
            o["idxMtx"] = matrix_index(n)
            ops.append(o)
            if len(n.children) > MAX_COMPACT_KIDS_COUNT:
                return ERR_KIDS_OVERFLOW, 1
            o["ctKids"] = len(n.children)
            o["kidStart"] = len(kids)
            kids.extend([0] * len(n.children))
            for i, c in enumerate(n.children):
                kid, isop = rec(c)
                if kid < 0:
                    return kid, 1
                kids[int(o["kidStart"]) + i] = kid | (isop << 16)
            t, pr = n.node_type, n.params
            if t not in _OPS:
                return ERR_NODE_NOT_RECOGNIZED, 1
            prm = [_F(0.0)] * 4
            if t == B.OP_PCM:
                prm = [_F(pr.get(k, 0.0)) for k in ("propagate_left", "propagate_right", "alpha_left", "alpha_right")]
            elif t == B.OP_RICCIBLEND:
                nn = _F(pr.get("n", 2.0))
                prm[0] = nn
                if nn != 0.0:
                    prm[1] = _F(_F(1.0) / nn)
            elif t in (B.OP_WARPTWIST, B.OP_WARPTAPER, B.OP_WARPBEND, B.OP_WARPSHEAR):
                prm = [_F(pr.get(f"res{k}", 0.0)) for k in "XYZW"]
            o["params"] = prm
            return cur, 1
        cur = len(prims)
        p = np.zeros((), PRIM_DTYPE)
        p["type"], p["orgID"] = int(n.node_type), n.node_id
        p["color"] = [_F(c) for c in n.material.diffused]
        p["octLo"], p["octHi"] = _v4(lo), _v4(hi)
        p["idxMtx"] = matrix_index(n)
        prims.append(p)
        t, pr = n.node_type, n.params
        if t == B.PRIM_POINT:
            p["pos"] = _v4(pr["position"])
        elif t == B.PRIM_LINE:
            p["res1"], p["res2"] = _v4(pr["start"]), _v4(pr["end"])
        elif t in (B.PRIM_RING, B.PRIM_DISC):
            r = _F(pr["radius"])
            p["pos"], p["dir"] = _v4(pr["position"]), _v4(pr["direction"])
            p["res1"], p["res2"] = [r] * 4, [_F(r * r)] * 4
        elif t == B.PRIM_CYLINDER:
            p["pos"], p["dir"] = _v4(pr["position"]), _v4(pr["direction"])
            p["res1"], p["res2"] = [_F(pr["radius"])] * 4, [_F(pr["height"])] * 4
        elif t == B.PRIM_CUBE:
            p["pos"], p["res1"] = _v4(pr["position"]), [_F(pr["side"])] * 4
        elif t == B.PRIM_TRIANGLE:
            c0, c1, c2 = pr["corners"]
            p["pos"], p["res1"], p["res2"] = _v4(c0), _v4(c1), _v4(c2)
        elif t == B.PRIM_QUADRICPOINT:
            p["pos"] = _v4(pr["position"])
            p["res1"], p["res2"] = [_F(pr["radius"])] * 4, [_F(pr["scale"])] * 4
        elif t == B.PRIM_NULL:
            p["pos"] = _v4((0.0, 0.0, 0.0))
        elif t == B.PRIM_INSTANCE:  # :383-391: (-1, origin id, origin isOp, origin type)
            o = pr["origin"]
            p["res1"] = [_F(-1.0), _F(o.node_id), _F(1.0 if o.is_operator() else 0.0), _F(int(o.node_type))]
            instances.append((cur, o))
        else:
            return ERR_NODE_NOT_RECOGNIZED, 0
        return cur, 0

    def rec(n):  # every converted node's (node, id) pair, in the reference's order (:404)
        r = convert_node(n)
        if r[0] >= 0:
            converted.append((n, r[0]))
        return r

    code, _ = rec(root)
    # updateInstanceNodes (:410-431): the origin's compact id, found by its node (the
    # reference matches the unique node id; identity is the same here, ids may be unset)
    for idx, o in instances:
        for n, cid in converted:
            if n is o:
                prims[idx]["res1"][0] = _F(cid)
                break
    tree = CompactTree(np.array(prims, PRIM_DTYPE), np.array(ops, OP_DTYPE), np.array(kids, np.uint32),
                       np.array([(m,) for m in mtx], MTX_DTYPE), root.octree)
    return code, tree


@dataclass
class GuiMesh:
    pos: np.ndarray       # (V, 3)
    nrm: np.ndarray       # (V, 3)
    col: np.ndarray       # (V, 4) rgba
    tris: np.ndarray      # (T, 3) mesh-wide vertex ids
    mpu_v: np.ndarray     # per lattice MPU: first vertex (ctLatticeMPUs + 1)
    mpu_t: np.ndarray     # per lattice MPU: first triangle
    stats: np.ndarray     # STATS_DTYPE per lattice MPU


_SIG = {
    "psgpu_gui_create": (["i32", "pvp"], "i32"),
    "psgpu_gui_destroy": (["vp"], None),
    "psgpu_gui_set_tree": (["vp", "vp", "u32", "vp", "u32", "vp", "u32", "vp", "u32"], "i32"),
    "psgpu_gui_polygonize": (["vp", "vp", "vp", "f32", "f32"], "i32"),
    "psgpu_gui_finish": (["vp", "pinfo"], "i32"),
    "psgpu_gui_download": (["vp", "vp", "vp", "vp", "vp", "vp", "vp"], "i32"),
    "psgpu_gui_field_values": (["vp", "vp", "u32", "vp", "vp"], "i32"),
    "psgpu_gui_set_option": (["vp", "i32", "i32"], "i32"),
    "psgpu_gui_jit_status": (["vp", "i32"], "i32"),
    "psgpu_gui_jit_compile": (["vp", "u32", "vp", "u32", "vp", "u32", "vp", "u32", "i32", "vp", "size"], "long"),
    "psgpu_gui_cull_boxes": (["vp", "u32", "vp", "u32", "vp", "u32", "vp", "u32", "vp", "vp"], "i32"),
    "psgpu_gui_get_pcm_state": (["vp", "vp"], "i32"),
    "psgpu_gui_set_pcm_state": (["vp", "vp"], "i32"),
}
OPT_JIT = 1
OPT_CULL = 2
JIT_NONE, JIT_PENDING, JIT_ACTIVE, JIT_FAILED = 0, 1, 2, 3
EXPORTED_SYMBOLS = list(_SIG)


def _lib():
    L = gpu.load()
    if not getattr(L, "_gui_bound", False):
        T = {"i32": ctypes.c_int, "u32": ctypes.c_uint32, "f32": ctypes.c_float, "vp": ctypes.c_void_p,
             "pvp": ctypes.POINTER(ctypes.c_void_p), "pinfo": ctypes.POINTER(PsGuiInfo), "size": ctypes.c_size_t,
             "long": ctypes.c_long, None: None}
        for name, (args, res) in _SIG.items():
            fn = getattr(L, name)
            fn.argtypes = [T[a] for a in args]
            fn.restype = T[res]
        L._gui_bound = True
    return L


def jit_compile(tree: "CompactTree", cull: bool = True, cap: int = 1 << 22):
    """Compile the tree's compat kernels without a device (hiprtc): (code-object bytes,
    generated source); raises with the compiler log on failure."""
    L = _lib()
    buf = ctypes.create_string_buffer(cap)
    p = tree.ptrs()
    n = L.psgpu_gui_jit_compile(p[0], p[1], p[2], p[3], p[4], p[5], p[6], p[7], 1 if cull else 0, buf, cap)
    if n < 0:
        raise RuntimeError(f"psgpu_gui_jit_compile: {n}\n{buf.value.decode(errors='replace')}")
    return n, buf.value.decode()


def cull_boxes(tree: "CompactTree"):
    """(prim boxes (nP, 2, 3), op boxes (nO, 2, 3)): world boxes outside which each node's
    value is exactly +0 (host only)."""
    L = _lib()
    p = tree.ptrs()
    pb = np.zeros((max(p[1], 1), 8), np.float32)
    ob = np.zeros((max(p[3], 1), 8), np.float32)
    gpu._check(L.psgpu_gui_cull_boxes(*p, pb.ctypes.data, ob.ctypes.data), "psgpu_gui_cull_boxes")
    box = lambda a: np.stack([a[:, 0:3], a[:, 4:7]], axis=1)  # noqa: E731
    return box(pb[:p[1]]), box(ob[:p[3]])


class ParsipOptimized:
    """CParsipOptimized (CPolyParsipOptimized.h:226-305) on the MI355X library.  jit: 0 the
    interpreter kernels only, 1 the tree's generated kernels once compiled (default), 2 wait
    for them in set_tree."""

    def __init__(self, device: int = 0, jit: int = None, cull: bool = None):
        self._L = _lib()
        self._g = ctypes.c_void_p()
        gpu._check(self._L.psgpu_gui_create(device, ctypes.byref(self._g)), "psgpu_gui_create")
        if jit is not None:
            gpu._check(self._L.psgpu_gui_set_option(self._g, OPT_JIT, int(jit)), "psgpu_gui_set_option")
        if cull is not None:
            gpu._check(self._L.psgpu_gui_set_option(self._g, OPT_CULL, int(bool(cull))), "psgpu_gui_set_option")
        self._info = None
        self._tree = None
        self._setup = None
        gpu._LIVE.add(self)

    def close(self):
        if getattr(self, "_g", None) and self._g.value:
            self._L.psgpu_gui_destroy(self._g)
            self._g = ctypes.c_void_p()

    __del__ = close

    def jit_status(self, wait: bool = False) -> int:
        """JIT_NONE / JIT_PENDING / JIT_ACTIVE / JIT_FAILED for the current tree."""
        rc = self._L.psgpu_gui_jit_status(self._g, 1 if wait else 0)
        if rc < 0:
            gpu._check(rc, "psgpu_gui_jit_status")
        return rc

    def set_tree(self, tree: CompactTree) -> None:
        rc = self._L.psgpu_gui_set_tree(self._g, *tree.ptrs())
        gpu._check(rc, "psgpu_gui_set_tree")
        self._tree = tree

    def setup(self, tree: CompactTree, octree=None, node_id: int = 0, cellsize: float = 0.25,
              isovalue: float = ISO_VALUE) -> None:
        """CParsipOptimized::setup (:330-390): the tree and the lattice over `octree`
        (default: the root's)."""
        if tree is not self._tree:
            self.set_tree(tree)
        lo, hi = octree if octree is not None else tree.root_octree
        self._setup = (np.ascontiguousarray(lo, np.float32)[:3].copy(), np.ascontiguousarray(hi, np.float32)[:3].copy(),
                       float(cellsize), float(isovalue), node_id)
        self._info = None

    def polygonize(self) -> None:
        lo, hi, cs, iso, _ = self._setup
        gpu._check(self._L.psgpu_gui_polygonize(self._g, lo.ctypes.data, hi.ctypes.data, cs, iso),
                   "psgpu_gui_polygonize")
        self._info = None

    def finish(self) -> PsGuiInfo:
        if self._info is None:
            info = PsGuiInfo()
            gpu._check(self._L.psgpu_gui_finish(self._g, ctypes.byref(info)), "psgpu_gui_finish")
            self._info = info
        return self._info

    def run(self) -> PsGuiInfo:
        """CParsipOptimized::run (:392-410)."""
        self.polygonize()
        return self.finish()

    # statistics (CPolyParsipOptimized.cpp:487-527, .h:278-302)
    def countMPUs(self) -> int:  # noqa: N802 (reference names)
        return self.finish().ctMPUs

    def statsIntersectedMPUs(self) -> int:  # noqa: N802
        return self.finish().ctIntersectedMPUs

    def statsMeshInfo(self):  # noqa: N802
        i = self.finish()
        return i.ctVertices, i.ctTriangles

    def statsTotalFieldEvals(self) -> int:  # noqa: N802
        return self.finish().ctFieldEvals

    def statsIntersectedCellsCount(self) -> int:  # noqa: N802
        return self.finish().ctIntersectedCells

    def statsTotalCellsInIntersectedMPUs(self) -> int:  # noqa: N802
        return self.finish().ctCellsInIntersectedMPUs

    def statsTotalCellInAllMPUs(self) -> int:  # noqa: N802
        return (GRID_DIM - 1) ** 3 * self.countMPUs()

    def exportMesh(self) -> GuiMesh:  # noqa: N802
        """exportMesh (:594-613): the MPU meshes in lattice order, mesh-wide triangle ids."""
        i = self.finish()
        V, T, N = i.ctVertices, i.ctTriangles, i.ctLatticeMPUs
        pos = np.zeros((V, 3), np.float32)
        nrm = np.zeros((V, 3), np.float32)
        col = np.zeros((V, 4), np.float32)
        tris = np.zeros((T, 3), np.uint32)
        off = np.zeros(N + 1, np.uint64)
        st = np.zeros(max(N, 1), STATS_DTYPE)
        gpu._check(self._L.psgpu_gui_download(self._g, pos.ctypes.data, nrm.ctypes.data, col.ctypes.data,
                                              tris.ctypes.data, off.ctypes.data, st.ctypes.data),
                   "psgpu_gui_download")
        return GuiMesh(pos, nrm, col, tris, (off & 0xFFFFFFFF).astype(np.int64), (off >> 32).astype(np.int64),
                       st[:N])

    @property
    def pcm_state(self) -> np.ndarray:
        """The PCM contact state (maxCompressionLeft, Right) the next run reads
        (include/parsip_gpu_gui.h: a run reads the state it started with and leaves the
        largest compression it met)."""
        s = np.zeros(2, np.float32)
        gpu._check(self._L.psgpu_gui_get_pcm_state(self._g, s.ctypes.data), "psgpu_gui_get_pcm_state")
        return s

    def set_pcm_state(self, state) -> None:
        s = np.ascontiguousarray(state, np.float32)[:2].copy()
        gpu._check(self._L.psgpu_gui_set_pcm_state(self._g, s.ctypes.data), "psgpu_gui_set_pcm_state")

    def field_values(self, xyz: np.ndarray):
        """COMPACTBLOBTREE::fieldvalue + baseColor at points: (values, rgba)."""
        xyz = np.ascontiguousarray(xyz, np.float32).reshape(-1, 3)
        out = np.zeros(len(xyz), np.float32)
        col = np.zeros((len(xyz), 4), np.float32)
        gpu._check(self._L.psgpu_gui_field_values(self._g, xyz.ctypes.data, len(xyz), out.ctypes.data,
                                                  col.ctypes.data), "psgpu_gui_field_values")
        return out, col


def Run_Polygonizer(root: bt.BlobNode, cellsize: float = 0.25, isovalue: float = ISO_VALUE,  # noqa: N802
                    device: int = 0) -> ParsipOptimized:
    """Run_Polygonizer (CPolyParsipOptimized.cpp:615-628): convert, setup over the root's
    octree, run.  Raises on a conversion error."""
    code, tree = compact_blobtree(root)
    if code < 0:
        raise gpu.PsgpuError(code, "COMPACTBLOBTREE::convert")
    p = ParsipOptimized(device)
    p.setup(tree, root.octree, root.node_id, cellsize, isovalue)
    p.run()
    return p

"""Byte-exact NumPy views of the PS_SimdPoly SoA contract (include/parsip_gpu.h).

The dtypes mirror the reference structs field for field, so ``model.prims.tobytes()``
is exactly the memory image a C++ host would hand to ``PS::SIMDPOLY::Polygonize``:

* ``SOABlobPrims``        9,500 B  -- Parsip100/PS_SimdPoly/include/PS_Polygonizer.h:98-130
* ``SOABlobOps``          5,636 B  -- PS_Polygonizer.h:134-154
* ``SOABlobPrimMatrices`` 6,148 B  -- PS_Polygonizer.h:161-165
* ``SOABlobBoxMatrices``  8,196 B  -- PS_Polygonizer.h:171-175
* ``MPU``                21,524 B  -- PS_Polygonizer.h:183-195
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

MAX_TREE_NODES = 128
PRIM_MATRIX_STRIDE = 12
BOX_MATRIX_STRIDE = 16
GRID_DIM = 8
CELLS_PER_MPU = GRID_DIM - 1
ISO_VALUE = np.float32(0.5)
ISO_DIST = np.float32(0.45420206)
MIN_CELL_SIZE = np.float32(0.01)
NORMAL_DELTA = np.float32(0.001)
MAX_MPU_COUNT = 24000
MAX_MPU_VERTEX_COUNT = 512
MAX_MPU_TRIANGLE_COUNT = 512

# Return codes (PS_Polygonizer.h:47-50 plus the library's explicit overflow codes).
RET_SUCCESS = 1
RET_PARAM_ERROR = -1
RET_NOT_ENOUGH_MEM = -2
RET_INVALID_BVH = -3
RET_MPU_OVERFLOW = -4
RET_MPU_VT_OVERFLOW = -5
RET_DEVICE_ERROR = -6


class NodeType:
    """The hot path's own enum ordering (PS_Polygonizer.h:84-91)."""

    CYLINDER, DISC, LINE, POINT, RING, POLYGON, CUBE, TRIANGLE = range(8)
    CATMULLROM, SKELETON, QUADRICPOINT, FASTQPS, HALFPLANE, NULL = range(8, 14)
    UNION, INTERSECT, DIF, SMOOTHDIF, BLEND, RICCIBLEND, GRADIENTBLEND = range(14, 21)
    AFFINE, WARPTWIST, WARPTAPER, WARPBEND, WARPSHEAR, CACHE, TEXTURE, PCM = range(21, 29)


# Caller-side codes of PS_BlobTree (_constSettings.h:26-38) -> hot-path codes.
_BLOBTREE_NAMES = [
    "POINT", "LINE", "CYLINDER", "DISC", "RING", "POLYGON", "CUBE", "TRIANGLE", "CATMULLROM",
    "SKELETON", "QUADRICPOINT", "HALFPLANE", "NULL", None,  # bntPrimInstance has no SIMD code
    "UNION", "INTERSECT", "DIF", "SMOOTHDIF", "BLEND", "RICCIBLEND", "GRADIENTBLEND",
    "FASTQPS", "PCM", "CACHE", "WARPTWIST", "WARPTAPER", "WARPBEND", "WARPSHEAR", "TEXTURE",
]


def translate_blobtree_type(code: int) -> int:
    """Map a PS_BlobTree node type (_constSettings.h:26-38) to the PS_Polygonizer.h code.

    The two enums disagree; the linearizer must translate.
    Returns -1 for codes with no SIMD counterpart (bntPrimInstance) or out of range.
    """
    if code < 0 or code >= len(_BLOBTREE_NAMES) or _BLOBTREE_NAMES[code] is None:
        return -1
    return getattr(NodeType, _BLOBTREE_NAMES[code])


def _f(name, n=MAX_TREE_NODES):
    return (name, "<f4", (n,))


PRIMS_DTYPE = np.dtype(
    [_f(n) for n in ("posX", "posY", "posZ", "dirX", "dirY", "dirZ", "resX", "resY", "resZ",
                     "colorX", "colorY", "colorZ", "vPrimBoxLoX", "vPrimBoxLoY", "vPrimBoxLoZ",
                     "vPrimBoxHiX", "vPrimBoxHiY", "vPrimBoxHiZ")]
    + [("skeletType", "u1", (MAX_TREE_NODES,)), ("idxMatrix", "u1", (MAX_TREE_NODES,)),
       ("bboxLo", "<f4", (3,)), ("bboxHi", "<f4", (3,)), ("ctPrims", "<u4")]
)
OPS_DTYPE = np.dtype(
    [("opType", "u1", (MAX_TREE_NODES,)), ("opLeftChild", "u1", (MAX_TREE_NODES,)),
     ("opRightChild", "u1", (MAX_TREE_NODES,)), ("opChildKind", "u1", (MAX_TREE_NODES,))]
    + [_f(n) for n in ("vBoxLoX", "vBoxLoY", "vBoxLoZ", "vBoxHiX", "vBoxHiY", "vBoxHiZ",
                       "resX", "resY", "resZ", "resW")]
    + [("ctOps", "<u4")]
)
PRIM_MATRICES_DTYPE = np.dtype([("matrix", "<f4", (MAX_TREE_NODES * PRIM_MATRIX_STRIDE,)),
                                ("count", "<u4")])
BOX_MATRICES_DTYPE = np.dtype([("matrix", "<f4", (MAX_TREE_NODES * BOX_MATRIX_STRIDE,)),
                               ("count", "<u4")])
MPU_DTYPE = np.dtype(
    [("vPos", "<f4", (MAX_MPU_VERTEX_COUNT * 3,)), ("vNorm", "<f4", (MAX_MPU_VERTEX_COUNT * 3,)),
     ("vColor", "<f4", (MAX_MPU_VERTEX_COUNT * 3,)), ("triangles", "<u2", (MAX_MPU_TRIANGLE_COUNT * 3,)),
     ("ctVertices", "<u2"), ("ctTriangles", "<u2"), ("bboxLo", "<f4", (3,)), ("ctFieldEvals", "<u4")]
)
MPU_STATS_DTYPE = np.dtype([("passedPrecheck", "<u4"), ("ctFieldEvals", "<u4"),
                            ("ctVertices", "<u4"), ("ctTriangles", "<u4")])
# MPUSTATS (PS_Polygonizer.h:201-207) in its LP64 layout (parsip_gpu.h PsMpuProcessStats):
# tbb_thread::id = a pthread_t, tbb::tick_count = one long long (CLOCK_REALTIME ns)
MPUSTATS_DTYPE = np.dtype([("idxThread", "<i4"), ("bIntersected", "<i4"), ("threadID", "<u8"),
                           ("tickStart", "<i8"), ("tickEnd", "<i8")])

assert PRIMS_DTYPE.itemsize == 9500
assert PRIMS_DTYPE.fields["skeletType"][1] == 9216
assert PRIMS_DTYPE.fields["ctPrims"][1] == 9496
assert OPS_DTYPE.itemsize == 5636
assert MPUSTATS_DTYPE.itemsize == 32 and MPUSTATS_DTYPE.fields["tickStart"][1] == 16
assert OPS_DTYPE.fields["vBoxLoX"][1] == 512 and OPS_DTYPE.fields["resX"][1] == 3584
assert PRIM_MATRICES_DTYPE.itemsize == 6148
assert BOX_MATRICES_DTYPE.itemsize == 8196
assert MPU_DTYPE.itemsize == 21524
assert MPU_DTYPE.fields["triangles"][1] == 18432 and MPU_DTYPE.fields["ctFieldEvals"][1] == 21520


@dataclass
class Model:
    """A linearised BlobTree: the three SoA structs the hot path consumes."""

    prims: np.ndarray      # shape (1,), PRIMS_DTYPE
    ops: np.ndarray        # shape (1,), OPS_DTYPE
    mats: np.ndarray       # shape (1,), PRIM_MATRICES_DTYPE
    boxmats: np.ndarray    # shape (1,), BOX_MATRICES_DTYPE
    name: str = "model"

    @classmethod
    def empty(cls, name: str = "model") -> "Model":
        prims = np.zeros(1, PRIMS_DTYPE)
        ops = np.zeros(1, OPS_DTYPE)
        mats = np.zeros(1, PRIM_MATRICES_DTYPE)
        boxmats = np.zeros(1, BOX_MATRICES_DTYPE)
        ident = np.eye(4, dtype=np.float32).reshape(-1)
        mats["matrix"][0, :PRIM_MATRIX_STRIDE] = ident[:PRIM_MATRIX_STRIDE]
        mats["count"][0] = 1
        boxmats["matrix"][0, :BOX_MATRIX_STRIDE] = ident
        boxmats["count"][0] = 1
        return cls(prims, ops, mats, boxmats, name)

    @property
    def ct_prims(self) -> int:
        return int(self.prims["ctPrims"][0])

    @property
    def ct_ops(self) -> int:
        return int(self.ops["ctOps"][0])

    @property
    def bbox(self):
        return (self.prims["bboxLo"][0].copy(), self.prims["bboxHi"][0].copy())

    def copy(self) -> "Model":
        return Model(self.prims.copy(), self.ops.copy(), self.mats.copy(), self.boxmats.copy(), self.name)

    def ptrs(self):
        """ctypes void pointers to the three structs (valid while self is alive)."""
        return (self.prims.ctypes.data_as(ctypes.c_void_p), self.mats.ctypes.data_as(ctypes.c_void_p),
                self.ops.ctypes.data_as(ctypes.c_void_p))


def mpu_dims(cellsize: float, lo, hi):
    """MPU lattice per axis exactly as Polygonize computes it (PS_Polygonizer.cpp:335-352)."""
    cs = np.float32(cellsize)
    dims = []
    for a in range(3):
        ext = np.float32(np.float32(hi[a]) - np.float32(lo[a]))
        cells = int(np.ceil(np.float32(ext / cs)))
        dims.append(cells // CELLS_PER_MPU + (1 if cells % CELLS_PER_MPU else 0))
    return tuple(dims)


def count_mpus(cellsize: float, lo, hi) -> int:
    """CountMPUNeeded (PS_Polygonizer.cpp:388-412)."""
    d = mpu_dims(cellsize, lo, hi)
    return d[0] * d[1] * d[2]


def mpu_origins(cellsize: float, lo, hi, begin: int = 0, end: int | None = None) -> np.ndarray:
    """MPU bboxLo in x-major order: lo + (float)i * (cellsize * 7.0f) (PS_Polygonizer.cpp:360-371)."""
    d = mpu_dims(cellsize, lo, hi)
    n = d[0] * d[1] * d[2]
    end = n if end is None else min(end, n)
    idx = np.arange(begin, end, dtype=np.int64)
    k = idx % d[2]
    j = (idx // d[2]) % d[1]
    i = idx // (d[2] * d[1])
    side = np.float32(np.float32(cellsize) * np.float32(CELLS_PER_MPU))
    out = np.empty((len(idx), 3), np.float32)
    for a, c in enumerate((i, j, k)):
        out[:, a] = np.float32(lo[a]) + c.astype(np.float32) * side
    return out

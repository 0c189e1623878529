"""TEST INFRASTRUCTURE ONLY: ctypes wrapper of the CPU restatement (psoracle.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use this
module, and only as the checker / the CPU baseline -- never as the product path.
Parity status: see psoracle.c (reference unbuildable here; pinned to the reference's
recorded C1/C2/C3 counts and its marching-cubes table; vertex bits "parity unpinned").
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from dataclasses import dataclass

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_LIBS = {}


class _ModelRef(ctypes.Structure):
    _fields_ = [("prims", ctypes.c_void_p), ("mats", ctypes.c_void_p), ("ops", ctypes.c_void_p)]


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE, "CC=gcc"], check=True)


def lib(sse_approx: bool = False, count: bool = False):
    key = "count" if count else ("sse" if sse_approx else "ieee")
    if key not in _LIBS:
        name = "libpsoracle_count.so" if count else ("libpsoracle_sse.so" if sse_approx else "libpsoracle.so")
        path = os.path.join(HERE, "_build", name)
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        vp, u32, f32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_float
        L.psor_polygonize.argtypes = [f32, vp, u32, u32, ctypes.c_int, ctypes.c_int, ctypes.POINTER(vp)]
        L.psor_polygonize.restype = ctypes.c_int
        L.psor_result_info.argtypes = [vp, ctypes.POINTER(u32), ctypes.POINTER(u32), ctypes.POINTER(u32)]
        L.psor_result_copy.argtypes = [vp, vp, vp, vp, vp, vp]
        L.psor_result_free.argtypes = [vp]
        L.psor_field_value.argtypes = [vp, vp, vp, vp, vp]
        L.psor_field_value_and_color.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp]
        L.psor_prim_field1.argtypes = [vp, u32, f32, f32, f32]
        L.psor_prim_field1.restype = f32
        L.psor_count_mpus.argtypes = [f32, vp, vp]
        L.psor_count_mpus.restype = u32
        L.psor_tritable.argtypes = [vp]
        L.psor_prepare_bboxes.argtypes = [vp, vp, vp]
        L.psor_prepare_bboxes.restype = ctypes.c_int
        L.psor_work_counts.argtypes = [vp]
        _LIBS[key] = L
    return _LIBS[key]


def _ref(model):
    p, m, o = model.ptrs()
    return _ModelRef(p, m, o)


@dataclass
class OracleMesh:
    """Per-MPU outcome + concatenated mesh in MPU order (PolyMPUs order)."""

    mpu_begin: int
    stats: np.ndarray   # (ctMPUs, 5): passed, evals, ctV, ctT, overflow
    pos: np.ndarray     # (V, 3) f32
    nrm: np.ndarray
    col: np.ndarray
    tris: np.ndarray    # (T, 3) u16, MPU-local vertex ids

    @property
    def vertex_offsets(self) -> np.ndarray:
        return np.concatenate([[0], np.cumsum(self.stats[:, 2].astype(np.int64))])

    @property
    def triangle_offsets(self) -> np.ndarray:
        return np.concatenate([[0], np.cumsum(self.stats[:, 3].astype(np.int64))])

    def global_tris(self) -> np.ndarray:
        """Triangles with global vertex ids (local id + the MPU's vertex offset)."""
        voff = self.vertex_offsets[:-1]
        per = np.repeat(voff, self.stats[:, 3].astype(np.int64))
        return self.tris.astype(np.int64) + per[:, None]


def polygonize(model, cellsize: float, mpu_begin: int = 0, mpu_end: int = 0xFFFFFFFF,
               threads: int = 1, keep: bool = True, sse_approx: bool = False,
               count: bool = False) -> OracleMesh | None:
    """``count=True`` runs the work-counting build (slower; see work_counts)."""
    L = lib(sse_approx, count)
    ref = _ref(model)
    res = ctypes.c_void_p()
    rc = L.psor_polygonize(cellsize, ctypes.byref(ref), mpu_begin, mpu_end, threads, 1 if keep else 0,
                           ctypes.byref(res))
    if rc != 1:
        raise RuntimeError(f"psor_polygonize failed: {rc}")
    try:
        n, v, t = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
        L.psor_result_info(res, ctypes.byref(n), ctypes.byref(v), ctypes.byref(t))
        stats = np.zeros((n.value, 5), np.uint32)
        if not keep:
            L.psor_result_copy(res, stats.ctypes.data, None, None, None, None)
            return OracleMesh(mpu_begin, stats, np.zeros((0, 3), np.float32), np.zeros((0, 3), np.float32),
                              np.zeros((0, 3), np.float32), np.zeros((0, 3), np.uint16))
        pos = np.zeros((v.value, 3), np.float32)
        nrm = np.zeros_like(pos)
        col = np.zeros_like(pos)
        tri = np.zeros((t.value, 3), np.uint16)
        L.psor_result_copy(res, stats.ctypes.data, pos.ctypes.data, nrm.ctypes.data, col.ctypes.data,
                           tri.ctypes.data)
        return OracleMesh(mpu_begin, stats, pos, nrm, col, tri)
    finally:
        L.psor_result_free(res)


def field_value(model, x, y, z, sse_approx: bool = False) -> np.ndarray:
    """FieldComputer::fieldValue on points grouped 4 at a time (len must be a multiple of 4)."""
    L = lib(sse_approx)
    ref = _ref(model)
    x, y, z = (np.ascontiguousarray(a, np.float32) for a in (x, y, z))
    assert len(x) % 4 == 0
    out = np.zeros(len(x), np.float32)
    for q in range(0, len(x), 4):
        L.psor_field_value(ctypes.byref(ref), x[q:].ctypes.data, y[q:].ctypes.data, z[q:].ctypes.data,
                           out[q:].ctypes.data)
    return out


def field_value_and_color(model, x, y, z):
    L = lib()
    ref = _ref(model)
    x, y, z = (np.ascontiguousarray(a, np.float32) for a in (x, y, z))
    f = np.zeros(len(x), np.float32)
    c = np.zeros((3, len(x)), np.float32)
    for q in range(0, len(x), 4):
        L.psor_field_value_and_color(ctypes.byref(ref), x[q:].ctypes.data, y[q:].ctypes.data, z[q:].ctypes.data,
                                     f[q:].ctypes.data, c[0, q:].ctypes.data, c[1, q:].ctypes.data,
                                     c[2, q:].ctypes.data)
    return f, c.T.copy()


def tritable() -> np.ndarray:
    t = np.zeros((256, 16), np.int32)
    lib().psor_tritable(t.ctypes.data)
    return t


def count_mpus(cellsize, lo, hi) -> int:
    lo = np.asarray(lo, np.float32)
    hi = np.asarray(hi, np.float32)
    return int(lib().psor_count_mpus(cellsize, lo.ctypes.data, hi.ctypes.data))


def prepare_bboxes(model) -> int:
    return lib().psor_prepare_bboxes(model.prims.ctypes.data, model.boxmats.ctypes.data, model.ops.ctypes.data)


PHASES = ("s1", "s2", "roots", "normals", "colour")


def work_counts() -> np.ndarray:
    """(5 phases x 64 slots) lane-evaluation counters of the last polygonize(count=True):
    see the t_cnt comment in psoracle.c."""
    out = np.zeros((5, 64), np.uint64)
    lib(count=True).psor_work_counts(out.ctypes.data)
    return out

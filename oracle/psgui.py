"""TEST INFRASTRUCTURE ONLY: ctypes wrapper of psgui.c, the CPU restatement of
ParsipHaptics' own polygonizer (CParsipOptimized + COMPACTBLOBTREE), the checker of the
compat mode (parsip_amd/gui.py).  Only tests/ may use it.  Parity status: see psgui.c
("parity unpinned" beyond the restatement)."""
from __future__ import annotations

import ctypes
import os
import subprocess
import sys
from dataclasses import dataclass

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from parsip_amd.gui import PsGuiInfo, STATS_DTYPE  # noqa: E402  (layouts only)

_L = None


def lib():
    global _L
    if _L is None:
        path = os.path.join(HERE, "_build", "libpsgui.so")
        if not os.path.exists(path):
            subprocess.run(["make", "-s", "-C", HERE, "CC=gcc"], check=True)
        L = ctypes.CDLL(path)
        vp, u32, f32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_float
        L.psgui_polygonize.argtypes = [vp, u32, vp, u32, vp, vp, vp, vp, f32, f32, vp, ctypes.c_int,
                                       ctypes.POINTER(vp), vp]
        L.psgui_polygonize.restype = ctypes.c_int
        L.psgui_result_info.argtypes = [vp, ctypes.POINTER(PsGuiInfo)]
        L.psgui_result_copy.argtypes = [vp, vp, vp, vp, vp, vp, vp]
        L.psgui_result_free.argtypes = [vp]
        L.psgui_field_values.argtypes = [vp, u32, vp, u32, vp, vp, vp, u32, vp, vp, vp]
        L.psgui_set_grid_dim.argtypes = [ctypes.c_int]
        L.psgui_set_grid_dim.restype = ctypes.c_int
        L.psgui_libm_agreement.argtypes = [vp, vp, u32, vp, vp]
        _L = L
    return _L


def _tri_table():
    sys.path.insert(0, HERE)
    import psoracle

    return np.ascontiguousarray(psoracle.tritable(), np.int32).reshape(256, 16)


@dataclass
class GuiOracleResult:
    info: PsGuiInfo
    pos: np.ndarray
    nrm: np.ndarray
    col: np.ndarray
    tris: np.ndarray
    mpu_v: np.ndarray
    mpu_t: np.ndarray
    stats: np.ndarray
    pcm_state: np.ndarray  # the PCM contact state the run left (left, right)


def _tree_args(tree):
    def p(a):
        return a.ctypes.data if len(a) else None
    return (p(tree.prims), len(tree.prims), p(tree.ops), len(tree.ops), p(tree.kids), p(tree.mtx))


def polygonize(tree, lo, hi, cellsize: float, isovalue: float = 0.5, threads: int = 4,
               grid_dim: int = 8, pcm_state=None) -> GuiOracleResult:
    """CParsipOptimized::setup + run on the CPU (lattice over [lo, hi]); grid_dim is the
    header's GRID_DIM (8 in this snapshot; 16 / 32 its other settings).  pcm_state: the PCM
    contact state the run reads (default ISO_VALUE, as after convert); the result carries
    the state it leaves."""
    L = lib()
    assert L.psgui_set_grid_dim(grid_dim) == 1
    lo = np.ascontiguousarray(lo, np.float32)[:3].copy()
    hi = np.ascontiguousarray(hi, np.float32)[:3].copy()
    tri = _tri_table()
    h = ctypes.c_void_p()
    pcm = np.array([0.5, 0.5] if pcm_state is None else pcm_state, np.float32)
    L.psgui_polygonize(*_tree_args(tree), lo.ctypes.data, hi.ctypes.data, cellsize, isovalue, tri.ctypes.data,
                       threads, ctypes.byref(h), pcm.ctypes.data)
    info = PsGuiInfo()
    L.psgui_result_info(h, ctypes.byref(info))
    V, T, N = info.ctVertices, info.ctTriangles, info.ctLatticeMPUs
    pos = np.zeros((V, 3), np.float32)
    nrm = np.zeros((V, 3), np.float32)
    col = np.zeros((V, 4), np.float32)
    tris = np.zeros((T, 3), np.uint32)
    off = np.zeros(N + 1, np.uint64)
    st = np.zeros(max(N, 1), STATS_DTYPE)
    L.psgui_result_copy(h, pos.ctypes.data, nrm.ctypes.data, col.ctypes.data, tris.ctypes.data, off.ctypes.data,
                        st.ctypes.data)
    L.psgui_result_free(h)
    return GuiOracleResult(info, pos, nrm, col, tris, (off & 0xFFFFFFFF).astype(np.int64),
                           (off >> 32).astype(np.int64), st[:N], pcm)


def field_values(tree, xyz, pcm_state=None):
    L = lib()
    xyz = np.ascontiguousarray(xyz, np.float32).reshape(-1, 3)
    out = np.zeros(len(xyz), np.float32)
    col = np.zeros((len(xyz), 4), np.float32)
    pcm = np.array([0.5, 0.5] if pcm_state is None else pcm_state, np.float32)
    L.psgui_field_values(*_tree_args(tree), xyz.ctypes.data, len(xyz), out.ctypes.data, col.ctypes.data,
                         pcm.ctypes.data)
    return out, col


def libm_agreement(x, y):
    """glibc powf(x, y), cosf(x), sinf(x) against the correctly rounded results the oracle
    and the device use: (differing counts, max ulp difference), each (pow, cos, sin)."""
    L = lib()
    x = np.ascontiguousarray(x, np.float32)
    y = np.ascontiguousarray(y, np.float32)
    d = np.zeros(3, np.uint32)
    u = np.zeros(3, np.uint32)
    L.psgui_libm_agreement(x.ctypes.data, y.ctypes.data, len(x), d.ctypes.data, u.ctypes.data)
    return d, u

"""ctypes binding of the C-ABI library (include/parsip_gpu.h) and the host-side mirror of
the reference's polygonizer interface.

Reference interface mirrored (Parsip100/PS_SimdPoly/include/PS_Polygonizer.h:384-393):

    U32 CountMPUNeeded(float cellsize, const svec3f& lo, const svec3f& hi);
    int PrepareBBoxes(float cellsize, SOABlobPrims&, SOABlobBoxMatrices&, SOABlobOps&);
    int Polygonize(float cellsize, const SOABlobPrims&, const SOABlobPrimMatrices&,
                   const SOABlobOps&, PolyMPUs&, MPUSTATS* = NULL);

``Polygonize`` returns the reference's codes (1 success, -1 parameter error) plus the
library's explicit -3..-6 (invalid tree, MPU capacity, per-MPU capacity, device error).
There is no CPU fallback: if the HIP library or a GPU is missing, the calls raise.
"""
from __future__ import annotations

import atexit
import ctypes
import os
import threading
import weakref
from dataclasses import dataclass

import numpy as np

from . import soa

_LIB = None
_LIVE = weakref.WeakSet()  # contexts / groups closed at interpreter exit (psgpu_destroy
                           # waits for an in-flight hiprtc compile: none may outlive the process)
LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libparsip_gpu.so")
# A/B tooling only (tools/*_ab.sh): time another build of the library from the same tree
LIB_PATH = os.environ.get("PSGPU_AB_LIB") or LIB_PATH


class PsMeshInfo(ctypes.Structure):
    _fields_ = [("ctMPUs", ctypes.c_uint32), ("ctPassedPrecheck", ctypes.c_uint32),
                ("ctSurfaceMPUs", ctypes.c_uint32), ("ctVertices", ctypes.c_uint32),
                ("ctTriangles", ctypes.c_uint32), ("firstOverflowMPU", ctypes.c_int32),
                ("ctLaneEvals", ctypes.c_uint64), ("ctFieldMPUs", ctypes.c_uint32),
                ("launchFlags", ctypes.c_uint32)]


class PsGroupPart(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int32), ("mpuBegin", ctypes.c_uint32), ("mpuEnd", ctypes.c_uint32),
                ("vertexBase", ctypes.c_uint32), ("triangleBase", ctypes.c_uint32), ("reserved", ctypes.c_uint32),
                ("info", PsMeshInfo)]


class PsMeshDevice(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in ("pos", "nrm", "col", "tris", "mpuOffsets")]


EXPORTED_SYMBOLS = [
    "psgpu_count_mpus", "psgpu_mpu_dims", "psgpu_prepare_bboxes", "psgpu_translate_blobtree_type",
    "psgpu_tritable", "psgpu_version", "psgpu_create", "psgpu_destroy", "psgpu_device_count",
    "psgpu_set_model", "psgpu_polygonize", "psgpu_finish", "psgpu_mesh_device", "psgpu_download_mesh",
    "psgpu_download_stats", "psgpu_export_polympus", "psgpu_polygonize_mpus", "psgpu_last_kernel_times",
    "psgpu_field_values", "psgpu_set_option", "psgpu_jit_active", "psgpu_jit_source", "psgpu_jit_compile",
    "psgpu_jit_pending", "psgpu_jit_wait", "psgpu_jit_tier", "psgpu_mpu_costs", "psgpu_split_costs",
    "psgpu_group_create", "psgpu_group_destroy", "psgpu_group_size", "psgpu_group_context",
    "psgpu_group_set_option", "psgpu_group_set_model", "psgpu_group_jit_wait", "psgpu_group_set_split",
    "psgpu_group_get_split", "psgpu_group_polygonize", "psgpu_group_finish", "psgpu_group_download_mesh",
    "psgpu_group_gather", "psgpu_group_export_polympus", "psgpu_group_polygonize_mpus",
    "psgpu_comm_unique_id", "psgpu_comm_create", "psgpu_comm_destroy", "psgpu_comm_exchange",
    "psgpu_comm_result", "psgpu_download_stamps", "psgpu_comm_exchange_group", "psgpu_download_spans",
    "psgpu_comm_reexchanged", "psgpu_polygonize_mpus_ex", "psgpu_download_process_stats",
    "psgpu_print_thread_results", "psgpu_thread_result_count",
]

OPT_KERNEL_TIMING = 1
OPT_CULLING = 2
OPT_JIT = 3
OPT_DEBUG = 9
OPT_VERTEX_BLOCKS_PER_CU = 4
OPT_FINISH_BLOCKS_PER_CU = 5
OPT_CAPACITY = 6
OPT_GRAPH = 7
OPT_BOUND = 10
OPT_JIT_ASYNC = 11
OPT_STAMPS = 12
OPT_SPANS = 13
OPT_FINISH_QUAD = 14
OPT_VERTEX_WIDE = 15
OPT_TREE_SPLIT = 16
OPT_SPLIT_MAX_QUEUED = 17
OPT_TIER_RUNS = 18
OPT_MPU_TICKS = 19
OPT_FUSED_SURFACE = 21
OPT_FRONT = 22
LAUNCH_TREE_SPLIT, LAUNCH_SURFACE, LAUNCH_FRONT, LAUNCH_RERUN = 1, 2, 4, 8  # PsMeshInfo.launchFlags
DEBUG_SURFACE_LATE_SCAN = 1 << 25  # test hooks of the in-kernel waits (OPT_DEBUG bits, one run each)
DEBUG_LOOKBACK_TIMEOUT = 1 << 26
DEBUG_FRONT_LATE_S1 = 1 << 27
DEBUG_EPOCH_NEAR_WRAP = 1 << 28  # test hook: the next run starts 3 runs short of the epoch's wrap
DEBUG_EXPORT_POISON = 1 << 23  # test hooks of the blocking export (OPT_DEBUG bits)
DEBUG_EXPORT_STRAGGLER = 1 << 24
JIT_INTERP, JIT_STRUCTURE, JIT_BAKED, JIT_TIERED = 0, 1, 2, 3  # OPT_JIT values
STAMP_KERNELS = ("k_precheck", "k_mpu", "k_vertex", "k_finish")
GROUP_OPT_BALANCE = 100
GROUP_OPT_MIN_PART_MPUS = 101
BLOCKING_MIN_PART_MPUS = 16384  # parsip_gpu.hpp kBlockingMinPartMpus: small lattices run as one chain
BALANCE_EVEN, BALANCE_PLAN, BALANCE_EVERY_RUN, BALANCE_FIXED = 0, 1, 2, 3
COMM_ID_BYTES = 128


def load(build_if_missing: bool = True):
    """Load libparsip_gpu.so (building it in-tree with hipcc if absent)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH) and build_if_missing:
        from .build import build
        build()
    L = ctypes.CDLL(LIB_PATH)
    vp, u32, i32, f32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int, ctypes.c_float
    sig = {
        "psgpu_count_mpus": ([f32, vp, vp], u32),
        "psgpu_mpu_dims": ([f32, vp, vp], i32),
        "psgpu_prepare_bboxes": ([f32, vp, vp, vp], i32),
        "psgpu_translate_blobtree_type": ([i32], i32),
        "psgpu_tritable": ([vp], None),
        "psgpu_version": ([], ctypes.c_char_p),
        "psgpu_create": ([i32, ctypes.POINTER(vp)], i32),
        "psgpu_destroy": ([vp], None),
        "psgpu_device_count": ([], i32),
        "psgpu_set_model": ([vp, vp, vp, vp], i32),
        "psgpu_polygonize": ([vp, f32, u32, u32, vp], i32),
        "psgpu_finish": ([vp, ctypes.POINTER(PsMeshInfo)], i32),
        "psgpu_mesh_device": ([vp, ctypes.POINTER(PsMeshDevice)], i32),
        "psgpu_download_mesh": ([vp, vp, vp, vp, vp, vp], i32),
        "psgpu_download_stats": ([vp, vp], i32),
        "psgpu_export_polympus": ([vp, vp, u32, ctypes.POINTER(u32)], i32),
        "psgpu_polygonize_mpus": ([vp, f32, vp, vp, vp, vp, u32, ctypes.POINTER(u32), vp], i32),
        "psgpu_polygonize_mpus_ex": ([vp, f32, vp, vp, vp, vp, u32, ctypes.POINTER(u32), vp, vp], i32),
        "psgpu_download_process_stats": ([vp, vp], i32),
        "psgpu_last_kernel_times": ([vp, vp, i32, vp], i32),
        "psgpu_print_thread_results": ([i32, vp, vp, u32, i32], i32),
        "psgpu_thread_result_count": ([], i32),
        "psgpu_field_values": ([vp, vp, u32, i32, vp, vp], i32),
        "psgpu_set_option": ([vp, i32, ctypes.c_int64], i32),
        "psgpu_jit_active": ([vp], i32),
        "psgpu_jit_pending": ([vp], i32),
        "psgpu_jit_wait": ([vp], i32),
        "psgpu_jit_tier": ([vp], i32),
        "psgpu_jit_source": ([vp, ctypes.c_char_p, ctypes.c_size_t], i32),
        "psgpu_jit_compile": ([vp, vp, vp, i32, ctypes.c_char_p, ctypes.c_size_t], ctypes.c_long),
        "psgpu_mpu_costs": ([vp, vp], i32),
        "psgpu_download_stamps": ([vp, vp, ctypes.POINTER(u32)], i32),
        "psgpu_download_spans": ([vp, vp, ctypes.POINTER(u32)], i32),
        "psgpu_split_costs": ([vp, u32, u32, u32, vp], i32),
        "psgpu_group_create": ([vp, i32, ctypes.POINTER(vp)], i32),
        "psgpu_group_destroy": ([vp], None),
        "psgpu_group_size": ([vp], i32),
        "psgpu_group_context": ([vp, i32], vp),
        "psgpu_group_set_option": ([vp, i32, ctypes.c_int64], i32),
        "psgpu_group_set_model": ([vp, vp, vp, vp], i32),
        "psgpu_group_jit_wait": ([vp], i32),
        "psgpu_group_set_split": ([vp, vp], i32),
        "psgpu_group_get_split": ([vp, vp], i32),
        "psgpu_group_polygonize": ([vp, f32], i32),
        "psgpu_group_finish": ([vp, ctypes.POINTER(PsMeshInfo), vp], i32),
        "psgpu_group_download_mesh": ([vp, vp, vp, vp, vp, vp], i32),
        "psgpu_group_gather": ([vp, i32, ctypes.POINTER(PsMeshDevice)], i32),
        "psgpu_group_export_polympus": ([vp, vp, u32, ctypes.POINTER(u32)], i32),
        "psgpu_group_polygonize_mpus": ([vp, f32, vp, vp, vp, vp, u32, ctypes.POINTER(u32)], i32),
        "psgpu_comm_unique_id": ([vp], i32),
        "psgpu_comm_create": ([vp, vp, i32, i32, ctypes.POINTER(vp)], i32),
        "psgpu_comm_destroy": ([vp], None),
        "psgpu_comm_exchange": ([vp, vp], i32),
        "psgpu_comm_exchange_group": ([vp, vp], i32),
        "psgpu_comm_result": ([vp, ctypes.POINTER(PsMeshInfo), vp], i32),
        "psgpu_comm_reexchanged": ([vp], i32),
    }
    for name, (args, res) in sig.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    _LIB = L
    return L


class PsgpuError(RuntimeError):
    def __init__(self, code: int, what: str):
        super().__init__(f"{what} failed with code {code}")
        self.code = code


def _check(rc: int, what: str) -> int:
    if rc != soa.RET_SUCCESS:
        raise PsgpuError(rc, what)
    return rc


# ---------------------------------------------------------------------------
# host-only helpers (no GPU needed)
def count_mpus(cellsize: float, lo, hi) -> int:
    """CountMPUNeeded (PS_Polygonizer.cpp:388-412)."""
    lo = np.ascontiguousarray(lo, np.float32)
    hi = np.ascontiguousarray(hi, np.float32)
    return int(load().psgpu_count_mpus(cellsize, lo.ctypes.data, hi.ctypes.data))


def prepare_bboxes(cellsize: float, model: soa.Model) -> int:
    """PrepareBBoxes (PS_Polygonizer.cpp:55-309), in place on the model's SoA."""
    return load().psgpu_prepare_bboxes(cellsize, model.prims.ctypes.data, model.boxmats.ctypes.data,
                                       model.ops.ctypes.data)


def tritable() -> np.ndarray:
    t = np.zeros((256, 16), np.int32)
    load().psgpu_tritable(t.ctypes.data)
    return t


def jit_compile(model: soa.Model, mode: int = 1) -> int:
    """Host-only: compile the model's specialised kernels (hiprtc); returns code size."""
    log = ctypes.create_string_buffer(1 << 16)
    n = load().psgpu_jit_compile(*model.ptrs(), mode, log, len(log))
    if n < 0:
        raise PsgpuError(n, "psgpu_jit_compile: " + log.value.decode(errors="replace"))
    return n


def device_count() -> int:
    return int(load().psgpu_device_count())


def split_costs(costs: np.ndarray, parts: int, begin: int = 0) -> np.ndarray:
    """Contiguous MPU ranges of near-equal cost (host only): bounds[0..parts]."""
    c = np.ascontiguousarray(costs, np.uint32)
    b = np.zeros(parts + 1, np.uint32)
    _check(load().psgpu_split_costs(c.ctypes.data, len(c), parts, begin, b.ctypes.data), "psgpu_split_costs")
    return b


def rank_range(costs: np.ndarray, world: int, rank: int) -> tuple[int, int]:
    """One rank's MPU range [begin, end) of the strong-scaling split (bench.py, one process
    per GPU): psgpu_split_costs of the same per-MPU costs on every rank, so the ranks agree
    without communicating."""
    b = split_costs(costs, world)
    return int(b[rank]), int(b[rank + 1])


def rebalance(costs: np.ndarray, bounds, times) -> np.ndarray:
    """One step of measured-time load balancing of a contiguous split (strong scaling): the
    per-MPU costs of rank r's range are scaled by that rank's measured time per unit of
    cost (times[r] / sum of its costs), so regions the cost model underprices (surface-heavy
    ones) weigh more, and the scaled costs are split again by psgpu_split_costs.  The inputs
    are the same on every rank (the times are all-gathered), so every rank derives the same
    new split."""
    c = np.asarray(costs, np.float64)
    b = [int(x) for x in bounds]
    scaled = np.zeros_like(c)
    for r in range(len(b) - 1):
        lo, hi = b[r], b[r + 1]
        tot = c[lo:hi].sum()
        if hi > lo and tot > 0:
            scaled[lo:hi] = c[lo:hi] * (float(times[r]) / tot)
    if scaled.sum() <= 0:
        return np.asarray(b, np.uint32)
    q = np.rint(scaled / scaled.max() * 4.0e6).astype(np.uint32)  # fixed point for the integer split
    return split_costs(np.maximum(q, 1).astype(np.uint32) if len(q) else q, len(b) - 1, b[0])


def exclusive_bases(per_rank_counts) -> np.ndarray:
    """(MPU, vertex, triangle) base of each rank's part in the global mesh from the
    all-gathered (ctMPUs, ctVertices, ctTriangles) per rank, in rank order -- the host form
    of what psgpu_comm_result derives from the RCCL all-gather."""
    c = np.asarray(per_rank_counts, np.int64).reshape(len(per_rank_counts), -1)
    return np.concatenate([np.zeros((1, c.shape[1]), np.int64), np.cumsum(c, axis=0)[:-1]])


@dataclass
class Mesh:
    """Compact mesh in the reference's MPU order (concatenation of vMPUs[i] arrays)."""

    pos: np.ndarray            # (V,3) f32
    nrm: np.ndarray            # (V,3) f32
    col: np.ndarray            # (V,3) f32
    tris: np.ndarray           # (T,3) u32 global vertex ids
    vertex_offsets: np.ndarray  # (ctMPUs+1,) per MPU of the processed range
    triangle_offsets: np.ndarray  # (ctMPUs+1,)

    def local_tris(self) -> np.ndarray:
        """Triangles with MPU-local (U16) ids, as stored in MPU::triangles."""
        per = np.repeat(self.vertex_offsets[:-1].astype(np.int64),
                        np.diff(self.triangle_offsets).astype(np.int64))
        return (self.tris.astype(np.int64) - per[:, None]).astype(np.uint16)


class Polygonizer:
    """One device context: a model in HBM and the buffers of the last polygonization."""

    def __init__(self, device: int = 0):
        L = load()
        if L.psgpu_device_count() <= device:
            raise PsgpuError(soa.RET_DEVICE_ERROR, f"no HIP device {device}")
        self._ctx = ctypes.c_void_p()
        _check(L.psgpu_create(device, ctypes.byref(self._ctx)), "psgpu_create")
        self._L = L
        self.model = None
        self.info = None
        _LIVE.add(self)

    def close(self):
        if getattr(self, "_ctx", None) and self._ctx.value:
            self._L.psgpu_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    __del__ = close

    def set_option(self, option: int, value: int) -> None:
        _check(self._L.psgpu_set_option(self._ctx, option, value), "psgpu_set_option")

    @property
    def jit_active(self) -> bool:
        return bool(self._L.psgpu_jit_active(self._ctx))

    def jit_source(self) -> str:
        n = self._L.psgpu_jit_source(self._ctx, None, 0)
        buf = ctypes.create_string_buffer(n + 1)
        self._L.psgpu_jit_source(self._ctx, buf, n + 1)
        return buf.value.decode()

    @property
    def jit_pending(self) -> bool:
        return bool(self._L.psgpu_jit_pending(self._ctx))

    def jit_wait(self) -> bool:
        """Block until the model's specialised kernels are compiled; True if they run."""
        return bool(self._L.psgpu_jit_wait(self._ctx))

    @property
    def jit_tier(self) -> int:
        """The kernels the next run uses: 0 interpreter, 1 structure-specialised, 2 baked."""
        return int(self._L.psgpu_jit_tier(self._ctx))

    def set_model(self, model: soa.Model, wait_jit: bool = True) -> None:
        """Upload a model.  The library compiles its specialised kernels on a host thread
        and serves polygonizations from the interpreter meanwhile (bit-identical output);
        ``wait_jit`` blocks until they are in place."""
        p, m, o = model.ptrs()
        _check(self._L.psgpu_set_model(self._ctx, p, m, o), "psgpu_set_model")
        self.model = model
        if wait_jit:
            self.jit_wait()

    def polygonize(self, cellsize: float, mpu_begin: int = 0, mpu_end: int | None = None,
                   stream: int | None = None) -> None:
        """Enqueue (async).  ``stream`` is a raw hipStream_t handle or None."""
        end = 0xFFFFFFFF if mpu_end is None else mpu_end
        _check(self._L.psgpu_polygonize(self._ctx, cellsize, mpu_begin, end, stream), "psgpu_polygonize")

    def finish(self) -> PsMeshInfo:
        info = PsMeshInfo()
        _check(self._L.psgpu_finish(self._ctx, ctypes.byref(info)), "psgpu_finish")
        self.info = info
        return info

    def run(self, cellsize: float, mpu_begin: int = 0, mpu_end: int | None = None) -> PsMeshInfo:
        self.polygonize(cellsize, mpu_begin, mpu_end)
        return self.finish()

    def download(self) -> Mesh:
        info = self.finish()
        V, T, N = info.ctVertices, info.ctTriangles, info.ctMPUs
        pos = np.zeros((V, 3), np.float32)
        nrm = np.zeros((V, 3), np.float32)
        col = np.zeros((V, 3), np.float32)
        tris = np.zeros((T, 3), np.uint32)
        off = np.zeros(N + 1, np.uint64)
        _check(self._L.psgpu_download_mesh(self._ctx, pos.ctypes.data, nrm.ctypes.data, col.ctypes.data,
                                           tris.ctypes.data, off.ctypes.data), "psgpu_download_mesh")
        return Mesh(pos, nrm, col, tris, (off & 0xFFFFFFFF).astype(np.int64), (off >> 32).astype(np.int64))

    def stats(self) -> np.ndarray:
        info = self.finish()
        st = np.zeros(info.ctMPUs, soa.MPU_STATS_DTYPE)
        _check(self._L.psgpu_download_stats(self._ctx, st.ctypes.data), "psgpu_download_stats")
        return st

    def export_polympus(self, capacity: int | None = None) -> np.ndarray:
        info = self.finish()
        cap = info.ctMPUs if capacity is None else capacity
        out = np.zeros(max(cap, 1), soa.MPU_DTYPE)
        ct = ctypes.c_uint32()
        _check(self._L.psgpu_export_polympus(self._ctx, out.ctypes.data, cap, ctypes.byref(ct)),
               "psgpu_export_polympus")
        return out[:ct.value]

    def polygonize_mpus(self, cellsize: float, model: soa.Model, poly_mpus: np.ndarray | None = None,
                        stats: np.ndarray | None = None, process_stats: np.ndarray | None = None):
        """psgpu_polygonize_mpus(_ex) on this context: the reference's blocking Polygonize (model
        upload, run, download and scatter into the caller's PolyMPUs).  ``process_stats``: the
        reference's MPUSTATS* (a MPUSTATS_DTYPE array of at least ctMPUs records; threadID,
        tickStart, tickEnd written).  Returns ``(code, ctMPUs, poly_mpus)``."""
        if poly_mpus is None:
            poly_mpus = np.zeros(soa.MAX_MPU_COUNT, soa.MPU_DTYPE)
        ct = ctypes.c_uint32()
        p, m, o = model.ptrs()
        # the library writes one record per MPU of the lattice (at most len(poly_mpus)): check
        # the caller's arrays hold that many (a ValueError, not an assert: -O strips asserts)
        need = min(len(poly_mpus), count_mpus(cellsize, *model.bbox))
        for name, arr, dt in (("stats", stats, soa.MPU_STATS_DTYPE), ("process_stats", process_stats, soa.MPUSTATS_DTYPE)):
            if arr is None:
                continue
            if arr.dtype != dt or not arr.flags.c_contiguous:
                raise ValueError(f"{name}: a C-contiguous {dt} array is required")
            if len(arr) < need:
                raise ValueError(f"{name}: {len(arr)} records, the lattice needs {need}")
        rc = self._L.psgpu_polygonize_mpus_ex(self._ctx, cellsize, p, m, o, poly_mpus.ctypes.data, len(poly_mpus),
                                              ctypes.byref(ct), None if stats is None else stats.ctypes.data,
                                              None if process_stats is None else process_stats.ctypes.data)
        self.model = model
        return rc, ct.value, poly_mpus

    def process_stats(self) -> np.ndarray:
        """MPUSTATS of the last run (it must have run with OPT_MPU_TICKS set)."""
        info = self.finish()
        st = np.zeros(max(info.ctMPUs, 1), soa.MPUSTATS_DTYPE)
        _check(self._L.psgpu_download_process_stats(self._ctx, st.ctypes.data), "psgpu_download_process_stats")
        return st[:info.ctMPUs]

    def device_mesh(self) -> PsMeshDevice:
        d = PsMeshDevice()
        _check(self._L.psgpu_mesh_device(self._ctx, ctypes.byref(d)), "psgpu_mesh_device")
        return d

    def mpu_costs(self) -> np.ndarray:
        """Per-MPU lane-evaluations of the last run (balances ranges across devices)."""
        info = self.finish()
        c = np.zeros(max(info.ctMPUs, 1), np.uint32)
        _check(self._L.psgpu_mpu_costs(self._ctx, c.ctypes.data), "psgpu_mpu_costs")
        return c[:info.ctMPUs]

    def plan_split(self, cellsize: float, parts: int) -> np.ndarray:
        """Cost split of the whole lattice into `parts` ranges from one full run on this
        context (deterministic: every rank computes the same split)."""
        self.run(cellsize)
        return split_costs(self.mpu_costs(), parts)

    def stamps(self) -> dict:
        """Per-wave timeline of the last run (OPT_STAMPS): kernel -> (waves, 3) uint64 array
        of start, end (100 MHz ticks), item | hw id << 32, launched waves only."""
        return _stamps(self._L, self._ctx)

    def spans(self, raw: bool = False) -> np.ndarray:
        """(runs, kernels) device-clock kernel spans in ms of the runs recorded since
        OPT_SPANS was set (kernels in STAMP_KERNELS order); raw: (runs, kernels, 2) start /
        end ticks of the 100 MHz device clock."""
        return _spans(self._L, self._ctx, raw)

    def kernel_times(self) -> dict:
        """Per-kernel hipEvent times (ms) of the last finished run (OPT_KERNEL_TIMING)."""
        return _kernel_times(self._L, self._ctx)

    def field_values(self, xyz: np.ndarray, mode: int = 0):
        """mode 0: quads of consecutive points; 1: per point; 2: per point + colour."""
        xyz = np.ascontiguousarray(xyz, np.float32).reshape(-1, 3)
        n = len(xyz)
        out = np.zeros(n, np.float32)
        col = np.zeros((n, 3), np.float32)
        _check(self._L.psgpu_field_values(self._ctx, xyz.ctypes.data, n, mode, out.ctypes.data, col.ctypes.data),
               "psgpu_field_values")
        return (out, col) if mode == 2 else out


def PrintThreadResults(ct_attempts: int, processed: np.ndarray | None = None, crossed: np.ndarray | None = None,
                       echo: bool = True) -> int:
    """PS::SIMDPOLY::PrintThreadResults (PS_Polygonizer.h:393, .cpp:414-428): per worker (here a
    device context, in the order contexts first finished a run since the last call) the MPUs
    processed and those with ctTriangles > 0, summed over every polygonization of the process,
    divided by ``ct_attempts``, written into ``processed`` / ``crossed`` (uint32 arrays, one
    entry per worker: ``thread_result_count()``), printed as the reference prints them when
    ``echo``, then cleared.  Returns the number of workers."""
    L = load()
    arrs = []
    for a in (processed, crossed):
        if a is not None and (a.dtype != np.uint32 or not a.flags.c_contiguous):
            raise ValueError("processed / crossed: C-contiguous uint32 arrays are required")
        arrs.append(a)
    cap = min([len(a) for a in arrs if a is not None], default=0)
    n = L.psgpu_print_thread_results(int(ct_attempts), None if processed is None else processed.ctypes.data,
                                     None if crossed is None else crossed.ctypes.data, cap, int(echo))
    if n < 0:
        raise PsgpuError(n, "psgpu_print_thread_results")
    return n


def thread_result_count() -> int:
    """Workers PrintThreadResults would report now."""
    return int(load().psgpu_thread_result_count())


_DEFAULT = threading.local()  # per host thread: {device: Polygonizer}, as parsip_gpu.hpp's default_context()


def Polygonize(cellsize: float, model: soa.Model, poly_mpus: np.ndarray | None = None, device: int = 0,
               stats: np.ndarray | None = None, process_stats: np.ndarray | None = None):
    """Blocking drop-in for PS::SIMDPOLY::Polygonize.

    Fills ``poly_mpus`` (a MPU_DTYPE array, default capacity MAX_MPU_COUNT as in PolyMPUs)
    and returns ``(code, ctMPUs, poly_mpus)``.  Runs on the calling thread's default context of the
    device, as parsip_gpu.hpp's psgpu::Polygonize (a 2-part group's whole call measures the
    same; DESIGN.md §4 "Blocking"); ``stats`` receives per-MPU PsMpuStats, ``process_stats``
    the reference's MPUSTATS (``lpProcessStats``, PS_Polygonizer.h:391).
    """
    if model.ct_prims == 0:
        return soa.RET_PARAM_ERROR, 0, poly_mpus
    mine = _DEFAULT.__dict__.setdefault("polys", {})
    if device not in mine:
        mine[device] = Polygonizer(device)
    return mine[device].polygonize_mpus(cellsize, model, poly_mpus, stats, process_stats)


def _mesh_from_arrays(V, T, N, fill):
    pos = np.zeros((V, 3), np.float32)
    nrm = np.zeros((V, 3), np.float32)
    col = np.zeros((V, 3), np.float32)
    tris = np.zeros((T, 3), np.uint32)
    off = np.zeros(N + 1, np.uint64)
    fill(pos, nrm, col, tris, off)
    return Mesh(pos, nrm, col, tris, (off & 0xFFFFFFFF).astype(np.int64), (off >> 32).astype(np.int64))


class Group:
    """One MPU lattice over several device contexts (psgpu_group_*): contiguous ranges of
    near-equal cost, all devices launched at once; the parts concatenate to the
    single-device mesh."""

    def __init__(self, devices):
        L = load()
        devs = (ctypes.c_int * len(devices))(*devices)
        self._g = ctypes.c_void_p()
        _check(L.psgpu_group_create(devs, len(devices), ctypes.byref(self._g)), "psgpu_group_create")
        self._L = L
        self.n = len(devices)
        _LIVE.add(self)

    def close(self):
        if getattr(self, "_g", None) and self._g.value:
            self._L.psgpu_group_destroy(self._g)
            self._g = ctypes.c_void_p()

    __del__ = close

    def set_option(self, option: int, value: int) -> None:
        _check(self._L.psgpu_group_set_option(self._g, option, value), "psgpu_group_set_option")

    def set_model(self, model: soa.Model, wait_jit: bool = True) -> None:
        _check(self._L.psgpu_group_set_model(self._g, *model.ptrs()), "psgpu_group_set_model")
        if wait_jit:
            self._L.psgpu_group_jit_wait(self._g)

    def jit_wait(self) -> bool:
        """Block until every part's specialised kernels (and a started baked compile) are in place."""
        return bool(self._L.psgpu_group_jit_wait(self._g))

    @property
    def jit_tier(self) -> int:
        """The lowest tier the parts' next runs use (0 interpreter, 1 structure, 2 baked)."""
        L = self._L
        return min(int(L.psgpu_jit_tier(L.psgpu_group_context(self._g, i))) for i in range(self.n))

    def set_split(self, bounds) -> None:
        b = np.ascontiguousarray(bounds, np.uint32)
        assert len(b) == self.n + 1
        _check(self._L.psgpu_group_set_split(self._g, b.ctypes.data), "psgpu_group_set_split")

    def split(self) -> np.ndarray:
        b = np.zeros(self.n + 1, np.uint32)
        _check(self._L.psgpu_group_get_split(self._g, b.ctypes.data), "psgpu_group_get_split")
        return b

    def polygonize(self, cellsize: float) -> None:
        _check(self._L.psgpu_group_polygonize(self._g, cellsize), "psgpu_group_polygonize")

    def finish(self):
        info = PsMeshInfo()
        parts = (PsGroupPart * self.n)()
        _check(self._L.psgpu_group_finish(self._g, ctypes.byref(info), parts), "psgpu_group_finish")
        return info, list(parts)

    def run(self, cellsize: float):
        self.polygonize(cellsize)
        return self.finish()

    def download(self) -> Mesh:
        info, _ = self.finish()

        def fill(pos, nrm, col, tris, off):
            _check(self._L.psgpu_group_download_mesh(self._g, pos.ctypes.data, nrm.ctypes.data, col.ctypes.data,
                                                     tris.ctypes.data, off.ctypes.data), "psgpu_group_download_mesh")
        return _mesh_from_arrays(info.ctVertices, info.ctTriangles, info.ctMPUs, fill)

    def gather(self, dst_part: int = 0) -> PsMeshDevice:
        d = PsMeshDevice()
        _check(self._L.psgpu_group_gather(self._g, dst_part, ctypes.byref(d)), "psgpu_group_gather")
        return d

    def export_polympus(self, capacity: int | None = None) -> np.ndarray:
        info, _ = self.finish()
        cap = info.ctMPUs if capacity is None else capacity
        out = np.zeros(max(cap, 1), soa.MPU_DTYPE)
        ct = ctypes.c_uint32()
        _check(self._L.psgpu_group_export_polympus(self._g, out.ctypes.data, cap, ctypes.byref(ct)),
               "psgpu_group_export_polympus")
        return out[:ct.value]

    def polygonize_mpus(self, cellsize: float, model: soa.Model, poly_mpus: np.ndarray | None = None):
        """psgpu_group_polygonize_mpus: the reference's blocking Polygonize over the group's
        parts (model upload, run, download and scatter into the caller's PolyMPUs).
        Returns ``(code, ctMPUs, poly_mpus)``."""
        if poly_mpus is None:
            poly_mpus = np.zeros(soa.MAX_MPU_COUNT, soa.MPU_DTYPE)
        ct = ctypes.c_uint32()
        p, m, o = model.ptrs()
        rc = self._L.psgpu_group_polygonize_mpus(self._g, cellsize, p, m, o, poly_mpus.ctypes.data, len(poly_mpus),
                                                 ctypes.byref(ct))
        return rc, ct.value, poly_mpus

    def context_ptr(self, part: int):
        return self._L.psgpu_group_context(self._g, part)

    def kernel_times(self, part: int) -> dict:
        """Per-kernel hipEvent times (ms) of part `part` in the last finished run."""
        return _kernel_times(self._L, ctypes.c_void_p(self.context_ptr(part)))

    def spans(self, part: int, raw: bool = False) -> np.ndarray:
        """Recorded kernel spans (OPT_SPANS) of part `part`: (runs, kernels) in ms (raw: start / end ticks)."""
        return _spans(self._L, ctypes.c_void_p(self.context_ptr(part)), raw)

    def stamps(self, part: int) -> dict:
        """The per-wave timeline (OPT_STAMPS) of part `part` in the last finished run."""
        return _stamps(self._L, ctypes.c_void_p(self.context_ptr(part)))


def _stamps(L, ctx) -> dict:
    cap = ctypes.c_uint32()
    _check(L.psgpu_download_stamps(ctx, None, ctypes.byref(cap)), "psgpu_download_stamps")
    n = max(cap.value, 1)
    raw = np.zeros(len(STAMP_KERNELS) * n * 3 + n * 8, np.uint64)
    _check(L.psgpu_download_stamps(ctx, raw.ctypes.data, ctypes.byref(cap)), "psgpu_download_stamps")
    buf = raw[:len(STAMP_KERNELS) * n * 3].reshape(len(STAMP_KERNELS), n, 3)
    out = {k: buf[i][buf[i][:, 0] != 0] for i, k in enumerate(STAMP_KERNELS)}
    out["mpu_phases"] = raw[len(STAMP_KERNELS) * n * 3:].reshape(n, 8)
    return out


def _spans(L, ctx, raw: bool = False) -> np.ndarray:
    runs = ctypes.c_uint32()
    _check(L.psgpu_download_spans(ctx, None, ctypes.byref(runs)), "psgpu_download_spans")
    out = np.zeros((max(runs.value, 1), len(STAMP_KERNELS), 2), np.uint64)
    _check(L.psgpu_download_spans(ctx, out.ctypes.data, ctypes.byref(runs)), "psgpu_download_spans")
    out = out[:runs.value].astype(np.int64)
    if raw:  # (runs, kernels, {first wave start, last wave end}) in 100 MHz device ticks
        return out
    return (out[:, :, 1] - out[:, :, 0]) * 1e-5  # (runs, kernels) in ms (100 MHz ticks)


def kernel_spans(stamps: dict, front: bool = False) -> dict:
    """Per kernel, first wave start -> last wave end (ms, device clock) of one run; front: the
    run's S1 and S2 waves were one launch (k_front, PsMeshInfo.launchFlags), whose span is added."""
    out = {}
    for k in STAMP_KERNELS:
        st = stamps.get(k)
        if st is not None and len(st):
            out[k] = float(int(st[:, 1].max()) - int(st[:, 0].min())) * 1e-5  # 100 MHz ticks -> ms
    if front:
        st = [stamps[k] for k in ("k_precheck", "k_mpu") if stamps.get(k) is not None and len(stamps[k])]
        if st:
            out["k_front"] = float(max(int(x[:, 1].max()) for x in st) - min(int(x[:, 0].min()) for x in st)) * 1e-5
    return out


def _kernel_times(L, ctx) -> dict:
    ms = (ctypes.c_float * 8)()
    names = (ctypes.c_char_p * 8)()
    n = L.psgpu_last_kernel_times(ctx, ms, 8, names)
    return {names[i].decode(): ms[i] for i in range(n)}


def comm_unique_id() -> bytes:
    buf = (ctypes.c_uint8 * COMM_ID_BYTES)()
    _check(load().psgpu_comm_unique_id(buf), "psgpu_comm_unique_id")
    return bytes(buf)


class Comm:
    """RCCL count exchange of one rank's polygonization (one process per GPU)."""

    def __init__(self, poly, uid: bytes, nranks: int, rank: int):
        """poly: the rank's Polygonizer, or a Group of parts on the rank's one device."""
        assert len(uid) == COMM_ID_BYTES
        self._L = load()
        self._poly = poly
        self._group = poly if isinstance(poly, Group) else None
        ctx = ctypes.c_void_p(poly.context_ptr(0)) if self._group else poly._ctx
        self.nranks = nranks
        buf = (ctypes.c_uint8 * COMM_ID_BYTES).from_buffer_copy(uid)
        self._c = ctypes.c_void_p()
        _check(self._L.psgpu_comm_create(ctx, buf, nranks, rank, ctypes.byref(self._c)), "psgpu_comm_create")

    def close(self):
        if getattr(self, "_c", None) and self._c.value:
            self._L.psgpu_comm_destroy(self._c)
            self._c = ctypes.c_void_p()

    __del__ = close

    def exchange(self) -> None:
        if self._group:
            _check(self._L.psgpu_comm_exchange_group(self._c, self._group._g), "psgpu_comm_exchange_group")
        else:
            _check(self._L.psgpu_comm_exchange(self._c, self._poly._ctx), "psgpu_comm_exchange")

    def result(self):
        info = PsMeshInfo()
        parts = (PsGroupPart * self.nranks)()
        _check(self._L.psgpu_comm_result(self._c, ctypes.byref(info), parts), "psgpu_comm_result")
        return info, list(parts)

    def reexchanged(self) -> bool:
        """Whether the last result() needed the second, collectively agreed exchange."""
        return bool(self._L.psgpu_comm_reexchanged(self._c))


@atexit.register
def _close_live():
    for obj in list(_LIVE):
        try:
            obj.close()
        except Exception:  # noqa: BLE001 (best effort at exit)
            pass

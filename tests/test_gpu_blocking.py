"""The blocking drop-in (psgpu_polygonize_mpus = PS::SIMDPOLY::Polygonize, PS_Polygonizer.h:
386-391, .cpp:315-385) under adversarial conditions, and its MPUSTATS (.h:201-207).

The export packs the mesh on the device and writes it straight into pinned host memory piece
by piece; the host scatters a piece into PolyMPUs once every packing block has raised its
flag for it (DESIGN.md §4 "Blocking").  These tests run a C3 -> C2 -> C1 -> C3 sequence on one
context (the staging keeps its size, the mesh shrinks and grows under it) with two test hooks:
every staging word past the flags holds the call's own epoch before the export (any word a
flag check could mistake for "done" is one), and the last packing block arrives ~40 us late
on every piece (the race window made wide).  Every PolyMPUs must still hash to the committed
oracle digests (tests/golden/oracle_digests.json), so the scatter never read a share before
it landed.
"""
import json
import os
import subprocess

import numpy as np
import pytest

from parity_util import mesh_digests
from parsip_amd import gpu, soa, synth

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DIGESTS = json.load(open(os.path.join(ROOT, "tests", "golden", "oracle_digests.json")))


def polympus_digests(mpus: np.ndarray, stats: np.ndarray) -> dict:
    """The committed digest form of a PolyMPUs export (MPU order, MPU-local U16 triangles)."""
    nv = mpus["ctVertices"].astype(np.int64)
    nt = mpus["ctTriangles"].astype(np.int64)
    pos = np.concatenate([mpus["vPos"][i, :3 * nv[i]] for i in range(len(mpus))]).reshape(-1, 3)
    nrm = np.concatenate([mpus["vNorm"][i, :3 * nv[i]] for i in range(len(mpus))]).reshape(-1, 3)
    col = np.concatenate([mpus["vColor"][i, :3 * nv[i]] for i in range(len(mpus))]).reshape(-1, 3)
    tri = np.concatenate([mpus["triangles"][i, :3 * nt[i]] for i in range(len(mpus))]).reshape(-1, 3)
    st4 = np.stack([stats["passedPrecheck"], stats["ctFieldEvals"], stats["ctVertices"], stats["ctTriangles"]], 1)
    return mesh_digests(st4, pos, nrm, col, tri)


SEQUENCE = ("C3", "C2", "C1", "C3")


def _blocking_sequence(poly_mpus_call, sequence=SEQUENCE):
    for name in sequence:
        model, cs, _ = synth.make_config(name)
        n = gpu.count_mpus(cs, *model.bbox)
        mpus = np.zeros(n, soa.MPU_DTYPE)
        stats = np.zeros(n, soa.MPU_STATS_DTYPE)
        rc, ct = poly_mpus_call(cs, model, mpus, stats)
        assert rc == soa.RET_SUCCESS and ct == n, (name, rc, ct)
        assert polympus_digests(mpus, stats) == DIGESTS[name], name
        assert int(mpus["ctFieldEvals"].astype(bool).sum()) == DIGESTS[name]["passed_s1"]


def test_blocking_export_poisoned_staging_and_straggler_sequence():
    """One context, C3 -> C2 -> C1 -> C3 with the staging poisoned with each call's epoch and a
    straggling packing block: every PolyMPUs equals the oracle digests."""
    p = gpu.Polygonizer(0)
    try:
        p.set_option(gpu.OPT_DEBUG, gpu.DEBUG_EXPORT_POISON | gpu.DEBUG_EXPORT_STRAGGLER)

        def call(cs, model, mpus, stats):
            rc, ct, _ = p.polygonize_mpus(cs, model, mpus, stats)
            return rc, ct
        _blocking_sequence(call)
        # and once more without the hooks, on the same (now shrunken-and-regrown) staging
        p.set_option(gpu.OPT_DEBUG, 0)
        _blocking_sequence(call, ("C1", "C3"))
    finally:
        p.close()


def test_group_blocking_export_poisoned_sequence():
    """The same on a 2-part group of one device (each part's export has its own staging and
    flags; the parts' packing kernels queue in range order)."""
    g = gpu.Group([0, 0])
    try:
        g.set_option(gpu.GROUP_OPT_BALANCE, gpu.BALANCE_PLAN)
        g.set_option(gpu.OPT_DEBUG, gpu.DEBUG_EXPORT_POISON | gpu.DEBUG_EXPORT_STRAGGLER)
        L = gpu.load()

        def call(cs, model, mpus, stats):
            rc, ct, _ = g.polygonize_mpus(cs, model, mpus)
            if rc != soa.RET_SUCCESS:
                return rc, ct
            at = 0  # PsMpuStats per part through the C-ABI
            for k in range(g.n):
                info, parts = g.finish()
                m = parts[k].info.ctMPUs
                st = np.zeros(max(m, 1), soa.MPU_STATS_DTYPE)
                assert L.psgpu_download_stats(g.context_ptr(k), st.ctypes.data) == soa.RET_SUCCESS
                stats[at:at + m] = st[:m]
                at += m
            assert at == ct
            return rc, ct
        _blocking_sequence(call, ("C3", "C1", "C3"))
    finally:
        g.close()


def test_mpustats_filled_like_the_reference():
    """MPUSTATS (PS_Polygonizer.h:201-207): CMPUProcessor writes threadID, tickStart and tickEnd
    of every MPU (.cpp:449-461) and leaves idxThread / bIntersected alone.  Ticks are host
    CLOCK_REALTIME nanoseconds (legacy tbb::tick_count) inside the call, tickEnd >= tickStart for
    every MPU; MPUs with a surface finish in k_mpu, after every S1-only MPU."""
    model, cs, _ = synth.make_config("C2")
    n = gpu.count_mpus(cs, *model.bbox)
    p = gpu.Polygonizer(0)
    try:
        # without MPUSTATS no ticks are recorded, and asking for them is an error, not a no-op
        rc, ct, _ = p.polygonize_mpus(cs, model, np.zeros(n, soa.MPU_DTYPE))
        assert rc == soa.RET_SUCCESS
        with pytest.raises(gpu.PsgpuError):
            p.process_stats()
        mpus = np.zeros(n, soa.MPU_DTYPE)
        stats = np.zeros(n, soa.MPU_STATS_DTYPE)
        ps = np.zeros(n, soa.MPUSTATS_DTYPE)
        ps["idxThread"] = -7
        ps["bIntersected"] = np.arange(n)
        import time
        t0 = time.clock_gettime_ns(time.CLOCK_REALTIME)
        rc, ct, _ = p.polygonize_mpus(cs, model, mpus, stats, ps)
        t1 = time.clock_gettime_ns(time.CLOCK_REALTIME)
        assert rc == soa.RET_SUCCESS and ct == n
        assert polympus_digests(mpus, stats) == DIGESTS["C2"]  # the ticks change no output
        assert (ps["idxThread"] == -7).all() and (ps["bIntersected"] == np.arange(n)).all()
        slack = 50_000  # ns: the device-to-host clock mapping is good to a few microseconds
        assert (ps["tickStart"] >= t0 - slack).all() and (ps["tickEnd"] <= t1 + slack).all()
        assert (ps["tickEnd"] >= ps["tickStart"]).all()
        passed = stats["passedPrecheck"] != 0
        assert (ps["tickEnd"][passed] >= ps["tickStart"][passed]).all()
        surf = stats["ctVertices"] > 0
        assert surf.any() and (~passed).any()
        assert ps["tickEnd"][surf].min() > ps["tickEnd"][~passed].max()  # k_mpu after k_precheck
        xcc = (ps["threadID"] >> 16).astype(np.int64)
        assert (xcc < 8).all() and (ps["threadID"] < (1 << 20)).all()
        assert len(np.unique(ps["threadID"])) > 64  # spread over the chip's wave slots
        # the option form: ticks of a plain run on the context
        p.set_option(gpu.OPT_MPU_TICKS, 1)
        p.run(cs)
        again = p.process_stats()
        assert (again["tickEnd"] >= again["tickStart"]).all() and again["tickStart"].min() > ps["tickEnd"].max()
    finally:
        p.close()


def test_cpp_ps_simdpoly_polygonize_mpustats(tmp_path):
    """PS::SIMDPOLY::Polygonize(cs, prims, mats, ops, polyMPUs, lpProcessStats) compiled against a
    caller-side MPUSTATS whose thread id and ticks are opaque classes, as TBB's."""
    import shutil
    gpp = shutil.which("g++")
    if gpp is None:
        pytest.skip("no g++")
    gpu.load()
    exe = tmp_path / "simdpoly_check"
    lib_dir = os.path.join(ROOT, "parsip_amd")
    subprocess.run([gpp, "-std=c++17", "-O1", "-Wall", "-Wextra", "-I", os.path.join(ROOT, "include"),
                    "-I", os.path.join(ROOT, "tests", "cpp"), os.path.join(ROOT, "tests", "cpp", "simdpoly_check.cpp"),
                    "-L", lib_dir, "-l:libparsip_gpu.so", f"-Wl,-rpath,{lib_dir}", "-o", str(exe)], check=True)
    model, cs, _ = synth.make_config("C2")
    src, out = tmp_path / "soa.bin", tmp_path / "stats.bin"
    with open(src, "wb") as f:
        f.write(model.prims.tobytes() + model.mats.tobytes() + model.ops.tobytes() + model.boxmats.tobytes())
    r = subprocess.run([str(exe), "soa-stats", str(src), repr(float(cs)), str(out)], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    raw = open(out, "rb").read()
    rc, ct = np.frombuffer(raw[:8], np.int32)
    t0, t1 = np.frombuffer(raw[8:24], np.int64)
    assert rc == soa.RET_SUCCESS and ct == 6859
    ps = np.frombuffer(raw[24:], soa.MPUSTATS_DTYPE)
    assert len(ps) == ct
    assert (ps["idxThread"] == -7).all() and (ps["bIntersected"] == np.arange(ct)).all()
    assert (ps["tickEnd"] >= ps["tickStart"]).all()
    assert (ps["tickStart"] >= t0 - 50_000).all() and (ps["tickEnd"] <= t1 + 50_000).all()


def test_blocking_export_fuzz_sequence(oracle):
    """The blocking export over the fuzz trees (tests/test_gpu_fuzz.py: every node type, cell
    sizes off the round values) on one context, one after the other -- the mesh and the
    lattice shrink and grow under the same staging -- with both test hooks on: every PolyMPUs
    equals the live oracle's output for its tree."""
    import test_gpu_fuzz as fz

    p = gpu.Polygonizer(0)
    try:
        p.set_option(gpu.OPT_DEBUG, gpu.DEBUG_EXPORT_POISON | gpu.DEBUG_EXPORT_STRAGGLER)
        for seed in range(0, 40, 3):
            model, cs = fz.fuzz_case(seed)[:2]
            n = gpu.count_mpus(cs, *model.bbox)
            mpus = np.zeros(n, soa.MPU_DTYPE)
            stats = np.zeros(n, soa.MPU_STATS_DTYPE)
            rc, ct, _ = p.polygonize_mpus(cs, model, mpus, stats)
            om = oracle.polygonize(model, cs, 0, 0xFFFFFFFF, threads=8)
            if rc == soa.RET_MPU_VT_OVERFLOW:  # an MPU past the reference's 512 V / T
                assert (om.stats[:, 2:4] > 512).any(), seed
                continue
            assert rc == soa.RET_SUCCESS and ct == n, (seed, rc, ct)
            want = mesh_digests(om.stats[:, :4], om.pos, om.nrm, om.col, om.tris)
            assert polympus_digests(mpus, stats) == want, seed
    finally:
        p.close()

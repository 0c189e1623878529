"""The C-ABI library on the host (no GPU): it loads, exports every entry point the
header declares, its host-only helpers agree with the oracle / the reference layout, and
the run-time specialised kernels compile.  No compute call needs a device here."""
import glob
import os
import re
import subprocess
import sys

import numpy as np
import pytest

from parsip_amd import gpu, soa, synth
from parsip_amd.soa import NodeType

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    names = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        txt = re.sub(r"/\*.*?\*/|//[^\n]*", "", open(h).read(), flags=re.S)
        names.update(re.findall(r"\b(psgpu_[a-z0-9_]+)\s*\(", txt))
    return sorted(names)


def test_library_exports_every_header_symbol():
    L = gpu.load()
    names = header_functions()
    assert len(names) >= 20
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    from parsip_amd import gui

    assert set(gpu.EXPORTED_SYMBOLS) | set(gui.EXPORTED_SYMBOLS) == set(names)


def test_version_string():
    v = gpu.load().psgpu_version().decode()
    assert "gfx950" in v


def test_soa_layout_matches_reference_sizes():
    """PS_Polygonizer.h structs, byte-exact (SURVEY.md §8(b) [probe] sizeof/offsetof)."""
    assert soa.PRIMS_DTYPE.itemsize == 9500
    assert soa.OPS_DTYPE.itemsize == 5636
    assert soa.PRIM_MATRICES_DTYPE.itemsize == 6148
    assert soa.BOX_MATRICES_DTYPE.itemsize == 8196
    assert soa.MPU_DTYPE.itemsize == 21524
    f = soa.PRIMS_DTYPE.fields
    assert f["skeletType"][1] == 9216 and f["idxMatrix"][1] == 9344
    assert f["bboxLo"][1] == 9472 and f["ctPrims"][1] == 9496
    o = soa.OPS_DTYPE.fields
    assert o["vBoxLoX"][1] == 512 and o["resX"][1] == 3584 and o["ctOps"][1] == 5632
    m = soa.MPU_DTYPE.fields
    assert (m["vNorm"][1], m["vColor"][1], m["triangles"][1]) == (6144, 12288, 18432)
    assert (m["ctVertices"][1], m["ctTriangles"][1], m["bboxLo"][1], m["ctFieldEvals"][1]) == \
        (21504, 21506, 21508, 21520)


def test_tritable_equals_oracle(oracle):
    np.testing.assert_array_equal(gpu.tritable(), oracle.tritable())


def test_count_mpus_equals_oracle(oracle):
    rng = np.random.default_rng(1)
    for _ in range(100):
        lo = rng.uniform(-5, 0, 3).astype(np.float32)
        hi = (lo + rng.uniform(0.1, 9, 3)).astype(np.float32)
        cs = float(np.float32(rng.uniform(0.01, 0.3)))
        assert gpu.count_mpus(cs, lo, hi) == oracle.count_mpus(cs, lo, hi)


def test_prepare_bboxes_equals_oracle(oracle):
    types = [NodeType.POINT, NodeType.LINE, NodeType.CYLINDER, NodeType.CUBE, NodeType.DISC,
             NodeType.RING, NodeType.TRIANGLE]
    for seed in range(6):
        m = synth.random_model(seed, 4 + 3 * seed, types=types, matrices=seed % 2 == 1)
        a, b = m.copy(), m.copy()
        assert oracle.prepare_bboxes(a) == 1
        assert gpu.prepare_bboxes(0.05, b) == 1
        assert a.prims.tobytes() == b.prims.tobytes()
        assert a.ops.tobytes() == b.ops.tobytes()


def test_translate_blobtree_type():
    """_constSettings.h codes -> PS_Polygonizer.h codes (SURVEY.md §8(b) Enum row)."""
    L = gpu.load()
    expect = {0: NodeType.POINT, 1: NodeType.LINE, 2: NodeType.CYLINDER, 3: NodeType.DISC, 4: NodeType.RING,
              14: NodeType.UNION, 15: NodeType.INTERSECT, 16: NodeType.DIF, 17: NodeType.SMOOTHDIF,
              18: NodeType.BLEND, 19: NodeType.RICCIBLEND, 20: NodeType.GRADIENTBLEND, 24: NodeType.WARPTWIST,
              13: -1, -1: -1, 99: -1}
    for code, want in expect.items():
        assert L.psgpu_translate_blobtree_type(code) == want == soa.translate_blobtree_type(code), code
    for code in range(-2, 40):
        assert L.psgpu_translate_blobtree_type(code) == soa.translate_blobtree_type(code)


def test_mpu_dims_and_limits():
    L = gpu.load()
    m, cs, n = synth.make_config("C3")
    dims = np.zeros(3, np.uint32)
    assert L.psgpu_mpu_dims(cs, m.prims.ctypes.data, dims.ctypes.data) == 1
    assert tuple(dims) == soa.mpu_dims(cs, *m.bbox) == (37, 37, 37)


def test_no_device_fails_loudly():
    """Without a visible GPU the product path raises; there is no CPU fallback."""
    if gpu.device_count() > 0:
        pytest.skip("a device is visible")
    with pytest.raises(gpu.PsgpuError):
        gpu.Polygonizer(0)


def test_print_thread_results_host_contract(capfd):
    """PrintThreadResults' host side: ctAttempts <= 0 is a parameter error (the reference
    divides by it) and clears nothing; with no polygonization since the last call there is no
    worker entry, nothing is written or printed."""
    L = gpu.load()
    assert L.psgpu_print_thread_results(0, None, None, 0, 1) == soa.RET_PARAM_ERROR
    assert L.psgpu_print_thread_results(-3, None, None, 0, 1) == soa.RET_PARAM_ERROR
    if gpu.device_count() > 0:
        gpu.PrintThreadResults(1, echo=False)  # clear what earlier GPU tests of this process left
    assert gpu.thread_result_count() == 0
    p = np.full(4, 7, np.uint32)
    assert gpu.PrintThreadResults(3, p, None) == 0
    assert (p == 7).all()
    assert "Thread#" not in capfd.readouterr().out
    with pytest.raises(ValueError):
        gpu.PrintThreadResults(1, np.zeros(4, np.int64))


def test_bench_ranks_end_together_without_devices():
    """`bench.py --gpus 2` spawns its ranks; a rank without a HIP device exits with a
    message, and the parent ends the other ranks instead of leaving them in the rendezvous."""
    import subprocess
    import sys

    if gpu.device_count() > 0:
        pytest.skip("a device is visible")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "PSGPU_BENCH_DEVICE")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0"],
                       env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "needs HIP device" in r.stderr
    assert r.stdout == ""


def test_invalid_trees_rejected():
    """The walk-program builder rejects what the reference adapter rejects (-3)."""
    m, cs, _ = synth.make_config("C2")
    bad = m.copy()
    bad.ops["opLeftChild"][0, 1] = 0  # cycle back to the root
    bad.ops["opChildKind"][0, 1] |= 2
    with pytest.raises(gpu.PsgpuError) as e:
        gpu.jit_compile(bad, 1)
    assert e.value.code == soa.RET_INVALID_BVH


@pytest.mark.parametrize("mode", [1, 2])
def test_jit_compiles_c3(mode):
    """hiprtc specialisation of the C3 tree compiles for gfx950 without a device."""
    m, _, _ = synth.make_config("C3")
    assert gpu.jit_compile(m, mode) > 10000


def test_generated_kernels_resources():
    """Registers, LDS and scratch of C3's generated kernels (tools/kernel_resources.py, the
    code object's metadata; DESIGN.md §4 "Round 5: occupancy"): no spills, no scratch, and
    the occupancy each hot kernel was measured at -- a change that costs a wave per SIMD
    shows up here before it reaches a GPU."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import kernel_resources as kr

    ks = kr.compile_variant("C3", 1 | 4, {})
    floor = {"jit_precheck": 7, "jit_mpu": 6, "jit_vertex": 8, "jit_vertex_w": 8, "jit_finish": 7,
             "jit_finish_p": 7, "jit_finish_q": 6, "jit_precheck_s": 7, "jit_mpu_s": 7, "jit_surface": 6}
    for name, want in floor.items():
        r = ks[name]
        # k_surface (two walks in one kernel) sits at the SGPR ceiling and spills a few SGPRs
        # into VGPR lanes (v_writelane / v_readlane, no scratch); it was measured with them
        sgpr_ok = r["sgpr_spill"] <= (16 if name == "jit_surface" else 0)
        assert r["scratch"] == 0 and r["vgpr_spill"] == 0 and sgpr_ok, (name, r)
        assert r["waves_per_simd"] >= want, (name, r["waves_per_simd"], r["limited_by"], r["vgpr"], r["sgpr"])
    # k_surface reads the offsets its own scan blocks wrote with no acquire (an agent-scope
    # acquire invalidates the XCD's L2 on gfx950): the 64-bit agent-scope loads must keep the
    # sc1 bit that sends them past the non-coherent caches -- the look-back's, and the offsets
    # reads of the vertex and triangle passes (surface_offs); k_vertex has the look-back's only
    assert ks["jit_surface"]["load_x2_sc1"] >= 3, ks["jit_surface"]
    assert ks["jit_vertex"]["load_x2_sc1"] >= 1, ks["jit_vertex"]
    # k_front's hand-off (MI355X_MICROARCH.md's table, first row) needs every byte stored and loaded
    # sc1: entry, the mask's two words and the ready word on each side, and the poll loads
    for k in ("jit_front", "jit_front_s"):
        assert ks[k]["store_sc1"] >= 4 and ks[k]["load_sc1"] >= 5 and ks[k]["load_x2_sc1"] >= 2, (k, ks[k])


_JIT_TREES = r"""
import os, sys
sys.path.insert(0, os.environ["PSGPU_ROOT"])
from parsip_amd import gpu, synth
from parsip_amd.soa import NodeType
ops = [NodeType.BLEND, NodeType.UNION, NodeType.INTERSECT, NodeType.DIF, NodeType.SMOOTHDIF,
       NodeType.RICCIBLEND, NodeType.WARPTWIST, NodeType.WARPTAPER, NodeType.WARPBEND, NodeType.WARPSHEAR]
types = [NodeType.POINT, NodeType.LINE, NodeType.CYLINDER, NodeType.CUBE, NodeType.DISC, NodeType.RING,
         NodeType.TRIANGLE]
for seed, n in ((1, 6), (2, 17), (3, 40)):
    m = synth.random_model(seed, n, types=types, op_types=ops, matrices=seed % 2 == 1)
    assert gpu.jit_compile(m, 2) > 1000, seed
print("ok")
"""


def test_baked_tier_compiles_random_trees_in_process_safe_flags(tmp_path):
    """The baked tier compiles on a host thread of the caller's process, so its flags must
    never crash hiprtc: random trees with every primitive and operator type compile with the
    default flags (LLVM's default scheduler; r03's experimental strategies crashed hiprtc),
    in a child process so a crash fails this test instead of the runner."""
    env = dict(os.environ, PSGPU_ROOT=ROOT, PSGPU_JIT_CACHE=str(tmp_path / "jitcache"))
    env.pop("PSGPU_JIT_BAKED_FLAGS", None)
    r = subprocess.run([sys.executable, "-c", _JIT_TREES], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), (r.returncode, r.stderr[-2000:])


def test_cpp_shim_compiles_and_runs(tmp_path):
    """include/parsip_gpu.hpp against caller-side SoA types: host-only entry points work
    and Polygonize fails loudly (-6) without a device, or reports the too-small
    PolyMPUs capacity (-4) with one."""
    import shutil
    import subprocess

    gpp = shutil.which("g++")
    if gpp is None:
        pytest.skip("no g++")
    gpu.load()
    exe = tmp_path / "shim_check"
    lib_dir = os.path.join(ROOT, "parsip_amd")
    subprocess.run([gpp, "-std=c++17", "-O1", "-Wall", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "shim_check.cpp"), "-L", lib_dir, "-l:libparsip_gpu.so",
                    f"-Wl,-rpath,{lib_dir}", "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr


def test_export_thread_pool(tmp_path):
    """The blocking export's scatter threads (psgpu_pool.h): every task of every run exactly
    once, run returns only after all, with the workers spinning or asleep."""
    import shutil
    import subprocess

    gpp = shutil.which("g++")
    if gpp is None:
        pytest.skip("no g++")
    exe = tmp_path / "pool_check"
    subprocess.run([gpp, "-std=c++17", "-O2", "-Wall", "-pthread", "-I", os.path.join(ROOT, "parsip_amd", "csrc"),
                    os.path.join(ROOT, "tests", "cpp", "pool_check.cpp"), "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stdout + r.stderr

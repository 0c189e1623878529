"""The C++ drop-in faces (include/parsip_gpu.hpp, include/parsip_gpu_blobtree.hpp) compiled
as a host would compile them, against a mock of the ParsipHaptics BlobTree classes
(tests/cpp/mock_blobtree.hpp: the accessors SimdPoly::linearizeBlobTree calls,
PS_HighPerformanceRender.cpp:42-364).

CPU: the C++ linearizer gives the same SoA bytes as the Python mirror
(parsip_amd/blobtree.py) on the reference's own train scene and on a tree with every
primitive and parametrised operator, in translated and raw-code modes.
GPU: SimdPoly::run + draw on the device against the oracle, and
PS::SIMDPOLY::Polygonize into the reference-capacity PolyMPUs (C2 fits; C3 returns -4
with ctMPUs = 0)."""
import os
import shutil
import subprocess

import numpy as np
import pytest

from parsip_amd import blobtree as bt
from parsip_amd import gpu, soa, synth
from parsip_amd.blobtree import BlobNodeType as B

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")


@pytest.fixture(scope="module")
def exe(tmp_path_factory):
    gpp = shutil.which("g++")
    if gpp is None:
        pytest.skip("no g++")
    gpu.load()
    out = tmp_path_factory.mktemp("cpp") / "simdpoly_check"
    lib_dir = os.path.join(ROOT, "parsip_amd")
    subprocess.run([gpp, "-std=c++17", "-O1", "-Wall", "-Wextra", "-pthread", "-I", os.path.join(ROOT, "include"),
                    "-I", os.path.join(ROOT, "tests", "cpp"), os.path.join(ROOT, "tests", "cpp", "simdpoly_check.cpp"),
                    "-L", lib_dir, "-l:libparsip_gpu.so", f"-Wl,-rpath,{lib_dir}", "-o", str(out)], check=True)
    return str(out)


def _v3(x):
    return [float(np.float32(c)) for c in x]


def write_tree(root: bt.BlobNode, path: str) -> None:
    """Pre-order node records for the mock (see simdpoly_check.cpp read_node)."""
    if root.octree is None:
        bt.compute_octrees(root)  # the linearizer's default (reference octrees)
    lines = []

    def rec(n):
        lo, hi = n.octree
        back = n.transform.backward()
        rows = np.concatenate([back.row(r) for r in range(4)])
        p = n.params
        q = [0.0] * 12
        t = n.node_type
        if n.is_operator():
            if t == B.OP_RICCIBLEND:
                q[0] = p.get("n", 2.0)
            elif t == B.OP_PCM:
                q[:4] = [p.get(k, 0.0) for k in ("propagate_left", "propagate_right", "alpha_left", "alpha_right")]
            else:
                q[:4] = [p.get(f"res{k}", 0.0) for k in "XYZW"]
        elif t == B.PRIM_POINT:
            q[0:3] = p["position"]
        elif t == B.PRIM_LINE:
            q[0:3], q[3:6] = p["start"], p["end"]
        elif t in (B.PRIM_CYLINDER, B.PRIM_DISC, B.PRIM_RING):
            q[0:3], q[3:6], q[9] = p["position"], p["direction"], p["radius"]
            q[10] = p.get("height", 0.0)
        elif t == B.PRIM_CUBE:
            q[0:3], q[9] = p["position"], p["side"]
        elif t == B.PRIM_TRIANGLE:
            q[0:3], q[3:6], q[6:9] = p["corners"]
        elif t == B.PRIM_QUADRICPOINT:
            q[0:3], q[9], q[10] = p["position"], p["radius"], p["scale"]
        elif t == B.PRIM_INSTANCE:
            q[0] = float(p["origin"].node_id)
        vals = [*_v3(lo), *_v3(hi), *_v3(n.material.diffused[:3]), 1.0 if back.is_identity() else 0.0,
                *[float(x) for x in rows], *[float(np.float32(x)) for x in q],
                float(np.float32(n.material.diffused[3])), float(n.node_id)]
        lines.append(f"{int(t)} {len(n.children)} " + " ".join(repr(v) for v in vals))
        for c in n.children:
            rec(c)

    rec(root)
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


def cpp_linearize(exe, root, tmp_path, translate=True, compat=False):
    tree, out = tmp_path / "tree.txt", tmp_path / "soa.bin"
    write_tree(root, str(tree))
    subprocess.run([exe, "tree", str(tree), str(out), str(int(translate)), str(int(compat))], check=True, timeout=60)
    raw = open(out, "rb").read()
    code = int(np.frombuffer(raw[:4], np.int32)[0])
    return code, raw[4:]


def py_bytes(model: soa.Model) -> bytes:
    return model.prims.tobytes() + model.mats.tobytes() + model.ops.tobytes() + model.boxmats.tobytes()


def all_types_tree():
    """Every primitive the adapter packs, every parametrised operator, matrices."""
    aff = bt.Affine(scale=(1.2, 0.8, 1.0), rotate=(0.0, 0.38268343, 0.0, 0.9238795), translate=(0.3, -0.2, 0.1))
    prims = [bt.Point((0.1, 0.2, 0.3)), bt.Line((-0.5, 0.0, 0.0), (0.5, 0.1, 0.0), transform=aff),
             bt.Cylinder((0.0, -0.3, 0.0), (0.0, 1.0, 0.0), 0.2, 0.6), bt.Disc((0.3, 0.3, 0.0), (0.0, 0.0, 1.0), 0.4),
             bt.Ring((-0.3, 0.3, 0.0), (1.0, 0.0, 0.0), 0.35, transform=aff), bt.Cube((0.0, 0.0, 0.4), 0.25),
             bt.Triangle((0.0, 0.0, 0.0), (0.5, 0.0, 0.1), (0.0, 0.5, 0.2)), bt.Null()]
    a = bt.Op(B.OP_RICCIBLEND, prims[0], prims[1], n=4.0)
    b = bt.Op(B.OP_PCM, prims[2], prims[3], propagate_left=0.5, propagate_right=0.25, alpha_left=2.0,
              alpha_right=3.0)
    c = bt.Op(B.OP_WARPBEND, bt.Op(B.OP_UNION, prims[4], prims[5]), prims[6], resX=0.7, resY=0.1, resZ=-1.0,
              resW=1.0)
    d = bt.Op(B.OP_WARPTWIST, prims[7], bt.Point((0.9, 0.9, 0.9)), resX=0.3, resY=1.0)
    e = bt.Op(B.OP_WARPSHEAR, bt.Op(B.OP_WARPTAPER, a, b, resX=0.2, resY=2.0, resZ=0.0), c, resX=0.1, resY=1.0,
              resZ=2.0)
    return bt.Op(B.OP_DIF, e, d)


def train_tree():
    from parsip_amd import scene

    return bt.binarize(scene.load_scene(os.path.join(GOLDEN, "train_corrected.scene"))[0])


@pytest.mark.parametrize("translate,compat", [(True, False), (False, True), (True, True)])
def test_cpp_linearizer_all_types(exe, tmp_path, translate, compat):
    root = all_types_tree()
    code, raw = cpp_linearize(exe, root, tmp_path, translate, compat)
    pcode, model = bt.linearize_blobtree(root, raw_types=not translate, triangle_compat=compat)
    assert code == pcode == 0
    assert raw == py_bytes(model)


def test_cpp_linearizer_train_scene(exe, tmp_path):
    root = train_tree()
    code, raw = cpp_linearize(exe, root, tmp_path)
    pcode, model = bt.linearize_blobtree(root)
    assert code == pcode == 0 and model.ct_prims == 95
    assert raw == py_bytes(model)


def test_cpp_linearizer_errors(exe, tmp_path):
    """-3 for a non-binary operator (PS_ERROR_NON_BINARY_OP), -1 past 128 primitives."""
    tri = bt.Op(B.OP_UNION, bt.Point((0, 0, 0)), bt.Point((1, 0, 0)), bt.Point((0, 1, 0)))
    assert cpp_linearize(exe, bt.Op(B.OP_BLEND, tri, bt.Point((0, 0, 1))), tmp_path)[0] == -3
    acc = bt.Point((0, 0, 0))
    for i in range(129):
        acc = bt.Op(B.OP_BLEND, acc, bt.Point((0.01 * i, 0, 0)))
    code, _ = cpp_linearize(exe, acc, tmp_path)
    assert code == bt.linearize_blobtree(acc)[0] in (-1, -2)


def _transformed_points(n):
    aff = bt.Affine(scale=(1.1, 1.0, 0.9), translate=(0.01, 0.0, 0.0))
    nodes = [bt.Point((0.01 * i, 0, 0), transform=aff) for i in range(n)]
    while len(nodes) > 1:  # balanced binary tree of Blends
        nodes = [bt.Op(B.OP_BLEND, nodes[i], nodes[i + 1]) if i + 1 < len(nodes) else nodes[i]
                 for i in range(0, len(nodes), 2)]
    return nodes[0]


def test_cpp_linearizer_matrix_slots(exe, tmp_path):
    """SOABlobPrimMatrices holds 128 slots, slot 0 the identity: 127 transformed primitives
    fit, a 128th is PS_ERROR_PRIM_OVERFLOW (-1) from both faces instead of a write past the
    array."""
    code, raw = cpp_linearize(exe, _transformed_points(127), tmp_path)
    pcode, model = bt.linearize_blobtree(_transformed_points(127))
    assert code == pcode == 0 and int(model.mats["count"][0]) == 128
    assert raw == py_bytes(model)
    code, _ = cpp_linearize(exe, _transformed_points(128), tmp_path)
    assert code == bt.linearize_blobtree(_transformed_points(128))[0] == bt.PS_ERROR_PRIM_OVERFLOW


@pytest.mark.gpu
def test_cpp_simdpoly_run_and_draw_train(exe, tmp_path, oracle):
    """SimdPoly::linearizeBlobTree + run + draw (compiled C++) on the device, against the
    oracle on the same SoA: every drawn MPU's arrays bit-exact."""
    from parity_util import assert_bits_equal

    root = train_tree()
    tree, mesh = tmp_path / "tree.txt", tmp_path / "mesh.bin"
    write_tree(root, str(tree))
    r = subprocess.run([exe, "run", str(tree), "0.2", str(mesh)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    _, model = bt.linearize_blobtree(root)
    om = oracle.polygonize(model, 0.2, threads=8)
    raw = open(mesh, "rb").read()
    at, drawn = 0, 0
    for i in np.flatnonzero(om.stats[:, 3]):  # draw() visits MPUs with triangles, in order
        nv, nt = np.frombuffer(raw[at:at + 8], np.uint32)
        at += 8
        assert (nv, nt) == (om.stats[i, 2], om.stats[i, 3])
        v0, t0 = om.vertex_offsets[i], om.triangle_offsets[i]
        for arr, ref, what in (("pos", om.pos, "pos"), ("nrm", om.nrm, "nrm"), ("col", om.col, "col")):
            got = np.frombuffer(raw[at:at + nv * 12], np.float32).reshape(-1, 3)
            at += nv * 12
            assert_bits_equal(got, ref[v0:v0 + nv], what)
        tris = np.frombuffer(raw[at:at + nt * 6], np.uint16).reshape(-1, 3)
        at += nt * 6
        np.testing.assert_array_equal(tris, om.tris[t0:t0 + nt])
        drawn += 1
    assert at == len(raw) and drawn > 100


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["C2", "C3"])
def test_cpp_ps_simdpoly_polygonize(exe, tmp_path, oracle, name):
    """PS::SIMDPOLY::Polygonize (the reference's free function and PolyMPUs type, 24,000
    MPUs) through the compiled shim: C2 fills it bit-exactly; C3 (50,653 MPUs) does not
    fit and returns -4 with ctMPUs = 0 (the reference truncates silently)."""
    model, cs, _ = synth.make_config(name)
    src, out = tmp_path / "soa.bin", tmp_path / "mpus.bin"
    with open(src, "wb") as f:
        f.write(model.prims.tobytes() + model.mats.tobytes() + model.ops.tobytes() + model.boxmats.tobytes())
    r = subprocess.run([exe, "soa", str(src), repr(float(cs)), str(out)], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    raw = open(out, "rb").read()
    rc, ct = np.frombuffer(raw[:8], np.int32)
    if name == "C3":
        assert (rc, ct) == (soa.RET_MPU_OVERFLOW, 0)
        return
    assert rc == soa.RET_SUCCESS and ct == 6859
    mpus = np.frombuffer(raw[8:], soa.MPU_DTYPE)
    om = oracle.polygonize(model, cs, threads=8)
    np.testing.assert_array_equal(mpus["ctVertices"], om.stats[:, 2])
    np.testing.assert_array_equal(mpus["ctTriangles"], om.stats[:, 3])
    for i in np.flatnonzero(om.stats[:, 2]):
        nv, nt = om.stats[i, 2], om.stats[i, 3]
        v0, t0 = om.vertex_offsets[i], om.triangle_offsets[i]
        assert mpus["vPos"][i, :nv * 3].tobytes() == om.pos[v0:v0 + nv].tobytes()
        np.testing.assert_array_equal(mpus["triangles"][i, :nt * 3].reshape(-1, 3), om.tris[t0:t0 + nt])


@pytest.mark.gpu
def test_cpp_ps_simdpoly_print_thread_results(exe, tmp_path):
    """PS::SIMDPOLY::PrintThreadResults (PS_Polygonizer.h:393, .cpp:414-428) after two
    Polygonize calls on C2: one worker (the calling thread's default context) whose counts,
    divided by ctAttempts = 2, are the MPUs of one call and those with ctTriangles > 0; the
    reference's lines on stdout; a second call finds nothing (the counters were cleared)."""
    model, cs, _ = synth.make_config("C2")
    src, out = tmp_path / "soa.bin", tmp_path / "threads.bin"
    with open(src, "wb") as f:
        f.write(model.prims.tobytes() + model.mats.tobytes() + model.ops.tobytes() + model.boxmats.tobytes())
    r = subprocess.run([exe, "soa-threads", str(src), repr(float(cs)), str(out)], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    raw = open(out, "rb").read()
    rc1, rc2, n, after = np.frombuffer(raw[:16], np.int32)
    assert rc1 == rc2 == soa.RET_SUCCESS and n == 1 and after == 0
    pr, cr = np.frombuffer(raw[16:16 + 8 * n], np.uint32).reshape(2, n)
    pr2 = np.frombuffer(raw[16 + 8 * n:32 + 8 * n], np.uint32)
    mpus = np.frombuffer(raw[32 + 8 * n:], soa.MPU_DTYPE)
    assert len(mpus) == 6859
    crossed = int((mpus["ctTriangles"] > 0).sum())
    assert int(pr.sum()) == 6859 and int(cr.sum()) == crossed > 0
    assert (pr2 == 0xdeadbeef).all()  # no entry: nothing written
    lines = [l for l in r.stdout.splitlines() if l.startswith("Thread#")]
    assert lines == [f"Thread#  1, Processed MPUs 6859, Crossed MPUs {crossed} "]


@pytest.mark.gpu
def test_cpp_ps_simdpoly_host_threads(exe, tmp_path, oracle):
    """PS::SIMDPOLY::Polygonize from 4 host threads at once (a host calling the free function
    from its own workers; each thread runs on its own default context), 3 calls each into its
    own PolyMPUs: every call succeeds with the same records, thread 0's equal the oracle's, and
    PrintThreadResults(3, ...) reports one worker per thread with one call's MPUs each."""
    model, cs, _ = synth.make_config("C2")
    src, out = tmp_path / "soa.bin", tmp_path / "mt.bin"
    with open(src, "wb") as f:
        f.write(model.prims.tobytes() + model.mats.tobytes() + model.ops.tobytes() + model.boxmats.tobytes())
    r = subprocess.run([exe, "soa-mt", str(src), repr(float(cs)), str(out)], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    raw = open(out, "rb").read()
    calls = int(np.frombuffer(raw[:4], np.int32)[0])
    at = 4
    rcs = np.frombuffer(raw[at:at + 4 * calls], np.int32)
    at += 4 * calls
    cts = np.frombuffer(raw[at:at + 4 * calls], np.uint32)
    at += 4 * calls
    sums = np.frombuffer(raw[at:at + 8 * calls], np.uint64)
    at += 8 * calls
    n = int(np.frombuffer(raw[at:at + 4], np.int32)[0])
    at += 4
    pr, cr = np.frombuffer(raw[at:at + 8 * n], np.uint32).reshape(2, n)
    at += 8 * n
    mpus = np.frombuffer(raw[at:], soa.MPU_DTYPE)
    assert calls == 12 and (rcs == soa.RET_SUCCESS).all() and (cts == 6859).all()
    assert len(set(sums.tolist())) == 1, sums
    om = oracle.polygonize(model, cs, threads=8)
    np.testing.assert_array_equal(mpus["ctVertices"], om.stats[:, 2])
    np.testing.assert_array_equal(mpus["ctTriangles"], om.stats[:, 3])
    for i in np.flatnonzero(om.stats[:, 2]):
        nv, nt = om.stats[i, 2], om.stats[i, 3]
        v0, t0 = om.vertex_offsets[i], om.triangle_offsets[i]
        assert mpus["vPos"][i, :nv * 3].tobytes() == om.pos[v0:v0 + nv].tobytes()
        np.testing.assert_array_equal(mpus["triangles"][i, :nt * 3].reshape(-1, 3), om.tris[t0:t0 + nt])
    crossed = int((mpus["ctTriangles"] > 0).sum())
    assert n == 4 and (pr == 6859).all() and (cr == crossed).all()


# ---- compat mode: COMPACTBLOBTREE::convert and CParsipOptimized in C++ (parsip_gpu_gui.hpp)
def cpp_compact(exe, root, tmp_path):
    tree, out = tmp_path / "tree.txt", tmp_path / "compact.bin"
    write_tree(root, str(tree))
    subprocess.run([exe, "gui-tree", str(tree), str(out)], check=True, timeout=60)
    raw = open(out, "rb").read()
    code = int(np.frombuffer(raw[:4], np.int32)[0])
    nP, nO, nK, nM = (int(x) for x in np.frombuffer(raw[4:20], np.uint32))
    at = 20
    parts = []
    for n, size in ((nP, 128), (nO, 80), (nK, 4), (nM, 64)):
        parts.append(raw[at:at + n * size])
        at += n * size
    return code, parts


def gui_all_types_tree():
    from parsip_amd import gui

    t = all_types_tree()
    t.children.append(gui.QuadricPoint((0.2, 0.1, -0.3), 0.9, 1.3, material=bt.Material(diffused=(0.1, 0.2, 0.3, 0.5))))
    t.children.append(bt.Op(B.OP_BLEND, bt.Point((0.0, 0.5, 0.0)), bt.Point((0.5, 0.5, 0.0)), bt.Cube((0.5, 0.0, 0.0), 0.1)))
    for i, n in enumerate(_walk(t)):
        n.node_id = 100 + i
    return t


def _walk(n):
    yield n
    for c in n.children:
        yield from _walk(c)


def gui_ext_tree():
    """PCM and Instances (of an operator and of a primitive) over the all-types tree."""
    from parsip_amd import gui

    t = gui_all_types_tree()
    x, y = t.children[-1], t.children[-1].children[0]
    t.children.append(gui.Pcm(bt.Point((0.0, 0.0, 0.0)), bt.Instance(y), alpha_left=0.7))
    t.children.append(bt.Instance(x, transform=bt.Affine((1, 1, 1), (0, 0, 0, 1), (0.4, 0.0, 0.0))))
    for i, n in enumerate(_walk(t)):
        n.node_id = 100 + i
    return t


@pytest.mark.parametrize("which", ["train", "all_types", "pcm_instance"])
def test_cpp_compact_tree_matches_python(exe, tmp_path, which):
    """CompactTreeT<Api>::convert over the mock BlobTree gives the same COMPACTBLOBTREE arrays,
    byte for byte, as parsip_amd/gui.py::compact_blobtree (n-ary operators kept)."""
    from parsip_amd import gui, scene

    root = (scene.load_scene(os.path.join(GOLDEN, "train_corrected.scene"))[0] if which == "train"
            else gui_all_types_tree() if which == "all_types" else gui_ext_tree())
    bt.compute_octrees(root)
    code, parts = cpp_compact(exe, root, tmp_path)
    pcode, tree = gui.compact_blobtree(root)
    assert code == pcode == 0
    for got, ref, what in zip(parts, (tree.prims, tree.ops, tree.kids, tree.mtx), ("prims", "ops", "kids", "mtx")):
        assert got == ref.tobytes(), what


def test_cpp_compact_tree_errors(exe, tmp_path):
    bad = bt.Op(B.OP_UNION, bt.Point((0, 0, 0)), bt.Op(B.OP_GRADIENTBLEND, bt.Point((1, 0, 0)), bt.Point((0, 1, 0))))
    code, _ = cpp_compact(exe, bad, tmp_path)
    assert code == -5  # ERR_NODE_NOT_RECOGNIZED (CompactBlobTree.cpp:233-239)


@pytest.mark.gpu
def test_cpp_parsip_optimized_run_train(exe, tmp_path):
    """PS::CParsipOptimizedGpu (compiled C++) setup + run + exportMesh + drawMesh on the device,
    against the CPU restatement of CParsipOptimized (oracle/psgui.c): bit-exact."""
    import psgui
    from gui_util import bits
    from parsip_amd import gui, scene

    root = scene.load_scene(os.path.join(GOLDEN, "train_corrected.scene"))[0]
    bt.compute_octrees(root)
    tree, mesh = tmp_path / "tree.txt", tmp_path / "mesh.bin"
    write_tree(root, str(tree))
    r = subprocess.run([exe, "gui-run", str(tree), "0.2", str(mesh)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    raw = open(mesh, "rb").read()
    V, T = (int(x) for x in np.frombuffer(raw[:8], np.uint32))
    _, ct = gui.compact_blobtree(root)
    om = psgui.polygonize(ct, *ct.root_octree, 0.2, 0.5, threads=8)
    assert (V, T) == (om.info.ctVertices, om.info.ctTriangles)
    at = 8
    for name, width in (("pos", 3), ("nrm", 3), ("col", 4)):
        got = np.frombuffer(raw[at:at + V * width * 4], np.float32).reshape(-1, width)
        at += V * width * 4
        assert np.array_equal(bits(got), bits(getattr(om, name))), name
    assert np.array_equal(np.frombuffer(raw[at:], np.uint32).reshape(-1, 3), om.tris)


@pytest.mark.gpu
def test_cpp_parsip_optimized_run_pcm_instance(exe, tmp_path):
    """PS::CParsipOptimizedGpu over a tree with a PCM and Instances (C++ conversion, origins
    resolved by node id) on the device, against the oracle on the Python conversion: the
    same arrays (test_cpp_compact_tree_matches_python), so the same mesh, bit-exact."""
    import psgui
    from gui_util import bits
    from parsip_amd import gui

    root = gui_ext_tree()
    bt.compute_octrees(root)
    tree, mesh = tmp_path / "tree.txt", tmp_path / "mesh.bin"
    write_tree(root, str(tree))
    r = subprocess.run([exe, "gui-run", str(tree), "0.06", str(mesh)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    raw = open(mesh, "rb").read()
    V, T = (int(x) for x in np.frombuffer(raw[:8], np.uint32))
    _, ct = gui.compact_blobtree(root)
    om = psgui.polygonize(ct, *ct.root_octree, 0.06, 0.5, threads=8)
    assert (V, T) == (om.info.ctVertices, om.info.ctTriangles) and V > 0
    at = 8
    for name, width in (("pos", 3), ("nrm", 3), ("col", 4)):
        got = np.frombuffer(raw[at:at + V * width * 4], np.float32).reshape(-1, width)
        at += V * width * 4
        assert np.array_equal(bits(got), bits(getattr(om, name))), name
    assert np.array_equal(np.frombuffer(raw[at:], np.uint32).reshape(-1, 3), om.tris)

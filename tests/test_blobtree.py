"""BlobTree model API + SimdPoly::linearizeBlobTree mirror (parsip_amd/blobtree.py,
SURVEY.md §8(f1)).  CPU only; the GPU side of the linearized trees is in
test_gpu_parity.py::test_scene_train."""
import numpy as np
import pytest

from parsip_amd import blobtree as bt
from parsip_amd import soa, synth
from parsip_amd.blobtree import BlobNodeType as B


def synth_tree(name: str) -> bt.BlobNode:
    """The synth.make_config tree rebuilt through the node API."""
    model, _, _ = synth.make_config(name)
    P, O = model.prims[0], model.ops[0]
    prims = []
    for i in range(model.ct_prims):
        t = int(P["skeletType"][i])
        pos = (P["posX"][i], P["posY"][i], P["posZ"][i])
        d = (P["dirX"][i], P["dirY"][i], P["dirZ"][i])
        col = bt.Material(diffused=(P["colorX"][i], P["colorY"][i], P["colorZ"][i], 1.0))
        if t == soa.NodeType.POINT:
            n = bt.Point(pos, material=col)
        elif t == soa.NodeType.LINE:
            n = bt.Line(pos, d, material=col)
        elif t == soa.NodeType.CYLINDER:
            n = bt.Cylinder(pos, d, P["resX"][i], P["resY"][i], material=col)
        else:
            n = bt.Cube(pos, P["resX"][i], material=col)
        prims.append(n)
    inv = {soa.translate_blobtree_type(int(b)): b for b in B if soa.translate_blobtree_type(int(b)) >= 0}

    def node(op):
        kind = int(O["opChildKind"][op])
        L, R = int(O["opLeftChild"][op]), int(O["opRightChild"][op])
        left = node(L) if kind & 2 else prims[L]
        right = node(R) if kind & 1 else prims[R]
        return bt.Op(B(inv[int(O["opType"][op])]), left, right)

    return node(0)


@pytest.mark.parametrize("name", ["C2", "C3"])
def test_linearize_reproduces_synth_soa(name):
    """Pre-order ids, child kinds, op types, prim packing and colours equal the SoA the
    synthetic generator writes directly (boxes re-derived by PrepareBBoxes on both)."""
    ref, _, _ = synth.make_config(name)
    code, m = bt.linearize_blobtree(synth_tree(name))
    assert code == 0
    synth.prepare_boxes(m)
    m.prims["bboxLo"][0] = ref.prims["bboxLo"][0]
    m.prims["bboxHi"][0] = ref.prims["bboxHi"][0]
    assert m.prims.tobytes() == ref.prims.tobytes()
    assert m.ops.tobytes() == ref.ops.tobytes()


def test_error_codes():
    p = [bt.Point((0, 0, 0)) for _ in range(3)]
    code, _ = bt.linearize_blobtree(bt.Op(B.OP_UNION, *p))
    assert code == bt.PS_ERROR_NON_BINARY_OP
    leaves = [bt.Point((i * 0.01, 0, 0)) for i in range(129)]
    acc = leaves[0]
    for leaf in leaves[1:]:
        acc = bt.Op(B.OP_BLEND, acc, leaf)
    code, _ = bt.linearize_blobtree(acc)
    assert code == bt.PS_ERROR_OPERATOR_OVERFLOW or code == bt.PS_ERROR_PRIM_OVERFLOW
    ok, m = bt.linearize_blobtree(bt.binarize(bt.Op(B.OP_UNION, *p)))
    assert ok == 0 and m.ct_ops == 2 and m.ct_prims == 3


def test_preorder_ids_and_child_kinds():
    a, b, c, d = (bt.Point((i, 0, 0)) for i in range(4))
    root = bt.Op(B.OP_UNION, bt.Op(B.OP_BLEND, a, b), bt.Op(B.OP_DIF, c, d))
    code, m = bt.linearize_blobtree(root)
    O = m.ops[0]
    assert code == 0 and m.ct_ops == 3
    assert list(O["opType"][:3]) == [soa.NodeType.UNION, soa.NodeType.BLEND, soa.NodeType.DIF]
    assert list(O["opChildKind"][:3]) == [3, 0, 0]
    assert (O["opLeftChild"][0], O["opRightChild"][0]) == (1, 2)
    assert (O["opLeftChild"][2], O["opRightChild"][2]) == (2, 3)
    assert list(m.prims[0]["posX"][:4]) == [0, 1, 2, 3]


def test_raw_types_and_triangle_compat():
    tri = bt.Triangle((0, 0, 0), (1, 0, 0), (0, 1, 2))
    root = bt.Op(B.OP_RICCIBLEND, tri, bt.Point((0, 0, 0)), n=4.0)
    _, m = bt.linearize_blobtree(root, raw_types=True, triangle_compat=True)
    assert m.ops[0]["opType"][0] == B.OP_RICCIBLEND  # the reference's raw code
    assert m.prims[0]["skeletType"][0] == B.PRIM_TRIANGLE
    assert m.prims[0]["resX"][0] == 2.0 and m.prims[0]["resZ"][0] == 0.0
    _, m = bt.linearize_blobtree(root)
    assert m.ops[0]["opType"][0] == soa.NodeType.RICCIBLEND
    assert m.prims[0]["resX"][0] == 0.0 and m.prims[0]["resZ"][0] == 2.0
    assert m.ops[0]["resX"][0] == 4.0 and m.ops[0]["resY"][0] == np.float32(0.25)


def test_affine_backward_matrix():
    rng = np.random.default_rng(7)
    for _ in range(20):
        ax = rng.normal(size=3)
        ax /= np.linalg.norm(ax)
        ang = rng.uniform(0, np.pi)
        q = (*(ax * np.sin(ang / 2)), np.cos(ang / 2))
        aff = bt.Affine(tuple(rng.uniform(0.5, 3, 3)), tuple(q), tuple(rng.uniform(-2, 2, 3)))
        f, b = aff.forward().e.astype(np.float64), aff.backward().e.astype(np.float64)
        np.testing.assert_allclose(f @ b, np.eye(4), atol=2e-5)
    # identity transform -> identity backward -> idxMatrix 0
    _, m = bt.linearize_blobtree(bt.Op(B.OP_BLEND, bt.Point((0, 0, 0)), bt.Point((1, 0, 0),
                                  transform=bt.Affine(translate=(0.5, 0, 0)))))
    assert m.prims[0]["idxMatrix"][0] == 0 and m.prims[0]["idxMatrix"][1] == 1
    assert m.mats["count"][0] == 2
    row = m.mats["matrix"][0, 12:24]
    assert row[3] == np.float32(-0.5)  # translation column of the backward rows


# ---------------------------------------------------------------------------
# .scene loader (parsip_amd/scene.py); the fixture is the reference's
# own Distrib/train_corrected.scene (data file, copied verbatim)
TRAIN = __import__("os").path.join(__import__("os").path.dirname(__file__), "golden", "train_corrected.scene")


def test_scene_train_structure():
    from parsip_amd import scene

    roots = scene.load_scene(TRAIN)
    assert len(roots) == 1
    assert scene.count_nodes(roots[0]) == (95, 31)  # 126 [BLOBNODE] sections
    kinds = {}

    def walk(n):
        kinds[n.node_type] = kinds.get(n.node_type, 0) + 1
        for c in n.children:
            walk(c)

    walk(roots[0])
    assert kinds[B.PRIM_CYLINDER] == 75 and kinds[B.PRIM_RING] == 11 and kinds[B.PRIM_CUBE] == 7
    assert kinds[B.OP_RICCIBLEND] == 23 and kinds[B.OP_UNION] == 3
    code, m = bt.linearize_blobtree(bt.binarize(roots[0]))
    assert code == 0 and m.ct_prims == 95 and m.ct_ops == 94
    assert int(m.mats["count"][0]) == 96  # every prim carries a non-identity transform


def test_scene_train_polygonizes_on_oracle(oracle):
    from parsip_amd import scene

    code, m = bt.linearize_blobtree(bt.binarize(scene.load_scene(TRAIN)[0]))
    om = oracle.polygonize(m, 0.2, threads=8)
    assert len(om.pos) > 10000 and len(om.tris) > 10000


def test_scene_parser_variants():
    from parsip_amd import scene

    text = ("[BLOBNODE 0]\nIsOperator=1\nOperatorType=BLEND\nChildrenCount=2\nChildrenIDsUseRange=1\n"
            "ChildrenIDsRange=(1, 2)\n[BLOBNODE 1]\nIsOperator=0\nPrimitiveType=POINT\nposition=(0.5, 0, 0)\n"
            "[BLOBNODE 2]\nIsOperator=0\nPrimitiveType=LINE\nstart=(0,0,0)\nend=(1,1,1)\n"
            "[Global]\nNumLayers=1\nRootIDs=(0)\n")
    (root,) = scene.load_scene(text, from_text=True)
    assert root.node_type == B.OP_BLEND and [c.node_type for c in root.children] == [B.PRIM_POINT, B.PRIM_LINE]
    assert root.children[1].params["end"] == (1.0, 1.0, 1.0)
    with pytest.raises(scene.SceneError):
        scene.load_scene("[BLOBNODE 0]\nIsOperator=0\nPrimitiveType=TEAPOT\n[Global]\nRootIDs=(0)\n", from_text=True)


def test_reference_octrees_follow_the_app():
    """compute_octrees_reference restates CLayer::recursive_RecomputeAllOctrees
    (CLayerManager.cpp:629-646): skeleton bounds in local coordinates (ISO_VALUE 0.5),
    only the two corners through the accumulated forward matrix, Difference keeps its
    first child's box, warps grow it by 0.6, blends take the union."""
    import numpy as np

    from parsip_amd import blobtree as bt
    from parsip_amd.blobtree import BlobNodeType as B

    p = bt.Point((1.0, 2.0, 3.0))
    q = bt.Point((0.0, 0.0, 0.0), transform=bt.Affine(translate=(5.0, 0.0, 0.0)))
    line = bt.Line((0.0, 0.0, 0.0), (-1.0, 0.0, 0.0))  # BBOX keeps its corners: lo > hi on x
    root = bt.Op(B.OP_DIF, bt.Op(B.OP_BLEND, p, q), bt.Op(B.OP_WARPTWIST, line, bt.Point((9.0, 9.0, 9.0))))
    bt.compute_octrees_reference(root)
    np.testing.assert_array_equal(p.octree[0], [0.5, 1.5, 2.5])
    np.testing.assert_array_equal(q.octree[0], [4.5, -0.5, -0.5])
    np.testing.assert_array_equal(root.children[0].octree[0], [0.5, -0.5, -0.5])
    np.testing.assert_array_equal(root.children[0].octree[1], [5.5, 2.5, 3.5])
    np.testing.assert_array_equal(root.octree[0], root.children[0].octree[0])  # Difference: first child
    # Line bound: start - (0.5 + 1.5 * (end - start)), end + ... -> x: 1.0 .. -2.0, min/max after transform
    np.testing.assert_array_equal(line.octree[0], np.float32([-2.0, -0.5, -0.5]))
    np.testing.assert_array_equal(root.children[1].octree[0], line.octree[0] - np.float32(0.6))


def test_train_scene_reference_lattice():
    """The reference's own scene with the app's octrees: the SimdPoly lattice at the
    ParsipHaptics_Release.ini cellsize (0.14, GRID_DIM 8) and the box the CSV run used."""
    import os

    import numpy as np

    from parsip_amd import blobtree as bt
    from parsip_amd import gpu, scene

    root = scene.load_scene(os.path.join(os.path.dirname(__file__), "golden", "train_corrected.scene"))[0]
    code, model = bt.linearize_blobtree(bt.binarize(root))
    assert code == 0 and model.ct_prims == 95
    lo, hi = model.bbox
    np.testing.assert_allclose(lo, [-5.153809, -1.25, -4.2197604], rtol=0, atol=1e-6)
    np.testing.assert_allclose(hi, [19.996407, 11.377769, 4.18024], rtol=0, atol=1e-6)
    assert gpu.count_mpus(np.float32(0.14), lo, hi) == 26 * 13 * 9

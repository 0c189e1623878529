"""The oracle (oracle/psoracle.c, CPU restatement of PS_SimdPoly) pinned against what the
reference itself provides, plus known-answer tests of the field function.  CPU only.

Pins:
* tests/golden/tritable.json — digests of the reference's g_triTableCache / corner1 /
  corner2 / edgeaxis (_CellConfigTable.h:48-51, 60-317), made from the reference text;
* tests/golden/reference_probe.json — MPU / S1 / vertex / triangle counts the reference's
  Polygonize produced for C1, C2, C3 (recorded in SURVEY.md §6, §8(d));
* tests/golden/oracle_digests.json — the oracle's own full-output digests (regression).
"""
import json
import os

import numpy as np
import pytest

from parity_util import assert_bits_equal, mesh_digests
from parsip_amd import soa, synth
from parsip_amd.soa import NodeType

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def test_tritable_matches_reference_digest(oracle):
    import hashlib

    g = golden("tritable.json")
    t = oracle.tritable()
    assert hashlib.sha256(t.astype("<i4").tobytes()).hexdigest() == g["tritable_sha256"]
    assert [int((r >= 0).sum() // 3) for r in t] == g["triangles_per_config"]


def test_tritable_properties(oracle):
    """Rows hold <= 5 triangles with trailing -1 only; configs 0 and 255 are empty and
    complementary configs use the same edge set (SURVEY.md §4 [probe])."""
    t = oracle.tritable()
    for c in range(256):
        row = t[c]
        n = int((row >= 0).sum())
        assert n % 3 == 0 and n <= 15
        assert (row[:n] >= 0).all() and (row[n:] == -1).all()
        assert set(row[:n].tolist()) == set(t[255 - c][t[255 - c] >= 0].tolist())
    assert (t[0] == -1).all() and (t[255] == -1).all()


@pytest.mark.parametrize("name", ["C1", "C2", "C3"])
def test_reference_probe_counts(oracle, name):
    """The reference's own recorded output (counts) for the survey's inputs."""
    g = golden("reference_probe.json")[name]
    model, cs, _ = synth.make_config(name)
    om = oracle.polygonize(model, cs, threads=os.cpu_count() or 1, keep=False)
    st = om.stats
    assert len(st) == g["mpus"]
    assert int(np.count_nonzero(st[:, 0])) == g["passed_s1"]
    assert int((st[:, 1] == 128).sum()) == g["passed_s1"]
    assert int(st[:, 2].sum()) == g["vertices"]
    assert int(st[:, 3].sum()) == g["triangles"]
    if "max_vertices_per_mpu" in g:
        assert int(st[:, 2].max()) == g["max_vertices_per_mpu"]
        assert int(st[:, 3].max()) == g["max_triangles_per_mpu"]


@pytest.mark.parametrize("name", ["C1", "C2"])
def test_oracle_digests(oracle, name):
    g = golden("oracle_digests.json")[name]
    model, cs, _ = synth.make_config(name)
    om = oracle.polygonize(model, cs, threads=os.cpu_count() or 1)
    assert mesh_digests(om.stats[:, :4], om.pos, om.nrm, om.col, om.tris) == g


def test_oracle_threads_deterministic(oracle):
    model, cs, _ = synth.make_config("C2")
    a = oracle.polygonize(model, cs, threads=1)
    b = oracle.polygonize(model, cs, threads=7)
    np.testing.assert_array_equal(a.stats, b.stats)
    assert_bits_equal(a.pos, b.pos, "positions")
    np.testing.assert_array_equal(a.tris, b.tris)


def test_mpu_range_concatenation(oracle):
    model, cs, _ = synth.make_config("C2")
    full = oracle.polygonize(model, cs, threads=8)
    parts = [oracle.polygonize(model, cs, a, b, threads=8) for a, b in [(0, 2000), (2000, 2001), (2001, 6859)]]
    np.testing.assert_array_equal(np.concatenate([p.stats for p in parts]), full.stats)
    assert_bits_equal(np.concatenate([p.pos for p in parts]), full.pos, "positions")


def _triangles_valid(om):
    voff, toff = om.vertex_offsets, om.triangle_offsets
    for m in np.flatnonzero(om.stats[:, 3]):
        t = om.tris[toff[m]:toff[m + 1]]
        nv = om.stats[m, 2]
        assert t.max() < nv
        # every vertex an MPU creates is used by one of its triangles
        assert len(np.unique(t)) == nv


def test_mesh_structure_c2(oracle):
    model, cs, _ = synth.make_config("C2")
    om = oracle.polygonize(model, cs, threads=8)
    _triangles_valid(om)
    # every vertex lies on a lattice edge of its MPU: >= 2 coordinates are lattice values
    origins = soa.mpu_origins(cs, *model.bbox)
    voff = om.vertex_offsets
    csf = np.float32(cs)
    for m in np.flatnonzero(om.stats[:, 2])[:300]:
        p = om.pos[voff[m]:voff[m + 1]]
        lat = [origins[m, a] + csf * np.arange(8, dtype=np.float32) for a in range(3)]
        on = np.stack([np.isin(p[:, a], lat[a]) for a in range(3)], axis=1).sum(axis=1)
        assert (on >= 2).all()


def test_sse_variant_normals_within_tolerance(oracle):
    """The reference normalises with _mm_rsqrt_ps (vendor-specific bits); the oracle's SSE
    build uses it too.  Positions/topology are identical; normals within 2e-3 (§8(c))."""
    model, cs, _ = synth.make_config("C2")
    a = oracle.polygonize(model, cs, threads=8)
    b = oracle.polygonize(model, cs, threads=8, sse_approx=True)
    np.testing.assert_array_equal(a.stats, b.stats)
    assert_bits_equal(a.pos, b.pos, "positions")
    np.testing.assert_array_equal(a.tris, b.tris)
    assert np.nanmax(np.abs(a.nrm - b.nrm)) <= 2e-3


# ---------------------------------------------------------------------------
# known answers for the field function (PS_Polygonizer.cpp:934-1179, 1184-1376)
def _single(ptype, centre=(0.0, 0.0, 0.0)):
    m = soa.Model.empty()
    synth.set_prim(m, 0, ptype, centre)
    m.prims["ctPrims"][0] = 1
    return m


def _f(oracle, model, pts):
    pts = np.asarray(pts, np.float32)
    pts = np.concatenate([pts, np.repeat(pts[-1:], (-len(pts)) % 4, axis=0)])
    return oracle.field_value(model, pts[:, 0], pts[:, 1], pts[:, 2])


def test_kat_point(oracle):
    m = _single(NodeType.POINT)
    f = _f(oracle, m, [(0.5, 0, 0), (0, 0, 0), (1.0, 0, 0), (2.0, 0, 0)])
    assert f.tolist() == [0.421875, 1.0, 0.0, 0.0]  # (1-d^2)^3 clamped at 0


def test_kat_line_is_unclamped(oracle):
    """Line projection is not clamped to the segment (a13): a point far beyond the end
    still sees distance 0.5 to the infinite line."""
    m = _single(NodeType.LINE)
    m.prims["dirX"][0, 0], m.prims["dirY"][0, 0], m.prims["dirZ"][0, 0] = (1.0, 0.0, 0.0)
    f = _f(oracle, m, [(5.0, 0.5, 0.0), (-3.0, 0.0, 0.5), (0.5, 0.0, 0.0), (0.0, 2.0, 0.0)])
    assert f.tolist() == [0.421875, 0.421875, 1.0, 0.0]


def test_kat_cube_and_cylinder(oracle):
    cube = _single(NodeType.CUBE)  # half side 0.3
    f = _f(oracle, cube, [(0.8, 0.0, 0.0), (0.8, 0.8, 0.0), (0.1, 0.2, -0.3), (0.0, 0.0, 2.0)])
    np.testing.assert_allclose(f, [0.421875, 0.125, 1.0, 0.0], rtol=0, atol=1e-6)
    cyl = _single(NodeType.CYLINDER)  # axis +y, r 0.2, h 0.8
    f = _f(oracle, cyl, [(0.7, 0.4, 0.0), (0.0, 1.3, 0.0), (0.0, 0.5, 0.1), (0.0, -0.5, 0.0)])
    np.testing.assert_allclose(f, [0.421875, 0.421875, 1.0, 0.421875], rtol=0, atol=1e-6)


def test_kat_triangle_and_null(oracle):
    tri = _single(NodeType.TRIANGLE)
    assert (_f(oracle, tri, [(0, 0, 0)] * 4) == 0).all()  # stub: FLT_MAX distance
    null = _single(NodeType.NULL)
    assert (_f(oracle, null, [(3, 3, 3)] * 4) == 1).all()  # no switch case: dist2 = 0


@pytest.mark.parametrize("op,fn", [
    (NodeType.BLEND, lambda l, r: l + r),
    (NodeType.UNION, np.maximum),
    (NodeType.INTERSECT, np.minimum),
    (NodeType.DIF, lambda l, r: np.minimum(l, np.float32(1) - r)),
    (NodeType.SMOOTHDIF, lambda l, r: l * (np.float32(1) - r)),
    (NodeType.WARPTWIST, lambda l, r: l),
])
def test_kat_ops(oracle, op, fn):
    m = soa.Model.empty()
    synth.set_prim(m, 0, NodeType.POINT, (0.0, 0.0, 0.0))
    synth.set_prim(m, 1, NodeType.POINT, (0.6, 0.0, 0.0))
    m.prims["ctPrims"][0] = 2
    O = m.ops
    O["opType"][0, 0], O["opLeftChild"][0, 0], O["opRightChild"][0, 0], O["opChildKind"][0, 0] = op, 0, 1, 0
    O["ctOps"][0] = 1
    synth.prepare_boxes(m)
    xs = np.linspace(-0.9, 1.5, 16, dtype=np.float32)
    pts = np.stack([xs, np.full(16, 0.1, np.float32), np.zeros(16, np.float32)], axis=1)
    l_ = _f(oracle, _single(NodeType.POINT), pts)
    r_ = _f(oracle, _single(NodeType.POINT, (0.6, 0.0, 0.0)), pts)
    assert_bits_equal(_f(oracle, m, pts), fn(l_, r_).astype(np.float32), f"op {op}")


def test_kat_no_ops_sums_prims(oracle):
    """ctOps == 0: the field is the sum of all primitive fields in index order (:1356-1368)."""
    m = soa.Model.empty()
    synth.set_prim(m, 0, NodeType.POINT, (0.0, 0.0, 0.0))
    synth.set_prim(m, 1, NodeType.POINT, (0.5, 0.0, 0.0))
    m.prims["ctPrims"][0] = 2
    pts = [(0.25, 0, 0), (0.0, 0.0, 0.0), (0.5, 0.5, 0.0), (3, 0, 0)]
    a = _f(oracle, _single(NodeType.POINT), pts)
    b = _f(oracle, _single(NodeType.POINT, (0.5, 0.0, 0.0)), pts)
    assert_bits_equal(_f(oracle, m, pts), a + b, "sum of prims")


def test_prepare_bboxes_matches_synth(oracle):
    """PrepareBBoxes restated in C (oracle) and in numpy (synth) give the same boxes."""
    for name in ("C2", "C3"):
        m, cs, _ = synth.make_config(name)
        a = m.copy()
        assert oracle.prepare_bboxes(a) == 1
        for f in soa.PRIMS_DTYPE.names:
            if f not in ("bboxLo", "bboxHi"):  # synth overrides the scene box with the cube
                np.testing.assert_array_equal(a.prims[f], m.prims[f], err_msg=f)
        assert a.ops.tobytes() == m.ops.tobytes()


def test_count_mpus_lattice(oracle):
    rng = np.random.default_rng(0)
    for _ in range(200):
        lo = rng.uniform(-5, 0, 3).astype(np.float32)
        hi = (lo + rng.uniform(0.1, 9, 3)).astype(np.float32)
        cs = float(np.float32(rng.uniform(0.01, 0.3)))
        n = oracle.count_mpus(cs, lo, hi)
        assert n == soa.count_mpus(cs, lo, hi)
    assert oracle.count_mpus(8 / 256, (-4, -4, -4), (4, 4, 4)) == 37 ** 3


def test_workload_ops_fixture(oracle):
    """tests/golden/workload_ops.json (bench.py's algorithmic-work figure) is what the
    oracle's counters give for C2 today."""
    import importlib.util

    spec = importlib.util.spec_from_file_location("mwo", os.path.join(GOLDEN, "make_workload_ops.py"))
    g = golden("workload_ops.json")["C2"]
    model, cs, _ = synth.make_config("C2")
    om = oracle.polygonize(model, cs, threads=4, keep=False, count=True)
    c = oracle.work_counts()
    assert int(c[1][:16].sum()) == g["prim_evals"]["s2"]
    assert int(c[3][:16].sum()) == g["prim_evals"]["normals"]
    assert int(om.stats[:, 2].sum()) == g["vertices"]
    assert spec is not None

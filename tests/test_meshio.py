"""Mesh output (parsip_amd/meshio.py) on the oracle's C2 mesh."""
import numpy as np

from parsip_amd import meshio, soa, synth


def polympus_from_oracle(om):
    n = len(om.stats)
    mpus = np.zeros(n, soa.MPU_DTYPE)
    voff, toff = om.vertex_offsets, om.triangle_offsets
    for i in np.flatnonzero(om.stats[:, 2]):
        nv, nt = om.stats[i, 2], om.stats[i, 3]
        mpus[i]["ctVertices"], mpus[i]["ctTriangles"] = nv, nt
        mpus[i]["vPos"][:nv * 3] = om.pos[voff[i]:voff[i + 1]].reshape(-1)
        mpus[i]["vNorm"][:nv * 3] = om.nrm[voff[i]:voff[i + 1]].reshape(-1)
        mpus[i]["vColor"][:nv * 3] = om.col[voff[i]:voff[i + 1]].reshape(-1)
        mpus[i]["triangles"][:nt * 3] = om.tris[toff[i]:toff[i + 1]].reshape(-1)
    return mpus


def test_polympus_to_compact_mesh(oracle):
    model, cs, _ = synth.make_config("C2")
    om = oracle.polygonize(model, cs, threads=8)
    m = meshio.from_polympus(polympus_from_oracle(om))
    assert m.n_vertices == len(om.pos) and m.n_triangles == len(om.tris)
    np.testing.assert_array_equal(m.tris, om.global_tris())
    np.testing.assert_array_equal(m.pos.view(np.uint32), om.pos.view(np.uint32))


def test_weld_and_file_round_trip(oracle, tmp_path):
    model, cs, _ = synth.make_config("C2")
    om = oracle.polygonize(model, cs, threads=8)
    m = meshio.TriMesh(om.pos, om.global_tris(), om.nrm, om.col)
    w = meshio.weld(m)
    assert w.n_vertices < m.n_vertices and w.n_triangles <= m.n_triangles
    assert w.tris.max() < w.n_vertices
    # every welded position is one of the originals, bit for bit
    orig = set(map(bytes, m.pos.view(np.uint32)))
    assert all(bytes(p) in orig for p in w.pos.view(np.uint32)[:500])
    meshio.write_off(w, str(tmp_path / "a.off"))
    r = meshio.read_off(str(tmp_path / "a.off"))
    np.testing.assert_array_equal(r.tris, w.tris)
    np.testing.assert_array_equal(r.pos, w.pos)  # %.9g round-trips fp32 exactly
    meshio.write_ply(w, str(tmp_path / "a.ply"))
    head = open(tmp_path / "a.ply").read().split("end_header")[0]
    assert f"element vertex {w.n_vertices}" in head and "property list uint8 int32 vertex_indices" in head
    meshio.write_obj(w, str(tmp_path / "a.obj"))
    lines = open(tmp_path / "a.obj").read().splitlines()
    assert sum(1 for x in lines if x.startswith("v ")) == w.n_vertices
    assert sum(1 for x in lines if x.startswith("f ")) == w.n_triangles

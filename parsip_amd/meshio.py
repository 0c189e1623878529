"""Mesh output for the polygonizer's result.

The reference consumes `PolyMPUs` per MPU (SimdPoly::draw,
Parsip100/ParsipHaptics/include/PS_HighPerformanceRender.cpp:378-426: one GL vertex /
normal / colour array and one U16 index list per MPU with ctTriangles > 0) and saves
meshes through CMeshVV::save (Parsip100/PS_FrameWork/include/PS_MeshVV.cpp:1023-1163:
OFF and ASCII PLY with "property float32 x|y|z" and "property list uint8 int32
vertex_indices", written in stream order).  Here:

* `from_polympus` turns the reference PolyMPUs layout (e.g. from
  `gpu.Polygonizer.export_polympus`) into one compact mesh, MPU by MPU, as draw() walks it;
* `weld` merges the duplicate vertices MPUs emit on shared faces (exact position bits;
  the reference keeps them, since every MPU is drawn on its own);
* `write_off`, `write_ply` follow CMeshVV::save's text layouts; `write_obj` adds the
  common OBJ form with normals (v / vn / f a//a b//b c//c).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np


@dataclass
class TriMesh:
    pos: np.ndarray          # (V, 3) f32
    tris: np.ndarray         # (T, 3) integer vertex ids
    nrm: np.ndarray | None = None
    col: np.ndarray | None = None

    @property
    def n_vertices(self) -> int:
        return len(self.pos)

    @property
    def n_triangles(self) -> int:
        return len(self.tris)


def from_mesh(mesh) -> TriMesh:
    """A gpu.Mesh (compact device download) as a TriMesh (global u32 ids)."""
    return TriMesh(mesh.pos, mesh.tris.astype(np.int64), mesh.nrm, mesh.col)


def from_polympus(mpus: np.ndarray, ct_mpus: int | None = None) -> TriMesh:
    """Concatenate vMPUs[0..ctMPUs) (soa.MPU_DTYPE) in draw() order."""
    n = len(mpus) if ct_mpus is None else ct_mpus
    pos, nrm, col, tris = [], [], [], []
    base = 0
    for i in range(n):
        m = mpus[i]
        nv, nt = int(m["ctVertices"]), int(m["ctTriangles"])
        if nt == 0:
            continue
        pos.append(m["vPos"][:nv * 3].reshape(-1, 3))
        nrm.append(m["vNorm"][:nv * 3].reshape(-1, 3))
        col.append(m["vColor"][:nv * 3].reshape(-1, 3))
        tris.append(m["triangles"][:nt * 3].reshape(-1, 3).astype(np.int64) + base)
        base += nv
    if not pos:
        z = np.zeros((0, 3), np.float32)
        return TriMesh(z, np.zeros((0, 3), np.int64), z, z)
    return TriMesh(np.concatenate(pos), np.concatenate(tris), np.concatenate(nrm), np.concatenate(col))


def weld(mesh: TriMesh) -> TriMesh:
    """Merge vertices with bit-identical positions (first occurrence keeps its normal and
    colour); drops triangles that become degenerate."""
    if mesh.n_vertices == 0:
        return mesh
    key = np.ascontiguousarray(mesh.pos, np.float32).view(np.uint32).reshape(-1, 3)
    _, first, inverse = np.unique(key, axis=0, return_index=True, return_inverse=True)
    order = np.argsort(first)
    remap = np.empty_like(order)
    remap[order] = np.arange(len(order))
    new_id = remap[inverse.reshape(-1)]
    keep = first[order]
    tris = new_id[mesh.tris]
    ok = (tris[:, 0] != tris[:, 1]) & (tris[:, 1] != tris[:, 2]) & (tris[:, 0] != tris[:, 2])
    return TriMesh(mesh.pos[keep], tris[ok], None if mesh.nrm is None else mesh.nrm[keep],
                   None if mesh.col is None else mesh.col[keep])


def _fmt(a) -> str:
    return " ".join(f"{float(x):.9g}" for x in a)


def write_off(mesh: TriMesh, path: str) -> None:
    """CMeshVV::save OFF (PS_MeshVV.cpp:1086-1108)."""
    with open(path, "w") as f:
        f.write("OFF\n")
        f.write(f"{mesh.n_vertices} {mesh.n_triangles} {mesh.n_triangles * 3}\n")
        for p in mesh.pos:
            f.write(_fmt(p) + " \n")
        for t in mesh.tris:
            f.write(f"3 {t[0]} {t[1]} {t[2]} \n")


def write_ply(mesh: TriMesh, path: str) -> None:
    """CMeshVV::save ASCII PLY (PS_MeshVV.cpp:1109-1143)."""
    with open(path, "w") as f:
        f.write("ply\nformat ascii 1.0\n")
        f.write(f"element vertex {mesh.n_vertices}\n")
        f.write("property float32 x\nproperty float32 y\nproperty float32 z\n")
        f.write(f"element face {mesh.n_triangles}\n")
        f.write("property list uint8 int32 vertex_indices\nend_header\n")
        for p in mesh.pos:
            f.write(_fmt(p) + " \n")
        for t in mesh.tris:
            f.write(f"3 {t[0]} {t[1]} {t[2]} \n")


def write_obj(mesh: TriMesh, path: str) -> None:
    """Wavefront OBJ with per-vertex normals (1-based ids)."""
    with open(path, "w") as f:
        f.write(f"# parsip_amd mesh: {mesh.n_vertices} vertices, {mesh.n_triangles} triangles\n")
        for p in mesh.pos:
            f.write("v " + _fmt(p) + "\n")
        if mesh.nrm is not None:
            for n in mesh.nrm:
                f.write("vn " + _fmt(n) + "\n")
            for t in mesh.tris + 1:
                f.write(f"f {t[0]}//{t[0]} {t[1]}//{t[1]} {t[2]}//{t[2]}\n")
        else:
            for t in mesh.tris + 1:
                f.write(f"f {t[0]} {t[1]} {t[2]}\n")


def read_off(path: str) -> TriMesh:
    with open(path) as f:
        toks = f.read().split()
    assert toks[0] == "OFF"
    nv, nt = int(toks[1]), int(toks[2])
    vals = toks[4:]
    pos = np.array(vals[:nv * 3], np.float32).reshape(-1, 3)
    faces = np.array(vals[nv * 3:nv * 3 + nt * 4], np.int64).reshape(-1, 4)
    return TriMesh(pos, faces[:, 1:])

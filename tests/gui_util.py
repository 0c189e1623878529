"""Shared helpers of the compat-mode (GUI path) tests: random BlobTrees exercising every
node type the compact walk evaluates, and the bit-level comparison of two GUI meshes."""
import numpy as np

from parsip_amd import blobtree as bt
from parsip_amd import gui

B = bt.BlobNodeType
OPS = (B.OP_UNION, B.OP_INTERSECT, B.OP_DIF, B.OP_SMOOTHDIF, B.OP_BLEND, B.OP_RICCIBLEND)
WARPS = (B.OP_WARPTWIST, B.OP_WARPTAPER, B.OP_WARPBEND, B.OP_WARPSHEAR)


def _rand_affine(rng, strength=1.0):
    if rng.random() < 0.4:
        return bt.Affine()
    axis = rng.normal(size=3)
    axis /= np.linalg.norm(axis)
    ang = rng.uniform(-1.0, 1.0) * strength
    q = (*(np.sin(ang / 2) * axis), np.cos(ang / 2))
    s = tuple(rng.uniform(0.7, 1.4, size=3)) if rng.random() < 0.5 else (1.0, 1.0, 1.0)
    t = tuple(rng.uniform(-0.4, 0.4, size=3))
    return bt.Affine(s, tuple(float(c) for c in q), t)


def _rand_prim(rng, kinds):
    k = kinds[rng.integers(len(kinds))]
    c = rng.uniform(-0.9, 0.9, size=3)
    mat = bt.Material(diffused=tuple(float(v) for v in rng.uniform(0, 1, size=4)))
    kw = {"transform": _rand_affine(rng), "material": mat}
    d = rng.normal(size=3)
    d /= np.linalg.norm(d)
    if k == "point":
        return bt.Point(tuple(c), **kw)
    if k == "line":
        return bt.Line(tuple(c), tuple(c + rng.uniform(-0.8, 0.8, size=3)), **kw)
    if k == "cylinder":
        return bt.Cylinder(tuple(c), tuple(d), float(rng.uniform(0.05, 0.3)), float(rng.uniform(0.1, 0.8)), **kw)
    if k == "disc":
        return bt.Disc(tuple(c), tuple(d), float(rng.uniform(0.1, 0.5)), **kw)
    if k == "ring":
        return bt.Ring(tuple(c), tuple(d), float(rng.uniform(0.1, 0.5)), **kw)
    if k == "cube":
        return bt.Cube(tuple(c), float(rng.uniform(0.05, 0.3)), **kw)
    if k == "triangle":
        return bt.Triangle(tuple(c), tuple(c + rng.uniform(-0.6, 0.6, size=3)),
                           tuple(c + rng.uniform(-0.6, 0.6, size=3)), **kw)
    if k == "quadric":
        return gui.QuadricPoint(tuple(c), float(rng.uniform(0.6, 1.3)), float(rng.uniform(0.6, 1.5)), **kw)
    return bt.Null(**kw)


PRIM_KINDS = ("point", "line", "cylinder", "disc", "ring", "cube", "triangle", "quadric", "null")


def random_tree(seed: int, n_prims: int = 12, warps: bool = True, op_transforms: bool = True):
    rng = np.random.default_rng(seed)
    nodes = [_rand_prim(rng, PRIM_KINDS) for _ in range(n_prims)]
    while len(nodes) > 1:
        k = int(min(len(nodes), rng.integers(2, 5)))
        idx = rng.choice(len(nodes), size=k, replace=False)
        kids = [nodes[i] for i in sorted(idx)]
        nodes = [n for i, n in enumerate(nodes) if i not in set(idx)]
        kind = OPS[rng.integers(len(OPS))]
        params = {"n": float(rng.choice([1.0, 2.0, 3.5, 8.0]))} if kind == B.OP_RICCIBLEND else {}
        op = bt.Op(kind, *kids, **params)
        if op_transforms and rng.random() < 0.3:
            op.transform = _rand_affine(rng, 0.5)
        if warps and rng.random() < 0.35:
            w = WARPS[rng.integers(len(WARPS))]
            if w == B.OP_WARPBEND:
                prm = {"resX": float(rng.uniform(0.2, 1.2)), "resY": float(rng.uniform(-0.3, 0.3)),
                       "resZ": float(rng.uniform(-1.0, -0.2)), "resW": float(rng.uniform(0.2, 1.0))}
            else:
                prm = {"resX": float(rng.uniform(-0.8, 0.8)), "resY": float(rng.integers(0, 3)),
                       "resZ": float(rng.integers(0, 3))}
            op = bt.Op(w, op, **prm)
        nodes.append(op)
    root = nodes[0]
    if not root.is_operator():
        root = bt.Op(B.OP_UNION, root)
    return root


def _subtrees(n):
    yield n
    for c in n.children:
        yield from _subtrees(c)


def random_ext_tree(seed: int, n_prims: int = 5):
    """A random tree with PCM and Instance nodes as the compat mode accepts them: a PCM over
    two random subtrees (one of its kids may be an Instance), Instances of a random operator
    and of a random primitive of those subtrees under their own transforms, and the rest
    blended or united with them."""
    rng = np.random.default_rng(1000 + seed)
    a = random_tree(2 * seed + 1, n_prims=n_prims, warps=seed % 2 == 0)
    b = random_tree(2 * seed + 2, n_prims=max(2, n_prims - 1), warps=False)
    ops_a = [n for n in _subtrees(a) if n.is_operator()]
    prims_b = [n for n in _subtrees(b) if not n.is_operator()]
    x = ops_a[int(rng.integers(len(ops_a)))]
    y = prims_b[int(rng.integers(len(prims_b)))]
    kid2 = b if seed % 3 else bt.Instance(y, transform=_rand_affine(rng, 0.4),
                                          material=bt.Material(diffused=(0.1, 0.9, 0.2, 1.0)))
    pcm = gui.Pcm(a, kid2, propagate_left=float(rng.uniform(0.1, 0.6)), propagate_right=float(rng.uniform(0.1, 0.6)),
                  alpha_left=float(rng.uniform(0.2, 1.0)), alpha_right=float(rng.uniform(0.2, 1.0)))
    if rng.random() < 0.4:
        pcm.transform = _rand_affine(rng, 0.5)
    inst_x = bt.Instance(x, transform=_rand_affine(rng, 0.6))
    inst_y = bt.Instance(y, transform=_rand_affine(rng, 0.6))
    kind = OPS[rng.integers(len(OPS))]
    params = {"n": 2.0} if kind == B.OP_RICCIBLEND else {}
    rest = bt.Op(kind, inst_x, _rand_prim(rng, PRIM_KINDS[:8]), **params)
    root = bt.Op(B.OP_UNION if seed % 2 else B.OP_BLEND, pcm, rest, inst_y)
    if kid2 is not b:  # keep b in the tree: the Instance's origin must be converted
        root.children.append(b)
    return root


def bits(a):
    """fp32 bit patterns, NaNs canonical: an invalid operation yields the negative default
    NaN on x86 SSE and the positive one on CDNA, the same result in IEEE terms."""
    a = np.ascontiguousarray(a, np.float32)
    b = a.view(np.uint32).copy()
    b[np.isnan(a)] = 0x7FC00000
    return b


def assert_gui_mesh_equal(gm, om, what=""):
    """Bit-identical GUI meshes (positions, normals, rgba colours, triangles, per-MPU
    offsets and statistics)."""
    assert len(gm.pos) == len(om.pos) and len(gm.tris) == len(om.tris), (what, len(gm.pos), len(om.pos))
    assert np.array_equal(gm.mpu_v, om.mpu_v) and np.array_equal(gm.mpu_t, om.mpu_t), what
    for name in ("fieldEvals", "intersectedCells", "ctVertices", "ctTriangles"):
        assert np.array_equal(gm.stats[name], om.stats[name]), (what, name)
    assert np.array_equal(gm.tris, om.tris), what
    for name in ("pos", "nrm", "col"):
        g, o = bits(getattr(gm, name)), bits(getattr(om, name))
        bad = np.nonzero(g != o)[0]
        assert len(bad) == 0, (what, name, len(bad), getattr(gm, name).ravel()[bad[:4]], getattr(om, name).ravel()[bad[:4]])

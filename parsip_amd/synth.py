"""Synthetic BlobTrees of the benchmark shapes.

Centres come from the stream the survey's reference probe used:
libstdc++ ``std::mt19937(42)`` with ``std::uniform_real_distribution<float>(-2, 2)``,
drawn x, y, z per primitive.  Both are restated here in pure Python (MT19937 is fixed by
the C++ standard; libstdc++'s ``generate_canonical<float, 24>`` with a 32-bit engine is
``float(u) / 2^32`` clamped below 1, then ``r * (b - a) + a`` in fp32), so the inputs are
identical to the reference run and its recorded outputs pin the oracle:
C2 1,417 full MPUs / 32,541 V / 50,034 T and C3 19,237 / 339,820 / 520,224.
The portable splitmix64 stream of §8(d) (``(u >> 40) * 2**-24``) stays available as
``rng="splitmix64"``.

* C1  1 Point at the origin, no ops, 32^3 cells over [-1,1]^3
* C2  8 prims (2 per type), 7 ops, 128^3 over [-4,4]^3
* C3 32 prims (8 per type), 31 ops, 256^3 over [-4,4]^3   (the headline workload)
* C5 64 prims, 63 ops, 512^3 over [-4,4]^3, animated: centre.x += 0.25 sin(2 pi f/60 + i)
  (C2-C4 animate by the same motion relative to frame 0, which stays the probe tree)

Prims cycle Point, Line (end = start + (0.8, 0.3, 0)), Cylinder (axis (0,1,0), r 0.2,
h 0.8), Cube (half side 0.3); centres uniform in [-2,2]^3; identity matrices.
The op tree is balanced (mid = (a+b)/2) with pre-order op ids, as
SimdPoly::linearizeBlobTree allocates them (PS_HighPerformanceRender.cpp:42-160):
depth-0 Union, depth-1 odd-id Dif, otherwise Blend.  Op depth reaches 4 for C3, so
the reference's depth>3 op-box pruning (PS_Polygonizer.cpp:1228-1252) is live.

Primitive and op boxes follow PrepareBBoxes (PS_Polygonizer.cpp:55-309) with the exact
iso distance ISO_DIST + 5*MIN_CELL_SIZE; the scene box is then set to the cubic box so
cellsize = extent / N is exact and the lattice has exactly N cells per axis.
"""
from __future__ import annotations

import math

import numpy as np

from .soa import ISO_DIST, MIN_CELL_SIZE, Model, NodeType

MASK64 = (1 << 64) - 1

CONFIGS = {
    # name: (prims, grid N, half extent)
    "C1": (1, 32, 1.0),
    "C2": (8, 128, 4.0),
    "C3": (32, 256, 4.0),
    "C4": (32, 256, 4.0),
    "C5": (64, 512, 4.0),
}


class SplitMix64:
    def __init__(self, seed: int = 42):
        self.state = seed & MASK64

    def next_u64(self) -> int:
        self.state = (self.state + 0x9E3779B97F4A7C15) & MASK64
        z = self.state
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK64
        return z ^ (z >> 31)

    def next_f32(self) -> np.float32:
        return np.float32((self.next_u64() >> 40) * (2.0 ** -24))


class MT19937:
    """std::mt19937 (C++ [rand.predef]: 32-bit Mersenne Twister, default seeding)."""

    def __init__(self, seed: int = 5489):
        mt = [seed & 0xFFFFFFFF]
        for i in range(1, 624):
            mt.append((1812433253 * (mt[-1] ^ (mt[-1] >> 30)) + i) & 0xFFFFFFFF)
        self.mt = mt
        self.idx = 624

    def next_u32(self) -> int:
        if self.idx >= 624:
            mt = self.mt
            for i in range(624):
                y = (mt[i] & 0x80000000) | (mt[(i + 1) % 624] & 0x7FFFFFFF)
                mt[i] = mt[(i + 397) % 624] ^ (y >> 1) ^ (0x9908B0DF if y & 1 else 0)
            self.idx = 0
        y = self.mt[self.idx]
        self.idx += 1
        y ^= y >> 11
        y ^= (y << 7) & 0x9D2C5680
        y ^= (y << 15) & 0xEFC60000
        return y ^ (y >> 18)

    def uniform_f32(self, a: float, b: float) -> np.float32:
        """libstdc++ uniform_real_distribution<float>(a, b) over this engine."""
        r = np.float32(self.next_u32()) / np.float32(2.0 ** 32)
        if r >= 1:
            r = np.nextafter(np.float32(1), np.float32(0))
        return np.float32(np.float32(r * np.float32(np.float32(b) - np.float32(a))) + np.float32(a))


_F = np.float32
ISO_BOX = _F(ISO_DIST + _F(_F(5.0) * MIN_CELL_SIZE))


def prim_box(prims, i: int):
    """Per-primitive AABB, PrepareBBoxes (PS_Polygonizer.cpp:71-195), fp32 arithmetic."""
    p = prims[0]
    t = int(p["skeletType"][i])
    pos = np.array([p["posX"][i], p["posY"][i], p["posZ"][i]], np.float32)
    d = np.array([p["dirX"][i], p["dirY"][i], p["dirZ"][i]], np.float32)
    iso = ISO_BOX
    one = _F(1.0)
    if t == NodeType.POINT:
        return pos - iso, pos + iso
    if t == NodeType.LINE:
        ex = (iso * one) + (_F(3.0) * iso) * (d - pos)
        return pos - ex, d + ex
    if t in (NodeType.RING, NodeType.DISC):
        r = _F(p["resX"][i] + iso)
        ex = (r + iso) * (one - d) + iso * d
        return pos - ex, pos + ex
    if t == NodeType.CYLINDER:
        r, h = p["resX"][i], p["resY"][i]
        s1 = pos + h * d
        ex = (iso + r) * one + (_F(0.5) * iso) * d
        return pos - ex, s1 + ex
    if t == NodeType.CUBE:
        s = _F(p["resX"][i] + iso)
        return pos - s, pos + s
    if t == NodeType.TRIANGLE:
        r = np.array([p["resX"][i], p["resY"][i], p["resZ"][i]], np.float32)
        lo = np.minimum(np.minimum(pos, d), r)
        hi = np.maximum(np.maximum(pos, d), r)
        return lo - iso, hi + iso
    lo = np.array([p["vPrimBoxLoX"][i], p["vPrimBoxLoY"][i], p["vPrimBoxLoZ"][i]], np.float32)
    hi = np.array([p["vPrimBoxHiX"][i], p["vPrimBoxHiY"][i], p["vPrimBoxHiZ"][i]], np.float32)
    return lo, hi


def prepare_boxes(model: Model) -> None:
    """Fill prim and op boxes (identity matrices only) and the union scene box."""
    P, O = model.prims, model.ops
    n = model.ct_prims
    los, his = [], []
    for i in range(n):
        lo, hi = prim_box(P, i)
        lo = np.asarray(lo, np.float32)
        hi = np.asarray(hi, np.float32)
        for a, c in enumerate("XYZ"):
            P[f"vPrimBoxLo{c}"][0, i] = lo[a]
            P[f"vPrimBoxHi{c}"][0, i] = hi[a]
        los.append(lo)
        his.append(hi)
    if n:
        P["bboxLo"][0] = np.min(np.stack(los), axis=0)
        P["bboxHi"][0] = np.max(np.stack(his), axis=0)

    def box(is_op, idx):
        src, pre = (O, "vBox") if is_op else (P, "vPrimBox")
        lo = np.array([src[f"{pre}Lo{c}"][0, idx] for c in "XYZ"], np.float32)
        hi = np.array([src[f"{pre}Hi{c}"][0, idx] for c in "XYZ"], np.float32)
        return lo, hi

    def rec(op):
        kind = int(O["opChildKind"][0, op])
        L, R = int(O["opLeftChild"][0, op]), int(O["opRightChild"][0, op])
        if kind & 2:
            rec(L)
        if kind & 1:
            rec(R)
        llo, lhi = box(kind & 2, L)
        rlo, rhi = box(kind & 1, R)
        lo, hi = np.minimum(llo, rlo), np.maximum(lhi, rhi)
        for a, c in enumerate("XYZ"):
            O[f"vBoxLo{c}"][0, op] = lo[a]
            O[f"vBoxHi{c}"][0, op] = hi[a]

    if model.ct_ops:
        rec(0)


def _colour(i: int):
    return (np.float32(((i * 53) % 97) / 96.0), np.float32(((i * 29) % 89) / 88.0),
            np.float32(((i * 17) % 83) / 82.0))


_CYCLE = (NodeType.POINT, NodeType.LINE, NodeType.CYLINDER, NodeType.CUBE)


def set_prim(model: Model, i: int, ptype: int, centre, colour=None) -> None:
    P = model.prims
    c = np.asarray(centre, np.float32)
    P["skeletType"][0, i] = ptype
    P["idxMatrix"][0, i] = 0
    P["posX"][0, i], P["posY"][0, i], P["posZ"][0, i] = c
    if ptype == NodeType.LINE:
        e = c + np.array([0.8, 0.3, 0.0], np.float32)
        P["dirX"][0, i], P["dirY"][0, i], P["dirZ"][0, i] = e
    elif ptype == NodeType.CYLINDER:
        P["dirX"][0, i], P["dirY"][0, i], P["dirZ"][0, i] = (0.0, 1.0, 0.0)
        P["resX"][0, i], P["resY"][0, i] = (0.2, 0.8)
    elif ptype == NodeType.CUBE:
        P["resX"][0, i] = 0.3
    col = _colour(i) if colour is None else colour
    P["colorX"][0, i], P["colorY"][0, i], P["colorZ"][0, i] = col


def build_balanced_ops(model: Model, n_prims: int) -> None:
    """Balanced binary op tree over prims [0, n) with pre-order op ids (root op = 0)."""
    O = model.ops
    counter = [0]

    def rec(a, b, depth):
        if b - a == 1:
            return 0, a
        op = counter[0]
        counter[0] += 1
        mid = (a + b) // 2
        lk, lid = rec(a, mid, depth + 1)
        rk, rid = rec(mid, b, depth + 1)
        if depth == 0:
            t = NodeType.UNION
        elif depth == 1 and op % 2 == 1:
            t = NodeType.DIF
        else:
            t = NodeType.BLEND
        O["opType"][0, op] = t
        O["opLeftChild"][0, op] = lid
        O["opRightChild"][0, op] = rid
        O["opChildKind"][0, op] = lk * 2 + rk
        return 1, op

    if n_prims > 1:
        rec(0, n_prims, 0)
    O["ctOps"][0] = counter[0]


def make_config(name: str, frame: int = 0, seed: int = 42, rng: str = "mt19937"):
    """Return (model, cellsize, N) for one of C1..C5.  ``frame`` animates C5."""
    n_prims, N, half = CONFIGS[name]
    model = Model.empty(name)
    if name == "C1":
        set_prim(model, 0, NodeType.POINT, (0.0, 0.0, 0.0))
        model.prims["ctPrims"][0] = 1
    else:
        if rng == "mt19937":
            gen = MT19937(seed)
            draw = lambda: gen.uniform_f32(-2.0, 2.0)  # noqa: E731
        elif rng == "splitmix64":
            sm = SplitMix64(seed)
            draw = lambda: _F(-2.0) + _F(4.0) * sm.next_f32()  # noqa: E731
        else:
            raise ValueError(f"unknown rng {rng!r}")
        for i in range(n_prims):
            c = np.array([draw() for _ in range(3)], np.float32)
            if name == "C5":
                c[0] = np.float32(c[0] + np.float32(0.25 * math.sin(2.0 * math.pi * frame / 60.0 + i)))
            elif frame:  # C2-C4 animate the same way but keep frame 0 = the reference-probe tree
                c[0] = np.float32(c[0] + np.float32(0.25 * (math.sin(2.0 * math.pi * frame / 60.0 + i) - math.sin(i))))
            set_prim(model, i, _CYCLE[i % 4], c)
        model.prims["ctPrims"][0] = n_prims
        build_balanced_ops(model, n_prims)
    prepare_boxes(model)
    model.prims["bboxLo"][0] = (-half, -half, -half)
    model.prims["bboxHi"][0] = (half, half, half)
    cellsize = float(np.float32(2.0 * half / N))
    return model, cellsize, N


def random_model(seed: int, n_prims: int, types=None, op_types=None, matrices: bool = False,
                 half: float = 2.0) -> Model:
    """Random small trees for parity tests: random prim types/params and op types."""
    rng = np.random.default_rng(seed)
    types = types or [NodeType.POINT, NodeType.LINE, NodeType.CYLINDER, NodeType.CUBE]
    model = Model.empty(f"rand{seed}")
    P = model.prims
    for i in range(n_prims):
        t = int(rng.choice(types))
        c = rng.uniform(-1.2, 1.2, 3).astype(np.float32)
        set_prim(model, i, t, c)
        if t == NodeType.LINE:
            e = c + rng.uniform(-0.8, 0.8, 3).astype(np.float32)
            P["dirX"][0, i], P["dirY"][0, i], P["dirZ"][0, i] = e
        elif t == NodeType.CYLINDER:
            d = rng.normal(size=3)
            d = (d / np.linalg.norm(d)).astype(np.float32)
            P["dirX"][0, i], P["dirY"][0, i], P["dirZ"][0, i] = d
            P["resX"][0, i], P["resY"][0, i] = rng.uniform(0.05, 0.4), rng.uniform(0.2, 1.0)
        elif t == NodeType.CUBE:
            P["resX"][0, i] = rng.uniform(0.1, 0.5)
        elif t in (NodeType.DISC, NodeType.RING):
            d = rng.normal(size=3)
            d = (d / np.linalg.norm(d)).astype(np.float32)
            P["dirX"][0, i], P["dirY"][0, i], P["dirZ"][0, i] = d
            r = np.float32(rng.uniform(0.2, 0.6))
            P["resX"][0, i], P["resY"][0, i] = r, r * r
        if matrices and rng.uniform() < 0.5:
            k = int(model.mats["count"][0])
            ang = rng.uniform(0, 2 * np.pi)
            ca, sa = np.cos(ang), np.sin(ang)
            m = np.array([[ca, -sa, 0, rng.uniform(-0.3, 0.3)], [sa, ca, 0, rng.uniform(-0.3, 0.3)],
                          [0, 0, 1, rng.uniform(-0.3, 0.3)]], np.float32).reshape(-1)
            model.mats["matrix"][0, k * 12:(k + 1) * 12] = m
            model.mats["count"][0] = k + 1
            P["idxMatrix"][0, i] = k
    P["ctPrims"][0] = n_prims
    if n_prims > 1:
        build_balanced_ops(model, n_prims)
        if op_types is not None:
            for op in range(model.ct_ops):
                model.ops["opType"][0, op] = int(rng.choice(op_types))
                model.ops["resY"][0, op] = np.float32(rng.uniform(0.2, 2.0))
    prepare_boxes(model)
    model.prims["bboxLo"][0] = (-half, -half, -half)
    model.prims["bboxHi"][0] = (half, half, half)
    return model

"""Algorithmic work model of the reference field evaluation.

fp32 VALU operations per lane-evaluation, counted from the restated reference formulas
(PS_Polygonizer.cpp:934-1179, 1228-1338) with contraction off: every add, sub, mul,
div, sqrt, compare and select counts one.  Identity matrices cost nothing; a primitive
matrix adds 18 (three rows of 3 mul + 3 add).
"""
from __future__ import annotations

from .soa import Model, NodeType

WYVILL = 4  # 1 - d2, t*t, *t, max
PRIM_OPS = {
    NodeType.POINT: 8 + WYVILL,        # 3 sub, 3 mul, 2 add
    NodeType.LINE: 31 + WYVILL,        # delta 3, |delta|^2 5, d 3, dot 5, div 1, nearest 9, d2 5
    NodeType.CYLINDER: 29 + WYVILL,    # 3 sub, y 5, r^2 7, sqrt/-r/max 3, mask/cap 8, d2 3
    NodeType.CUBE: 33 + WYVILL,        # 3 sub, 3 axes x (2 cmp, 2 sel, add, sub, 2 mul, add) + 3 acc
    NodeType.DISC: 40 + WYVILL,
    NodeType.RING: 42 + WYVILL,
    NodeType.TRIANGLE: WYVILL,
}
OP_OPS = {NodeType.BLEND: 1, NodeType.UNION: 2, NodeType.INTERSECT: 2, NodeType.DIF: 3,
          NodeType.SMOOTHDIF: 2, NodeType.RICCIBLEND: 6}
BOX_TEST = 14  # depth > 3: 6 compares, 3 and, 2 or, quad reduction


def ops_per_eval(model: Model) -> int:
    """Operations of one full (unpruned) tree evaluation of one point."""
    P, O = model.prims[0], model.ops[0]
    cost = 0

    def prim(i):
        c = PRIM_OPS.get(int(P["skeletType"][i]), WYVILL)
        return c + (18 if P["idxMatrix"][i] else 0)

    if model.ct_ops == 0:
        return sum(prim(i) + 1 for i in range(model.ct_prims))

    def rec(op, depth):
        nonlocal cost
        kind = int(O["opChildKind"][op])
        L, R = int(O["opLeftChild"][op]), int(O["opRightChild"][op])
        t = int(O["opType"][op])
        if depth > 3:
            cost += BOX_TEST
        if kind & 1:
            rec(R, depth + 1)
        elif t in OP_OPS or t in (NodeType.WARPTWIST,):
            cost += prim(R) if t in OP_OPS else 0
        if kind & 2:
            rec(L, depth + 1)
        elif t in OP_OPS or 22 <= t <= 25:
            cost += prim(L)
        cost += OP_OPS.get(t, 0)

    rec(0, 0)
    return cost


def lane_evals(ct_mpus: int, ct_passed: int, ct_vertices: int) -> int:
    """Lane-evaluations of one polygonization: 8 per MPU (S1), 512 per S1 survivor (S2),
    8 per vertex (4 root samples, 1 field+colour, 3 normal samples)."""
    return 8 * ct_mpus + 512 * ct_passed + 8 * ct_vertices

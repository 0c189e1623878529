"""Multi-GPU partition of the MPU lattice.

MPUs are independent (each evaluates its own 8^3 corners, shared faces included), so the
multi-GPU path needs no halo and no data-path collective:

* weak scaling: every rank polygonizes its own grid (its own animation frame);
* strong scaling: one grid split into contiguous ranges of the x-major MPU index.
  Concatenating the rank outputs in rank order reproduces the single-GPU MPU order, so
  the only exchange is a 3-integer all-gather (MPUs, vertices, triangles) from which every
  rank knows where its part lands in the global vertex / triangle index space.
"""
from __future__ import annotations

import numpy as np


def mpu_ranges(n_mpus: int, world: int, weights: np.ndarray | None = None) -> list[tuple[int, int]]:
    """Contiguous [begin, end) MPU ranges, one per rank, covering [0, n_mpus) in order.

    Without weights the split is even by MPU count.  With per-MPU ``weights`` (e.g. 1 for
    MPUs that pass the S1 precheck, 512 evals each, 8 evals otherwise) the cut points
    balance the prefix sum of the weights.
    """
    if world < 1:
        raise ValueError("world must be >= 1")
    if weights is None:
        per, extra = divmod(n_mpus, world)
        cuts = [0]
        for r in range(world):
            cuts.append(cuts[-1] + per + (1 if r < extra else 0))
    else:
        w = np.asarray(weights, np.float64)
        if len(w) != n_mpus:
            raise ValueError("weights must have one entry per MPU")
        csum = np.concatenate([[0.0], np.cumsum(w)])
        targets = csum[-1] * np.arange(1, world) / world
        inner = np.searchsorted(csum, targets, side="left").tolist()
        cuts = [0] + [int(min(max(c, 0), n_mpus)) for c in inner] + [n_mpus]
        for r in range(1, len(cuts)):
            cuts[r] = max(cuts[r], cuts[r - 1])
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


def exclusive_offsets(per_rank_counts) -> np.ndarray:
    """Rank -> (mpu, vertex, triangle) offset of that rank's part in the global mesh.

    ``per_rank_counts`` is the all-gathered (ctMPUs, ctVertices, ctTriangles) per rank.
    """
    c = np.asarray(per_rank_counts, np.int64).reshape(len(per_rank_counts), -1)
    return np.concatenate([np.zeros((1, c.shape[1]), np.int64), np.cumsum(c, axis=0)[:-1]])


def globalize_triangles(tris_rank: np.ndarray, vertex_offset: int) -> np.ndarray:
    """A rank's triangles (rank-global vertex ids) shifted into the job-global index space."""
    return np.asarray(tris_rank, np.int64) + int(vertex_offset)

"""Seeded fuzz parity: random trees over every primitive and operator type (warps included),
random matrices, cell sizes off the round values, ragged MPU ranges (a rank's share starts and
ends anywhere in the lattice), culling on and off, the interpreter and the generated kernels,
every k_vertex / k_finish layout, the tree split, the fused k_surface and k_front -- the HIP path through the C-ABI against
the CPU oracle, bit-exact (tests/parity_util.py)."""
import numpy as np
import pytest

from parity_util import assert_mesh_matches
from parsip_amd import gpu, soa, synth
from parsip_amd.soa import NodeType

pytestmark = pytest.mark.gpu

TYPES = [NodeType.POINT, NodeType.LINE, NodeType.CYLINDER, NodeType.CUBE, NodeType.DISC, NodeType.RING,
         NodeType.TRIANGLE]
OPS = [NodeType.BLEND, NodeType.UNION, NodeType.INTERSECT, NodeType.DIF, NodeType.SMOOTHDIF, NodeType.RICCIBLEND,
       NodeType.GRADIENTBLEND, NodeType.WARPTWIST, NodeType.WARPTAPER, NodeType.WARPBEND, NodeType.WARPSHEAR]


def fuzz_case(seed):
    rng = np.random.default_rng(1000 + seed)
    n = int(rng.integers(2, 25))
    model = synth.random_model(1000 + seed, n_prims=n, types=TYPES, op_types=OPS, matrices=bool(rng.integers(0, 2)))
    cs = float(np.float32(rng.uniform(4.0 / 120, 4.0 / 20)))
    total = int(np.prod(soa.mpu_dims(cs, *model.bbox)))
    begin = int(rng.integers(0, max(1, total // 3)))
    end = int(rng.integers(max(begin + 1, 2 * total // 3), total + 1))
    layout = (int(rng.integers(0, 3)), int(rng.integers(0, 4)), int(rng.integers(0, 2)))  # vwide, fquad, split
    return model, cs, begin, end, int(rng.integers(0, 2)), (1, 0)[seed % 2], layout


@pytest.mark.parametrize("seed", range(40))  # seeds 3, 7, 10, 21, 26: empty meshes (the empty path)
def test_fuzz_ranges_and_trees(gpu_poly, oracle, seed):
    model, cs, begin, end, cull, jit, (vwide, fquad, split) = fuzz_case(seed)
    try:
        gpu_poly.set_option(gpu.OPT_CULLING, cull)
        gpu_poly.set_option(gpu.OPT_JIT, jit)
        gpu_poly.set_option(gpu.OPT_VERTEX_WIDE, vwide)
        gpu_poly.set_option(gpu.OPT_FINISH_QUAD, fquad)
        front = (seed // 2) % 3  # k_front (with the small-launch kernels: split 0 compiles them as 2)
        gpu_poly.set_option(gpu.OPT_TREE_SPLIT, (split if split or not front else 2) if jit else 0)
        gpu_poly.set_option(gpu.OPT_FUSED_SURFACE, seed % 4)  # k_surface (3: k_surface_w) when the split compiled it
        gpu_poly.set_option(gpu.OPT_FRONT, front)
        gpu_poly.set_model(model)
        assert gpu_poly.jit_active == bool(jit)
        gpu_poly.run(cs, begin, end)
        gm = gpu_poly.download()
        gs = gpu_poly.stats()
    finally:  # the session's context goes back to the defaults
        gpu_poly.set_option(gpu.OPT_CULLING, 1)
        gpu_poly.set_option(gpu.OPT_JIT, 1)
        gpu_poly.set_option(gpu.OPT_VERTEX_WIDE, 2)
        gpu_poly.set_option(gpu.OPT_FINISH_QUAD, 2)
        gpu_poly.set_option(gpu.OPT_TREE_SPLIT, 0)
        gpu_poly.set_option(gpu.OPT_FUSED_SURFACE, 2)
        gpu_poly.set_option(gpu.OPT_FRONT, 2)
    om = oracle.polygonize(model, cs, begin, end, threads=8)
    assert_mesh_matches(gm, gs, om)

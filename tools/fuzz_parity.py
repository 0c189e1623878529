"""Long seeded fuzz run of the GPU path against the oracle (the cases of tests/test_gpu_fuzz.py,
many more seeds): random trees over every node type, matrices, off-round cell sizes, ragged
MPU ranges, culling on / off, interpreter / generated kernels, every layout, the tree split,
the fused k_surface / k_surface_w and k_front.  Prints one line per failure and a summary; exit status 1 if any case differs.

Usage (GPU): python tools/fuzz_parity.py [--first 0] [--count 400] [--big]
(--big: trees of 25-64 primitives; the generated kernels on every fourth case, the
interpreter on the others, since a large tree's hiprtc compile takes tens of seconds)
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--first", type=int, default=0)
    ap.add_argument("--count", type=int, default=400)
    ap.add_argument("--big", action="store_true")
    a = ap.parse_args()
    import psoracle
    import numpy as np
    import test_gpu_fuzz as fz
    from parity_util import assert_mesh_matches

    from parsip_amd import gpu, soa, synth

    psoracle.build()
    poly = gpu.Polygonizer(0)
    fails, verts, t0 = [], 0, time.time()
    for seed in range(a.first, a.first + a.count):
        model, cs, begin, end, cull, jit, (vwide, fquad, split) = fz.fuzz_case(seed)
        if a.big:
            rng = np.random.default_rng(9000 + seed)
            model = synth.random_model(9000 + seed, n_prims=int(rng.integers(25, 65)), types=fz.TYPES,
                                       op_types=fz.OPS, matrices=bool(rng.integers(0, 2)))
            cs = float(np.float32(rng.uniform(4.0 / 100, 4.0 / 40)))
            total = int(np.prod(soa.mpu_dims(cs, *model.bbox)))
            begin = int(rng.integers(0, max(1, total // 3)))
            end = int(rng.integers(max(begin + 1, 2 * total // 3), total + 1))
            jit = 1 if seed % 4 == 0 else 0
        poly.set_option(gpu.OPT_CULLING, cull)
        poly.set_option(gpu.OPT_JIT, jit)
        poly.set_option(gpu.OPT_VERTEX_WIDE, vwide)
        poly.set_option(gpu.OPT_FINISH_QUAD, fquad)
        front = (seed // 2) % 3  # k_front (with the small-launch kernels: split 0 compiles them as 2)
        poly.set_option(gpu.OPT_TREE_SPLIT, (split if split or not front else 2) if jit else 0)
        poly.set_option(gpu.OPT_FUSED_SURFACE, seed % 4)  # k_surface (3: k_surface_w) when the split compiled it
        poly.set_option(gpu.OPT_FRONT, front)
        poly.set_model(model)  # waits for the generated kernels when jit is on
        assert poly.jit_active == bool(jit), seed
        poly.run(cs, begin, end)
        gm, gs = poly.download(), poly.stats()
        om = psoracle.polygonize(model, cs, begin, end, threads=8)
        verts += len(om.pos)
        try:
            assert_mesh_matches(gm, gs, om)
        except AssertionError as e:
            fails.append(seed)
            print(f"seed {seed}: {str(e).splitlines()[0][:300]}", flush=True)
        if (seed - a.first) % 50 == 49:
            print(f"... {seed - a.first + 1} cases, {len(fails)} failing, {time.time() - t0:.0f} s", flush=True)
    poly.close()
    print(f"fuzz seeds [{a.first}, {a.first + a.count}): {a.count - len(fails)} bit-exact, {len(fails)} differ "
          f"({verts} oracle vertices in all), {time.time() - t0:.0f} s")
    sys.exit(1 if fails else 0)


if __name__ == "__main__":
    main()

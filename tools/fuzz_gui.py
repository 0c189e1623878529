"""Long seeded fuzz run of the compat mode (the GUI path, psgpu_gui_*) against its oracle
(oracle/psgui.c): random trees of every supported node type (tests/gui_util.py random_tree),
random cell sizes and iso values, interpreter / generated kernels, culling on / off; compares
the exported mesh and the run info bit for bit (tests/test_gui.py's checks).  Exit status 1 if
any case differs.

Usage (GPU): python tools/fuzz_gui.py [--first 100] [--count 120]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--first", type=int, default=100)
    ap.add_argument("--count", type=int, default=120)
    a = ap.parse_args()
    import psgui
    from gui_util import assert_gui_mesh_equal, random_tree
    from parsip_amd import gpu, gui

    gpu.load()
    ctxs = {(j, c): gui.ParsipOptimized(0, jit=j, cull=c) for j in (0, 2) for c in (0, 1)}
    fails, verts, t0 = [], 0, time.time()
    for seed in range(a.first, a.first + a.count):
        rng = np.random.default_rng(5000 + seed)
        code, tree = gui.compact_blobtree(random_tree(seed, n_prims=int(rng.integers(2, 16))))
        if code != 0:
            print(f"seed {seed}: conversion code {code} (skipped)")
            continue
        cs = float(np.float32(rng.uniform(0.04, 0.2)))
        iso = float(np.float32(rng.choice([0.5, 0.5, 0.3, 0.7])))
        ctx = ctxs[(int(rng.choice([0, 2])), int(rng.integers(0, 2)))]
        lo, hi = tree.root_octree
        ctx.setup(tree, (lo, hi), 0, cs, iso)
        ctx.run()
        gm = ctx.exportMesh()
        info = ctx.finish()
        om = psgui.polygonize(tree, lo, hi, cs, iso, threads=8)
        verts += int(om.info.ctVertices) if hasattr(om.info, "ctVertices") else 0
        try:
            for f, _ in gui.PsGuiInfo._fields_:
                va, vb = getattr(info, f), getattr(om.info, f)
                if f == "dims":
                    va, vb = list(va), list(vb)
                assert va == vb, (f, va, vb)
            assert_gui_mesh_equal(gm, om, f"seed {seed}")
        except AssertionError as e:
            fails.append(seed)
            print(f"seed {seed}: {str(e).splitlines()[0][:300]}", flush=True)
        if (seed - a.first) % 30 == 29:
            print(f"... {seed - a.first + 1} cases, {len(fails)} failing, {time.time() - t0:.0f} s", flush=True)
    for c in ctxs.values():
        c.close()
    print(f"compat-mode fuzz seeds [{a.first}, {a.first + a.count}): {a.count - len(fails)} bit-exact, "
          f"{len(fails)} differ ({verts} oracle vertices in all), {time.time() - t0:.0f} s")
    sys.exit(1 if fails else 0)


if __name__ == "__main__":
    main()

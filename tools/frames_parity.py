"""Per-frame parity of an animated configuration (C5: 512^3 cells, 64-primitive tree, re-polygonized
per frame; BASELINE.json configs[4]) against the oracle, over many frames: every frame on one
context as the animation driver runs it (set_model per frame, the generated kernels when they are
ready, graph replay on odd frames), bit-exact to the oracle's output (psoracle, 16 threads), and
the same frame split over 8 parts of one device (a Group), whose concatenated mesh must equal the
single context's.  Exit status 1 if any frame differs.

Usage (GPU): python tools/frames_parity.py [--config C5] [--first 0] [--count 12]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C5")
    ap.add_argument("--first", type=int, default=0)
    ap.add_argument("--count", type=int, default=12)
    ap.add_argument("--threads", type=int, default=16)
    a = ap.parse_args()
    import numpy as np
    import psoracle
    from parity_util import assert_bits_equal, assert_mesh_matches

    from parsip_amd import gpu, synth

    psoracle.build()
    poly = gpu.Polygonizer(0)
    grp = gpu.Group([0] * 8)
    fails, verts, t0 = [], 0, time.time()
    for f in range(a.first, a.first + a.count):
        model, cs, _ = synth.make_config(a.config, frame=f)
        poly.set_option(gpu.OPT_GRAPH, f & 1)
        poly.set_model(model, wait_jit=f == a.first)  # later frames: the structure kernels are loaded
        info = poly.run(cs)
        gm, gs = poly.download(), poly.stats()
        grp.set_model(model)
        grp.run(cs)
        pm = grp.download()
        om = psoracle.polygonize(model, cs, threads=a.threads)
        verts += len(om.pos)
        try:
            assert_mesh_matches(gm, gs, om)
            np.testing.assert_array_equal(pm.tris, gm.tris, err_msg="8-part triangles")
            np.testing.assert_array_equal(pm.vertex_offsets, gm.vertex_offsets, err_msg="8-part offsets")
            for k in ("pos", "nrm", "col"):
                assert_bits_equal(getattr(pm, k), getattr(gm, k), "8-part " + k)
        except AssertionError as e:
            fails.append(f)
            print(f"frame {f}: {str(e).splitlines()[0][:300]}", flush=True)
        print(f"frame {f}: V {info.ctVertices} T {info.ctTriangles} launch flags {info.launchFlags} "
              f"jit tier {poly.jit_tier} {'ok' if f not in fails else 'DIFFERS'} ({time.time() - t0:.0f} s)", flush=True)
    grp.close()
    poly.close()
    print(f"{a.config} frames [{a.first}, {a.first + a.count}): {a.count - len(fails)} bit-exact, {len(fails)} differ "
          f"({verts} oracle vertices in all), {time.time() - t0:.0f} s")
    sys.exit(1 if fails else 0)


if __name__ == "__main__":
    main()

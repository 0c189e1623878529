"""Compat mode (GUI path) timing: ParsipHaptics' train scene through CParsipOptimized on
the MI355X library (wall clock of setup+run, median of repeats) and through the CPU
restatement (oracle/psgui.c, host threads).  Prints one JSON line per cell size."""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from parsip_amd import gui, scene  # noqa: E402


def main():
    sizes = [float(a) for a in sys.argv[1:] if not a.startswith("--")] or [0.13, 0.05]
    root = scene.load_scene(os.path.join(ROOT, "tests", "golden", "train_corrected.scene"))[0]
    code, tree = gui.compact_blobtree(root)
    p = gui.ParsipOptimized(0)
    threads = int(os.environ.get("PSGPU_CPU_THREADS", "16"))
    for cs in sizes:
        p.setup(tree, tree.root_octree, 0, cs, 0.5)
        p.run()
        ts = []
        for _ in range(10):
            t0 = time.perf_counter()
            p.run()
            ts.append(time.perf_counter() - t0)
        i = p.finish()
        out = {"cellsize": cs, "gpu_ms": round(statistics.median(ts) * 1e3, 3), "lattice_mpus": i.ctLatticeMPUs,
               "processed_mpus": i.ctProcessedMPUs, "vertices": i.ctVertices, "triangles": i.ctTriangles,
               "field_evals": i.ctFieldEvals}
        if "--no-cpu" not in sys.argv:
            import psgui

            t0 = time.perf_counter()
            r = psgui.polygonize(tree, *tree.root_octree, cs, 0.5, threads=threads)
            out["cpu_ms"] = round((time.perf_counter() - t0) * 1e3, 1)
            out["cpu_threads"] = threads
            out["same_counts"] = (r.info.ctVertices, r.info.ctTriangles) == (i.ctVertices, i.ctTriangles)
        print(json.dumps(out), flush=True)
    p.close()


if __name__ == "__main__":
    main()

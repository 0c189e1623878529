"""Per-frame re-polygonization of an animated BlobTree.

The reference's animation loop (GLWidget::advanceAnimation,
Parsip100/ParsipHaptics/include/glwidget.cpp:3919-3940) advances the animated nodes
to time t, bumps the layer and re-polygonizes, t += ANIMATION_FRAME_TIME * speed until
t reaches 1.  Here a frame is: host model for frame f -> ``set_model`` (a 28 KB upload;
the specialised kernels depend on the tree's structure only, so animating parameters
never recompiles) -> the five-kernel polygonization, optionally replayed from a
hipGraph.  The mesh stays in HBM; ``sink`` receives the device-resident mesh
(``PsMeshDevice``) or, with ``download=True``, host arrays.

    python -m parsip_amd.animate --config C5 --frames 60
"""
from __future__ import annotations

import argparse
import json
import time

from . import gpu, synth


class Animation:
    def __init__(self, poly: "gpu.Polygonizer", frame_model, cellsize: float, graph: bool = True):
        self.poly = poly
        self.frame_model = frame_model  # f -> soa.Model
        self.cellsize = cellsize
        poly.set_option(gpu.OPT_GRAPH, 1 if graph else 0)

    def run(self, frames: int, sink=None, download: bool = False) -> dict:
        t0 = time.perf_counter()
        host = 0.0
        verts = tris = 0
        for f in range(frames):
            h = time.perf_counter()
            model = self.frame_model(f)
            self.poly.set_model(model)
            host += time.perf_counter() - h
            self.poly.polygonize(self.cellsize)
            info = self.poly.finish()
            verts += info.ctVertices
            tris += info.ctTriangles
            if sink is not None:
                sink(f, self.poly.download() if download else self.poly.device_mesh())
        dt = time.perf_counter() - t0
        return {"frames": frames, "seconds": dt, "frames_per_s": frames / dt, "host_model_s": host,
                "vertices": verts, "triangles": tris}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C5")
    ap.add_argument("--frames", type=int, default=60)
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--no-graph", action="store_true")
    a = ap.parse_args()
    _, cs, n = synth.make_config(a.config)
    poly = gpu.Polygonizer(a.device)
    anim = Animation(poly, lambda f: synth.make_config(a.config, frame=f)[0], cs, graph=not a.no_graph)
    anim.run(2)  # kernels compiled / cached, buffers sized
    out = anim.run(a.frames)
    out["config"] = a.config
    out["mcells_per_s"] = n ** 3 * a.frames / out["seconds"] / 1e6
    print(json.dumps(out))
    poly.close()


if __name__ == "__main__":
    main()

"""Time one frame split into K cost-balanced MPU ranges on K streams of ONE device
(psgpu_group with every part on device 0), against a single context.
usage: python tools/ab_parts.py [--config C3] [--rounds 11] 1 2 3 4"""
import argparse
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from parsip_amd import gpu, synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--rounds", type=int, default=11)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("parts", nargs="+", type=int)
    a = ap.parse_args()
    model, cs, N = synth.make_config(a.config)
    groups = {}
    for k in a.parts:
        g = gpu.Group([0] * k)
        g.set_model(model)
        info, _ = g.run(cs)
        print(f"K={k} V={info.ctVertices} T={info.ctTriangles} split={list(g.split())}", flush=True)
        groups[k] = g
    res = {k: [] for k in a.parts}
    for _ in range(a.rounds):
        for k, g in groups.items():
            t0 = time.perf_counter()
            for _ in range(a.steps):
                g.polygonize(cs)
            g.finish()
            res[k].append((time.perf_counter() - t0) / a.steps * 1e6)
    for k in a.parts:
        print(f"K={k}: median {statistics.median(res[k]):.1f} us/frame (min {min(res[k]):.1f})")


if __name__ == "__main__":
    main()

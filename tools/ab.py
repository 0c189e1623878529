"""Interleaved A/B timing of polygonizer variants in ONE process (one device, same clocks).

usage: python tools/ab.py [--config C3] [--rounds 15] "jit=1" "jit=1,debug=1" ...
Each variant is a comma list of option=value (jit, cull, debug).  Prints the median
per-kernel hipEvent times and the median whole-step time of every variant.
"""
import argparse
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from parsip_amd import gpu, synth  # noqa: E402

OPT = {"jit": gpu.OPT_JIT, "cull": gpu.OPT_CULLING, "debug": gpu.OPT_DEBUG, "graph": gpu.OPT_GRAPH, "vb": gpu.OPT_VERTEX_BLOCKS_PER_CU,
       "fb": gpu.OPT_FINISH_BLOCKS_PER_CU, "bound": gpu.OPT_BOUND, "fq": gpu.OPT_FINISH_QUAD,
       "vw": gpu.OPT_VERTEX_WIDE, "split": gpu.OPT_TREE_SPLIT}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--rounds", type=int, default=15)
    ap.add_argument("variants", nargs="+")
    a = ap.parse_args()
    model, cs, N = synth.make_config(a.config)
    polys = []
    for v in a.variants:
        p = gpu.Polygonizer(0)
        os.environ.pop("PSGPU_JIT_FLAGS", None)
        for kv in v.split(","):
            k, val = kv.split("=", 1)
            if k == "flags":  # extra hiprtc flags for this variant's kernels ('+' separates)
                os.environ["PSGPU_JIT_FLAGS"] = val.replace("+", " ")
                continue
            p.set_option(OPT[k], int(val))
        p.set_model(model)
        os.environ.pop("PSGPU_JIT_FLAGS", None)
        info = p.run(cs)
        print(f"{v:28s} V={info.ctVertices} T={info.ctTriangles} passedS1={info.ctPassedPrecheck} "
              f"fieldMPUs={info.ctFieldMPUs} surface={info.ctSurfaceMPUs}", flush=True)
        polys.append(p)
    kt = {v: {} for v in a.variants}
    step = {v: [] for v in a.variants}
    for _ in range(a.rounds):
        for v, p in zip(a.variants, polys):
            p.set_option(gpu.OPT_KERNEL_TIMING, 0)
            t0 = time.perf_counter()
            for _ in range(5):
                p.polygonize(cs)
            p.finish()
            step[v].append((time.perf_counter() - t0) / 5 * 1e3)
            p.set_option(gpu.OPT_KERNEL_TIMING, 1)
            p.run(cs)
            for k, ms in p.kernel_times().items():
                kt[v].setdefault(k, []).append(ms)
    for v in a.variants:
        ks = " ".join(f"{k}={statistics.median(x) * 1e3:.1f}" for k, x in kt[v].items())
        print(f"{v:28s} step={statistics.median(step[v]) * 1e3:.1f}us  {ks}")


if __name__ == "__main__":
    main()

"""Where a short timed loop loses time: the bench's engines (4 contexts taking the steps in
turn, queued without host sync) over K = 5 .. 320 steps; per K the host time of the whole
loop (median of 5) and, from OPT_SPANS, the device timeline: first kernel start -> last
kernel end, and how long the device ran fewer than 4 / 2 runs at once (fill and drain).
usage: python tools/k_sweep.py [--config C3] [--jit 1] [--engines 4]"""
import argparse
import os
import statistics
import sys
import time

os.environ["GPU_MAX_HW_QUEUES"] = "8"  # as bench.py: every engine on a hardware queue of its own
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from parsip_amd import gpu, synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--jit", type=int, default=1)
    ap.add_argument("--engines", type=int, default=4)
    ap.add_argument("--ks", default="5,10,20,40,80,160,320")
    a = ap.parse_args()
    model, cs, N = synth.make_config(a.config)
    E = a.engines
    engines = []
    for e in range(E):
        p = gpu.Polygonizer(0)
        if E > 1:
            p.set_option(gpu.OPT_VERTEX_BLOCKS_PER_CU, 8)
            p.set_option(gpu.OPT_FINISH_BLOCKS_PER_CU, 4)
        p.set_option(gpu.OPT_JIT, a.jit)
        p.set_model(model)
        p.run(cs)
        engines.append(p)
    for K in [int(x) for x in a.ks.split(",")]:
        host = []
        for rep in range(5):
            for k in range(max(5, E)):
                engines[k % E].polygonize(cs)
            for p in engines:
                p.finish()
            spans = rep == 4
            if spans:
                for p in engines:
                    p.set_option(gpu.OPT_SPANS, K // E + 2)
            t0 = time.perf_counter()
            for k in range(K):
                engines[k % E].polygonize(cs)
            for p in engines:
                p.finish()
            host.append((time.perf_counter() - t0) * 1e3)
        runs = np.concatenate([p.spans(raw=True) for p in engines])  # (K, 4, 2)
        for p in engines:
            p.set_option(gpu.OPT_SPANS, 0)
        starts, ends = runs[:, 0, 0], runs[:, 3, 1]
        t0d, t1d = starts.min(), ends.max()
        grid = np.arange(t0d, t1d, 10)  # 0.1 us bins
        live = ((starts[None, :] <= grid[:, None]) & (ends[None, :] > grid[:, None])).sum(1)
        lat = (ends - starts) * 1e-2
        print(f"K={K:4d} host {statistics.median(host):8.3f} ms = {statistics.median(host) / K * 1e3:6.1f} us/step | "
              f"device first->last {(t1d - t0d) * 1e-2:8.1f} us = {(t1d - t0d) * 1e-2 / K:5.1f} us/step | "
              f"<{E} runs live {np.count_nonzero(live < E) * 0.1:6.1f} us, <2 {np.count_nonzero(live < 2) * 0.1:6.1f} us | "
              f"run latency p50 {np.median(lat):6.1f} max {lat.max():6.1f} us", flush=True)


if __name__ == "__main__":
    main()

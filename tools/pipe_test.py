"""Throughput of consecutive complete polygonizations spread over several engines on one
device (each engine = one context / stream, or a Group of cost-balanced parts)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from parsip_amd import gpu, synth  # noqa: E402

model, cs, N = synth.make_config("C3")
plan = gpu.Polygonizer(0)
plan.set_model(model)
plan.run(cs)
costs = plan.mpu_costs()


def make(parts):
    if parts == 1:
        p = gpu.Polygonizer(0)
        p.set_model(model)
        return p, (lambda: p.polygonize(cs)), p.finish
    g = gpu.Group([0] * parts)
    g.set_model(model)
    g.set_split(gpu.split_costs(costs, parts))
    return g, (lambda: g.polygonize(cs)), g.finish


for neng, parts in [(1, 1), (1, 2), (2, 1), (3, 1), (4, 1), (2, 2), (1, 3), (1, 4)]:
    engs = [make(parts) for _ in range(neng)]
    for e, run, fin in engs:
        run(); fin(); run(); fin()
    K = 600
    t0 = time.perf_counter()
    for k in range(K):
        e, run, fin = engs[k % neng]
        run()  # queued behind the engine's previous run (stream order), no host sync
    for e, run, fin in engs:
        fin()
    dt = time.perf_counter() - t0
    print(f"{neng} engines x {parts} parts: ms/step {dt / K * 1e3:.4f}", flush=True)
    for e, _, _ in engs:
        e.close()

"""1/8 rank share of C3 with 2 engines: persistent grid sizes (k_vertex / k_finish blocks per CU)."""
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
for ranks in (8, 1):
    b = gpu.split_costs(costs, ranks)
    lo, hi = int(b[0]), int(b[1])
    for vb, fb in ((16, 8), (8, 4), (4, 2), (2, 1), (1, 1)):
        ps = []
        for _ in range(2):
            p = gpu.Polygonizer(0)
            p.set_option(gpu.OPT_VERTEX_BLOCKS_PER_CU, vb)
            p.set_option(gpu.OPT_FINISH_BLOCKS_PER_CU, fb)
            p.set_model(model)
            p.run(cs, lo, hi)
            ps.append(p)
        K = 400
        for k in range(20):
            ps[k % 2].polygonize(cs, lo, hi)
        for p in ps:
            p.finish()
        t0 = time.perf_counter()
        for k in range(K):
            ps[k % 2].polygonize(cs, lo, hi)
        for p in ps:
            p.finish()
        dt = (time.perf_counter() - t0) / K * 1e3
        print(f"share 1/{ranks}: vb {vb} fb {fb}: {dt:.4f} ms/step", flush=True)
        for p in ps:
            p.close()

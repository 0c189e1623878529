"""Strong-scaling rehearsal, latency side: one polygonization of ONE rank's share of C3 (the
first range of the cost-balanced 1/N split) with the device to itself — per-kernel hipEvent
times (OPT_KERNEL_TIMING) and the host-observed run latency, medians over 30 runs."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from parsip_amd import gpu, synth  # noqa: E402

model, cs, N = synth.make_config("C3")
p = gpu.Polygonizer(0)
p.set_model(model)
p.run(cs)
costs = p.mpu_costs()
p.set_option(gpu.OPT_KERNEL_TIMING, 1)
for ranks in [int(x) for x in os.environ.get("SHARES", "1,2,4,8").split(",")]:
    b = gpu.split_costs(costs, ranks)
    lo, hi = int(b[0]), int(b[1])
    for _ in range(5):
        p.run(cs, lo, hi)
    kt, wall = [], []
    for _ in range(30):
        t0 = time.perf_counter()
        info = p.run(cs, lo, hi)
        wall.append((time.perf_counter() - t0) * 1e3)
        kt.append(p.kernel_times())
    med = {k: round(float(np.median([d[k] for d in kt])), 4) for k in kt[0]}
    print(f"share 1/{ranks} MPUs {hi - lo} fieldMPUs {info.ctFieldMPUs} V {info.ctVertices}: "
          f"run {np.median(wall):.4f} ms, kernels {med}", flush=True)
p.close()

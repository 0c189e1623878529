"""Per-call times of the blocking contract (psgpu_polygonize_mpus) in the order bench.py's
extras run it: one context that polygonized C3, then C2 into a 24,000-MPU PolyMPUs array, then
C3 into a 50,653-MPU one.  ENGINES=n keeps n more idle contexts alive, as the bench process
does; DEBUG=4194304 (bit 22): the transfers without the scatter.  Prints every call's ms,
to tell a slow median from a bimodal one."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from parsip_amd import gpu, soa, synth  # noqa: E402

keep = [gpu.Polygonizer(0) for _ in range(int(os.environ.get("ENGINES", "0")))]
poly = gpu.Polygonizer(0)
poly.set_option(gpu.OPT_JIT, 1)
if os.environ.get("DEBUG"):
    poly.set_option(gpu.OPT_DEBUG, int(os.environ["DEBUG"]))
m3, cs3, _ = synth.make_config("C3")
poly.set_model(m3)
poly.run(cs3)
for cfg in os.environ.get("CONFIGS", "C2,C3").split(","):
    model, cs, n = synth.make_config(cfg)
    ct = gpu.count_mpus(cs, *model.bbox)
    out = np.zeros(max(soa.MAX_MPU_COUNT, ct), soa.MPU_DTYPE)
    t = []
    for _ in range(int(os.environ.get("REPS", "12"))):
        t0 = time.perf_counter()
        rc, c, _ = poly.polygonize_mpus(cs, model, out)
        t.append((time.perf_counter() - t0) * 1e3)
        assert rc == 1 and c == ct
    print(cfg, "median %.3f" % float(np.median(t)), " ".join("%.3f" % x for x in t), flush=True)

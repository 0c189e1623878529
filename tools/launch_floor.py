"""Launch floor: ms/step of a 1-MPU (and 64-MPU) range with 1, 2, 4 engines, and for
comparison an empty hip kernel via torch (if available)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from parsip_amd import gpu, synth  # noqa: E402

model, cs, N = synth.make_config("C3")
for lo, hi in ((25000, 25001), (25000, 25064)):
    for neng in (1, 2, 4):
        ps = []
        for _ in range(neng):
            p = gpu.Polygonizer(0)
            p.set_model(model)
            p.run(cs, lo, hi)
            ps.append(p)
        K = 1000
        for k in range(20):
            ps[k % neng].polygonize(cs, lo, hi)
        for p in ps:
            p.finish()
        t0 = time.perf_counter()
        for k in range(K):
            ps[k % neng].polygonize(cs, lo, hi)
        t1 = time.perf_counter()
        for p in ps:
            p.finish()
        dt = (time.perf_counter() - t0) / K * 1e3
        print(f"range {hi - lo} MPUs, {neng} engines: {dt:.4f} ms/step (host enqueue {(t1 - t0) / K * 1e3:.4f} ms)",
              flush=True)
        for p in ps:
            p.close()

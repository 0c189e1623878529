"""Per-call times of the blocking contract (psgpu_polygonize_mpus / the 2-part group's), in the
order bench.py's extras run them: a context that polygonized C3, then C2 and C3 calls alternating
between one context and a 2-part group of the device (blocking_contract), 2 warm-ups each.
With PSGPU_EXPORT_TRACE=1 (set here unless TRACE=0) the library prints every call's phases to
stderr (ms from the call's start: kernels done, packing enqueued, metadata in, first scatter
task, each piece in, scatter done, end); this script prints each call's host time and, at the
end, the per-phase medians of the fast calls against the slow ones (slower than 1.3 x the
median), which names the phase the tail is spent in.
Env: ENGINES=n more idle contexts alive (as the bench process); REPS (24); CONFIGS (C2,C3);
GROUP=0 for the one-context engine alone; DEBUG=4194304 (bit 22): the transfers without the scatter.
Usage (GPU): python tools/blocking_seq.py 2> trace.txt"""
import os
import sys
import time

if os.environ.get("TRACE", "1") != "0":
    os.environ["PSGPU_EXPORT_TRACE"] = "1"
import numpy as np  # noqa: E402

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
engines = {"one": poly}
if os.environ.get("GROUP", "1") != "0":
    g = gpu.Group([0, 0])
    g.set_option(gpu.OPT_JIT, 1)
    engines["2parts"] = g
REPS = int(os.environ.get("REPS", "24"))
for cfg in os.environ.get("CONFIGS", "C2,C3").split(","):
    model, cs, n = synth.make_config(cfg)
    ct = gpu.count_mpus(cs, *model.bbox)
    out = np.zeros(max(soa.MAX_MPU_COUNT, ct), soa.MPU_DTYPE)
    t = {k: [] for k in engines}
    for rep in range(REPS + 2):
        for k, e in engines.items():
            sys.stderr.flush()
            t0 = time.perf_counter()
            rc, c, _ = e.polygonize_mpus(cs, model, out)
            dt = (time.perf_counter() - t0) * 1e3
            assert rc == 1 and c == ct, (rc, c, ct)
            print(f"call {cfg} {k} {rep} {dt:.3f}", file=sys.stderr, flush=True)
            if rep >= 2:
                t[k].append(dt)
    for k, v in t.items():
        print(cfg, k, "median %.3f p90 %.3f best %.3f" % (np.median(v), np.percentile(v, 90), min(v)),
              " ".join("%.3f" % x for x in v), flush=True)

"""Device timeline of the driver's timed window (bench.py --steps 20 --warmup 5): 4 engines take
the 20 steps in turn, queued without host sync; every run records its four kernels' spans on the
device clock (PSGPU_OPT_SPANS: first wave start, last wave end).  Prints the host window (t0 ->
every engine finished), the device window (first kernel start -> last kernel end), and per
engine and step where each kernel ran, so the fill (the first round, all engines in the same
kernel) and the drain (the last steps with fewer engines in flight) can be read off.

Usage (GPU): python tools/window_timeline.py [--steps 20] [--warmup 5] [--engines 4] [--reps 3]
"""
import argparse
import os
import sys
import time

# at least 8 hardware queues, before HIP starts, as bench.py (the box exports 4: with 4, one
# engine's stream shares the null stream's queue and the engines serialise)
os.environ["GPU_MAX_HW_QUEUES"] = str(max(int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4), 8))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

from parsip_amd import gpu, synth  # noqa: E402

TICK_US = 0.01


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--engines", type=int, default=4)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--config", default="C3")
    ap.add_argument("--stagger-us", type=float, default=0.0, help="the first round's engines start this far apart")
    a = ap.parse_args()
    model, cs, N = synth.make_config(a.config)
    E = a.engines
    eng = [gpu.Polygonizer(0) for _ in range(E)]
    for e in eng:
        e.set_option(gpu.OPT_JIT, gpu.JIT_STRUCTURE)
        if E > 1:  # bench.py's grids with several engines
            e.set_option(gpu.OPT_VERTEX_BLOCKS_PER_CU, 8)
            e.set_option(gpu.OPT_FINISH_BLOCKS_PER_CU, 4)
        e.set_model(model)
    per = (a.steps + E - 1) // E
    for rep in range(a.reps):
        for k in range(max(a.warmup, E)):
            eng[k % E].polygonize(cs)
        for e in eng:
            e.finish()
        for e in eng:
            e.set_option(gpu.OPT_SPANS, per)
        t0 = time.perf_counter()
        for k in range(a.steps):
            eng[k % E].polygonize(cs)
            if k < E - 1 and a.stagger_us > 0:
                ts = time.perf_counter() + a.stagger_us * 1e-6
                while time.perf_counter() < ts:
                    pass
        t_enq = time.perf_counter()
        for e in eng:
            e.finish()
        t1 = time.perf_counter()
        sp = [e.spans(raw=True) for e in eng]  # (runs, kernels, 2) ticks
        lo = min(int(s[:, :, 0].min()) for s in sp if len(s))
        hi = max(int(s[:, :, 1].max()) for s in sp if len(s))
        print(f"rep {rep}: host window {(t1 - t0) * 1e3:.4f} ms ({(t1 - t0) * 1e3 / a.steps:.4f} ms/step), enqueue "
              f"{(t_enq - t0) * 1e3:.4f} ms; device window {(hi - lo) * TICK_US / 1e3:.4f} ms "
              f"({(hi - lo) * TICK_US / 1e3 / a.steps:.4f} ms/step)")
        ends = []
        for ei, s in enumerate(sp):
            for r in range(len(s)):
                st = (s[r, :, 0] - lo) * TICK_US
                en = (s[r, :, 1] - lo) * TICK_US
                ends.append(en[-1])
                if rep == a.reps - 1 and a.steps <= 40:
                    print(f"  engine {ei} step {r * E + ei:2d}: " +
                          " | ".join(f"{k[2:]} {st[i]:7.1f}-{en[i]:7.1f}" for i, k in enumerate(gpu.STAMP_KERNELS)))
        # round k = steps [kE, (k+1)E): from engine 0's step start to the next round's
        starts0 = (sp[0][:, 0, 0] - lo) * TICK_US
        rounds = np.diff(starts0)
        print(f"  rounds (engine 0 step to step, us): {' '.join(f'{x:.0f}' for x in rounds[:12])}"
              f"{' ...' if len(rounds) > 12 else ''} {' '.join(f'{x:.0f}' for x in rounds[-6:]) if len(rounds) > 12 else ''}")
        ends = np.sort(np.array(ends))
        gaps = np.diff(ends)
        print(f"  step completions (us): first {ends[0]:.1f}, then every {np.median(gaps):.1f} (median), last {ends[-1]:.1f}")
        for e in eng:
            e.set_option(gpu.OPT_SPANS, 0)
    for e in eng:
        e.close()


if __name__ == "__main__":
    main()

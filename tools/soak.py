"""Soak run of the pipelined engines: 4 contexts take C3 polygonizations in turn for a fixed
time, each run collected (psgpu_finish) while the other three are in flight, so every run's
counters are checked -- a run that hit a protocol error in one of the in-kernel waits (k_front's
hand-off, k_surface's scan) or a capacity overflow is re-run by finish and counted here -- and
every 256th collected mesh is compared with the oracle (the committed C3 digests for the full
grid, a live oracle run for a share).  Phases: the full grid (k_front on, separate k_vertex /
k_finish) and the slowest 1/8 cost share with the small-launch kernels (tree split 2: k_front +
k_surface), the regime of the strong-scaling ranks.  Exit status 1 on any differing mesh.

Usage (GPU): python tools/soak.py [--seconds 60]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=60.0)
    ap.add_argument("--engines", type=int, default=4)
    ap.add_argument("--check-every", type=int, default=256)
    a = ap.parse_args()
    import numpy as np
    import psoracle
    from parity_util import assert_mesh_matches, mesh_digests

    from parsip_amd import gpu, synth

    psoracle.build()
    model, cs, _ = synth.make_config("C3")
    golden = json.load(open(os.path.join(ROOT, "tests", "golden", "oracle_digests.json")))["C3"]
    probe = gpu.Polygonizer(0)
    probe.set_model(model)
    b = probe.plan_split(cs, 8)
    probe.close()
    shares = [(int(b[i]), int(b[i + 1])) for i in range(8)]
    fails = 0
    for phase, rng, split in (("full grid", (0, None), 0), ("slowest 1/8 share", None, 2)):
        lo, hi = rng if rng else (None, None)
        ps = [gpu.Polygonizer(0) for _ in range(a.engines)]
        for p in ps:
            p.set_option(gpu.OPT_TREE_SPLIT, split)
            p.set_model(model)
        if lo is None:  # the share whose isolated run is slowest
            t = []
            for s in shares:
                ps[0].run(cs, *s)
                t0 = time.perf_counter()
                for _ in range(20):
                    ps[0].run(cs, *s)
                t.append(time.perf_counter() - t0)
            lo, hi = shares[int(np.argmax(t))]
            om = psoracle.polygonize(model, cs, lo, hi, threads=16)

            def check(p):
                assert_mesh_matches(p.download(), p.stats(), om)
        else:
            def check(p):
                gm, gs = p.download(), p.stats()
                st = np.stack([gs["passedPrecheck"], gs["ctFieldEvals"], gs["ctVertices"], gs["ctTriangles"]], axis=1)
                assert mesh_digests(st, gm.pos, gm.nrm, gm.col, gm.local_tris()) == golden
        for p in ps:
            p.run(cs, lo, hi)  # sizes the buffers
        runs = reruns = front = surface = checks = 0
        pending = [False] * len(ps)
        t0 = time.perf_counter()
        k = 0
        while True:
            i = k % len(ps)
            p = ps[i]
            if pending[i]:
                info = p.finish()
                runs += 1
                reruns += bool(info.launchFlags & gpu.LAUNCH_RERUN)
                front += bool(info.launchFlags & gpu.LAUNCH_FRONT)
                surface += bool(info.launchFlags & gpu.LAUNCH_SURFACE)
                if runs % a.check_every == 0:
                    checks += 1
                    try:
                        check(p)
                    except AssertionError as e:
                        fails += 1
                        print(f"{phase}: run {runs}: {str(e).splitlines()[0][:300]}", flush=True)
                if runs % 100000 == 0:
                    print(f"... {phase}: {runs} runs, {reruns} re-run, {time.perf_counter() - t0:.0f} s", flush=True)
                if time.perf_counter() - t0 > a.seconds:
                    break
            p.polygonize(cs, lo, hi)
            pending[i] = True
            k += 1
        for j, p in enumerate(ps):
            if pending[j]:
                p.finish()
            p.close()
        dt = time.perf_counter() - t0
        print(f"{phase} (MPUs [{lo}, {hi if hi is not None else 'end'})), {len(ps)} engines: {runs} runs collected in "
              f"{dt:.0f} s ({1e3 * dt / max(runs, 1):.4f} ms per run with a finish each), {reruns} re-run by finish, "
              f"k_front {front}, k_surface {surface}, {checks} meshes checked, {fails} differ so far", flush=True)
    sys.exit(1 if fails else 0)


if __name__ == "__main__":
    main()

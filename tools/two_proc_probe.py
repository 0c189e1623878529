"""Does the device take more C3 steps per second with more chains in flight than four engines
give one process?  More engines in one process are slower (profiles/r05_engines_sweep.txt), so
this runs P processes, each with E engines, on the same GPU at once: they start their timed
loops together (a file barrier) and the combined rate is all their steps over the common
window.  A probe, not a bench: the bench contract is one process per GPU.

Usage (GPU): python tools/two_proc_probe.py [--procs 2] [--engines 4] [--steps 2000]
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(a):
    os.environ["GPU_MAX_HW_QUEUES"] = str(max(int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4), 8))
    sys.path.insert(0, ROOT)
    from parsip_amd import gpu, synth

    model, cs, N = synth.make_config("C3")
    E = a.engines
    eng = [gpu.Polygonizer(0) for _ in range(E)]
    for e in eng:
        e.set_option(gpu.OPT_JIT, gpu.JIT_STRUCTURE)
        if E > 1:
            e.set_option(gpu.OPT_VERTEX_BLOCKS_PER_CU, 8)
            e.set_option(gpu.OPT_FINISH_BLOCKS_PER_CU, 4)
        e.set_model(model)
    for k in range(max(20, E)):
        eng[k % E].polygonize(cs)
    for e in eng:
        e.finish()
    open(os.path.join(a.dir, f"ready{a.rank}"), "w").close()
    deadline = time.time() + 120
    while sum(os.path.exists(os.path.join(a.dir, f"ready{r}")) for r in range(a.procs)) < a.procs:
        if time.time() > deadline:
            sys.exit("barrier timeout")
        time.sleep(0.0005)
    t0 = time.time()
    for k in range(a.steps):
        eng[k % E].polygonize(cs)
    for e in eng:
        e.finish()
    t1 = time.time()
    print(json.dumps({"rank": a.rank, "t0": t0, "t1": t1, "steps": a.steps, "ms_per_step": (t1 - t0) * 1e3 / a.steps}))
    for e in eng:
        e.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, default=2)
    ap.add_argument("--engines", type=int, default=4)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--rank", type=int, default=-1)
    ap.add_argument("--dir", default=None)
    a = ap.parse_args()
    if a.rank >= 0:
        child(a)
        return
    with tempfile.TemporaryDirectory() as d:
        ps = [subprocess.Popen([sys.executable, __file__, "--procs", str(a.procs), "--engines", str(a.engines),
                                "--steps", str(a.steps), "--rank", str(r), "--dir", d], stdout=subprocess.PIPE, text=True)
              for r in range(a.procs)]
        try:
            outs = [p.communicate(timeout=300)[0] for p in ps]
        except subprocess.TimeoutExpired:
            for p in ps:  # never leave a child behind on the GPU
                p.kill()
                p.wait()
            sys.exit("a child did not finish within 300 s")
    if any(p.returncode for p in ps):
        sys.exit(f"a child failed: {[p.returncode for p in ps]}")
    res = [json.loads(o.strip().splitlines()[-1]) for o in outs]
    t0 = min(r["t0"] for r in res)
    t1 = max(r["t1"] for r in res)
    total = sum(r["steps"] for r in res)
    per = " ".join("%.4f" % r["ms_per_step"] for r in res)
    print(f"procs {a.procs} x engines {a.engines}: per process {per} ms/step; "
          f"start skew {(max(r['t0'] for r in res) - t0) * 1e3:.2f} ms; combined {(t1 - t0) * 1e3 / total:.4f} ms/step "
          f"over {(t1 - t0) * 1e3:.1f} ms")


if __name__ == "__main__":
    main()

"""Where the driver's short window loses time against the steady state, without instrumenting
the kernels: the bench's timed loop (4 engines taking K steps in turn, queued without host
sync, bracketed by host syncs) for each K of --ks, run under `rocprofv3 --kernel-trace`, whose
per-dispatch start / end timestamps are then read by --parse.  Windows are separated by 30 ms
of idle host time so that --parse can find them; each window's dispatches are the last 4 K
before its gap (the warmup steps run right before, as in bench.py).

Run (GPU):   rocprofv3 --kernel-trace --output-format csv -d OUT -o run -- python3 tools/window_trace.py --ks 20,40,200
Parse (CPU): python3 tools/window_trace.py --parse OUT/.../run_kernel_trace.csv --ks 20,40,200
"""
import argparse
import csv
import glob
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = ("jit_precheck", "jit_mpu", "jit_vertex", "jit_finish")


def run(a):
    # at least 8 hardware queues before HIP starts, as bench.py
    os.environ["GPU_MAX_HW_QUEUES"] = str(max(int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4), 8))
    sys.path.insert(0, ROOT)
    from parsip_amd import gpu, synth

    model, cs, N = synth.make_config(a.config)
    E = a.engines
    eng = [gpu.Polygonizer(0) for _ in range(E)]
    for i, e in enumerate(eng):
        e.set_option(gpu.OPT_JIT, gpu.JIT_STRUCTURE)
        if E > 1:  # bench.py's grids with several engines
            e.set_option(gpu.OPT_VERTEX_BLOCKS_PER_CU, 8)
            e.set_option(gpu.OPT_FINISH_BLOCKS_PER_CU, 4)
        if a.mix and i % 2 == 1:  # every second engine on other layouts: chains of other lengths
            e.set_option(gpu.OPT_FINISH_QUAD, a.mix_fquad)
            e.set_option(gpu.OPT_VERTEX_WIDE, a.mix_vwide)
        e.set_model(model)
    for rep in range(a.reps):
        for K, W in [(int(x), int(w)) for x in a.ks.split(",") for w in a.warmups.split(",")]:
            for k in range(max(W, E)):
                eng[k % E].polygonize(cs)
            for e in eng:
                e.finish()
            t0 = time.perf_counter()
            for k in range(K):
                eng[k % E].polygonize(cs)
            t_enq = time.perf_counter()
            for e in eng:
                e.finish()
            t1 = time.perf_counter()
            print(f"rep {rep} K {K} W {W}: host window {(t1 - t0) * 1e3:.4f} ms ({(t1 - t0) * 1e3 / K:.4f} ms/step), "
                  f"enqueue {(t_enq - t0) * 1e3:.4f} ms", flush=True)
            time.sleep(0.03)
    for e in eng:
        e.close()


def parse(a):
    path = a.parse
    if os.path.isdir(path):
        path = sorted(glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True))[0]
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"]
            k = next((i for i, n in enumerate(KERNELS) if name.startswith(n)), None)
            if k is None:
                continue
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k, int(r["Queue_Id"]), name))
    rows.sort()
    # windows: split where the host idled (a gap of > 5 ms between dispatches)
    groups, cur = [], [rows[0]]
    for r in rows[1:]:
        if r[0] - max(x[1] for x in cur[-8:]) > 5_000_000:
            groups.append(cur)
            cur = []
        cur.append(r)
    groups.append(cur)
    ks = [int(x) for x in a.ks.split(",") for _ in a.warmups.split(",")] * a.reps
    if len(groups) != len(ks):
        print(f"{len(groups)} dispatch groups for {len(ks)} windows: cannot match", file=sys.stderr)
    E = a.engines
    for K, g in zip(ks, groups):
        w = g[-4 * K:]
        lo = min(r[0] for r in w)
        hi = max(r[1] for r in w)
        # steps: every 4 consecutive dispatches of one queue, in order
        byq = {}
        for r in w:
            byq.setdefault(r[3], []).append(r)
        steps = []
        for q, rs in byq.items():
            rs.sort()
            for i in range(0, len(rs) - 3, 4):
                steps.append((rs[i][0], rs[i + 3][1], q, [(x[0], x[1]) for x in rs[i:i + 4]]))
        steps.sort()
        lat = [(s[1] - s[0]) / 1e3 for s in steps]
        ends = sorted(s[1] for s in steps)
        print(f"K {K}: device window {(hi - lo) / 1e6:.4f} ms ({(hi - lo) / 1e6 / K:.4f} ms/step) over {len(byq)} queues; "
              f"first step done at {(ends[0] - lo) / 1e3:.1f} us; chain latency p50 {sorted(lat)[len(lat) // 2]:.1f} us, "
              f"first round {' '.join(f'{x:.0f}' for x in lat[:E])}, last round {' '.join(f'{x:.0f}' for x in lat[-E:])}")
        # concurrency: how many engines have a kernel running, over the window
        ev = []
        for r in w:
            ev.append((r[0], 1))
            ev.append((r[1], -1))
        ev.sort()
        busy = {}
        n, t_prev = 0, lo
        for t, d in ev:
            busy[n] = busy.get(n, 0) + (t - t_prev)
            n += d
            t_prev = t
        tot = sum(busy.values())
        print("   kernels in flight (share of the window): " +
              " ".join(f"{k}:{v / tot:.2f}" for k, v in sorted(busy.items())))
        if a.verbose and K <= 40:
            for s in steps:
                print(f"   q{s[2]:3d} " + " | ".join(f"{KERNELS[i][4:]} {(x[0] - lo) / 1e3:7.1f}-{(x[1] - lo) / 1e3:7.1f}"
                                                  for i, x in enumerate(s[3])))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ks", default="20,40,200")
    ap.add_argument("--warmups", default="5", help="warmup steps before each window (a list: every K with every W)")
    ap.add_argument("--engines", type=int, default=4)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--config", default="C3")
    ap.add_argument("--parse", default=None, help="a rocprofv3 kernel_trace.csv (or a directory holding one)")
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--mix", action="store_true", help="odd engines take --mix-fquad / --mix-vwide layouts")
    ap.add_argument("--mix-fquad", type=int, default=3)
    ap.add_argument("--mix-vwide", type=int, default=0)
    a = ap.parse_args()
    if a.parse:
        parse(a)
    else:
        run(a)


if __name__ == "__main__":
    main()

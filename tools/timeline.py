"""Per-wave timeline of one polygonization (PSGPU_OPT_STAMPS, s_memrealtime at 100 MHz).

usage: python tools/timeline.py [--config C3] [--jit 1] [--json out.json]
Prints, per kernel: waves, span (first start -> last end), the gap after the previous
kernel, wave lifetime percentiles, the share of the span during which fewer than 1/4 of
the peak number of waves were running (the tail), and a 20-bin profile of running waves.
For k_mpu, waves that polygonized an MPU and empty waves are reported apart.
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from parsip_amd import gpu, synth  # noqa: E402

TICK_US = 0.01  # 100 MHz


def profile(st, t0, t1, bins=20):
    edges = np.linspace(t0, t1, bins + 1)
    mids = 0.5 * (edges[:-1] + edges[1:])
    return [int(np.count_nonzero((st[:, 0] <= m) & (st[:, 1] >= m))) for m in mids]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--jit", type=int, default=1)
    ap.add_argument("--runs", type=int, default=5)
    ap.add_argument("--json")
    ap.add_argument("--share", type=int, default=1, help="time the first 1/SHARE of the cost split (a rank's range)")
    ap.add_argument("--debug", type=int, default=0, help="PSGPU_OPT_DEBUG ablation bits")
    a = ap.parse_args()
    model, cs, N = synth.make_config(a.config)
    p = gpu.Polygonizer(0)
    p.set_option(gpu.OPT_JIT, a.jit)
    if a.debug:
        p.set_option(gpu.OPT_DEBUG, a.debug)
    p.set_model(model)
    lo, hi = 0, None
    if a.share > 1:
        b = p.plan_split(cs, a.share)
        lo, hi = int(b[0]), int(b[1])
    for _ in range(3):
        p.run(cs, lo, hi)
    p.set_option(gpu.OPT_STAMPS, 1 << 17)
    report = {}
    for run in range(a.runs):
        p.run(cs, lo, hi)
        S = p.stamps()
    prev_end = None
    first = min(int(S[k][:, 0].min()) for k in gpu.STAMP_KERNELS if len(S[k]))
    for k in gpu.STAMP_KERNELS:
        st = S[k].astype(np.int64)
        if not len(st):
            continue
        t0, t1 = int(st[:, 0].min()), int(st[:, 1].max())
        life = (st[:, 1] - st[:, 0]) * TICK_US
        prof = profile(st, t0, t1)
        peak = max(prof)
        tail = sum(1 for x in prof if x < peak / 4) / len(prof)
        e = {"waves": int(len(st)), "start_us": round((t0 - first) * TICK_US, 2), "span_us": round((t1 - t0) * TICK_US, 2),
             "gap_before_us": None if prev_end is None else round((t0 - prev_end) * TICK_US, 2),
             "life_us_p50": round(float(np.percentile(life, 50)), 2),
             "life_us_p90": round(float(np.percentile(life, 90)), 2), "life_us_max": round(float(life.max()), 2),
             "last_start_us": round((int(st[:, 0].max()) - t0) * TICK_US, 2),
             "tail_share": round(tail, 2), "running_waves_20bins": prof}
        if k == "k_mpu":
            item = (st[:, 2] & 0xFFFFFFFF).astype(np.int64)
            real = item != 0xFFFFFFFF
            e["real_waves"] = int(real.sum())
            e["real_life_us_p50"] = round(float(np.percentile(life[real], 50)), 2) if real.any() else None
            e["real_life_us_max"] = round(float(life[real].max()), 2) if real.any() else None
            e["empty_life_us_p50"] = round(float(np.percentile(life[~real], 50)), 2) if (~real).any() else None
        report[k] = e
        prev_end = t1
        print(f"{k:10s} waves={e['waves']:6d} start={e['start_us']:7.2f} span={e['span_us']:6.2f}us "
              f"gap={e['gap_before_us']} life p50/p90/max={e['life_us_p50']}/{e['life_us_p90']}/{e['life_us_max']} "
              f"last_start={e['last_start_us']} tail={e['tail_share']}")
        print(f"{'':10s} running: {prof}")
        if k == "k_mpu":
            print(f"{'':10s} real waves={e['real_waves']} life p50/max={e['real_life_us_p50']}/{e['real_life_us_max']} "
                  f"empty p50={e['empty_life_us_p50']}")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(report, f, indent=1)




def _share_range(p, cs, share):
    if share <= 1:
        return 0, None
    b = p.plan_split(cs, share)
    return int(b[0]), int(b[1])


def mpu_phases(config="C3", share=1):
    """k_mpu phase stamps (debug bit 4096): per real wave, the time spent between entry,
    table staging, MPU fetch + cull mask, S2 walk, the inside-bit barrier, pass 1 (+barrier),
    pass 2 (+barrier) and the end (the k_mpu record's end stamp)."""
    model, cs, N = synth.make_config(config)
    p = gpu.Polygonizer(0)
    p.set_model(model)
    lo, hi = _share_range(p, cs, share)
    for _ in range(3):
        p.run(cs, lo, hi)
    p.set_option(gpu.OPT_STAMPS, 1 << 17)
    p.set_option(gpu.OPT_DEBUG, 4096)
    p.run(cs, lo, hi)
    S = p.stamps()
    ph = S["mpu_phases"].astype(np.int64)
    rec = S["k_mpu"].astype(np.int64)
    n = len(rec)
    ph = ph[:n]
    item = (rec[:, 2] & 0xFFFFFFFF)
    real = (item != 0xFFFFFFFF) & (ph[:, 3] != 0)
    t0 = rec[:, 0].min()
    names = ["stage tables", "fetch+cullmask", "S2 walk", "ins barrier", "pass 1", "pass 2", "pass 3+end"]
    cols = [ph[:, 0], ph[:, 1], ph[:, 2], ph[:, 3], ph[:, 4], ph[:, 5], ph[:, 6], rec[:, 1]]
    print(f"k_mpu real waves {int(real.sum())} of {n}")
    for i, nm in enumerate(names):
        a, b = cols[i][real], cols[i + 1][real]
        ok = (a > 0) & (b > 0)
        dt = (b[ok] - a[ok]) * TICK_US
        if len(dt):
            print(f"  {nm:15s} median {np.median(dt):6.2f} us  p90 {np.percentile(dt, 90):6.2f}  max {dt.max():6.2f}")
    st = (ph[real, 0] - t0) * TICK_US
    print(f"  wave entry time: median {np.median(st):.2f} us, p90 {np.percentile(st, 90):.2f}, max {st.max():.2f}")
    w7 = ph[:, 7]
    if (w7[real] != 0).any():  # built with -DPSGPU_MPU_LIVE_STAMP=1: live primitives, V, T per wave
        live = (w7 & 0xFFFF) - (128 - model.ct_prims)
        V = (w7 >> 16) & 0xFFFF
        T = (w7 >> 32) & 0xFFFF
        s2 = (ph[:, 3] - ph[:, 2]) * TICK_US
        life = (rec[:, 1] - rec[:, 0]) * TICK_US
        _live_table("k_mpu", live, real, {"S2 walk": s2, "life": life}, {"V": V, "T": T})


def _live_table(kernel, live, real, times, counts):
    """Per bucket of live primitives: waves, the summed counts (vertices / triangles), the
    p50 / max of each phase -- how much of the work sits in the heavy waves that set the span."""
    print(f"  {kernel} by live primitives:")
    tot = {k: max(1, int(v[real].sum())) for k, v in counts.items()}
    for lo, hi in ((0, 4), (4, 8), (8, 12), (12, 16), (16, 20), (20, 24), (24, 28), (28, 33)):
        sel = real & (live >= lo) & (live < hi)
        if not sel.any():
            continue
        line = f"    [{lo:2d},{hi:2d}): waves {int(sel.sum()):5d}"
        for k, v in counts.items():
            line += f"  {k} {int(v[sel].sum()):7d} ({100 * v[sel].sum() / tot[k]:4.1f} %)"
        for k, v in times.items():
            line += f"  {k} p50 {np.median(v[sel]):5.2f} max {v[sel].max():5.2f}"
        print(line)


def precheck_phases(config="C3", share=1):
    """k_precheck phase stamps (debug bit 8192): per wave, entry -> S1 walk done, -> field
    bounds done (waves holding a survivor), -> queue append, -> end (culling masks)."""
    model, cs, N = synth.make_config(config)
    p = gpu.Polygonizer(0)
    p.set_model(model)
    lo, hi = _share_range(p, cs, share)
    for _ in range(3):
        p.run(cs, lo, hi)
    p.set_option(gpu.OPT_STAMPS, 1 << 17)
    p.set_option(gpu.OPT_DEBUG, 8192)
    p.run(cs, lo, hi)
    S = p.stamps()
    rec = S["k_precheck"].astype(np.int64)
    n = len(rec)
    ph = S["mpu_phases"].astype(np.int64)[:n]
    t0 = rec[:, 0].min()
    life = (rec[:, 1] - rec[:, 0]) * TICK_US
    heavy = ph[:, 2] != 0
    print(f"k_precheck waves {n}, with survivors (bounded) {int(heavy.sum())}")
    for nm, sel in (("all", np.ones(n, bool)), ("bounded", heavy), ("no survivor", ~heavy)):
        if not sel.any():
            continue
        s1 = (ph[sel, 1] - ph[sel, 0]) * TICK_US
        print(f"  {nm:12s} life p50 {np.median(life[sel]):6.2f} p90 {np.percentile(life[sel], 90):6.2f} "
              f"max {life[sel].max():6.2f} | S1 walk p50 {np.median(s1):6.2f} max {s1.max():6.2f}")
    if heavy.any():
        b = (ph[heavy, 2] - ph[heavy, 1]) * TICK_US
        q = (ph[heavy, 3] - ph[heavy, 2]) * TICK_US
        e = (rec[heavy, 1] - ph[heavy, 3]) * TICK_US
        print(f"  bounded: bound p50 {np.median(b):.2f} max {b.max():.2f} | queue p50 {np.median(q):.2f} "
              f"max {q.max():.2f} | masks p50 {np.median(e):.2f} max {e.max():.2f}")
        live = ph[:, 7] & 0xFFFF
        live = live - (128 - model.ct_prims)  # primitives of the tree not culled for the wave
        s1 = (ph[:, 1] - ph[:, 0]) * TICK_US
        for lo, hi in ((0, 1), (1, 4), (4, 8), (8, 16), (16, 24), (24, 33)):
            sel = (live >= lo) & (live < hi)
            if sel.any():
                print(f"  live prims [{lo},{hi}): waves {int(sel.sum()):5d}  S1 walk p50 {np.median(s1[sel]):6.2f} "
                      f"max {s1[sel].max():6.2f}  life p50 {np.median(life[sel]):6.2f} max {life[sel].max():6.2f}")
        worst = np.argsort(life)[-10:]
        for w in worst:
            print(f"  worst wave {w} (live prims {int(live[w])}): start {(rec[w, 0] - t0) * TICK_US:.2f} life {life[w]:.2f} | "
                  + " ".join(f"{(ph[w, i + 1] - ph[w, i]) * TICK_US:.2f}" if ph[w, i + 1] else "-" for i in range(3))
                  + f" | end {(rec[w, 1] - ph[w, 3]) * TICK_US if ph[w, 3] else -1:.2f}")


def finish_phases(config="C3", share=1):
    """k_finish phase stamps of the 64-vertex layout (debug bit 2048; the kernels must be
    compiled with PSGPU_JIT_FLAGS=-DPSGPU_FIN_PHASES=1): per wave with a batch, entry ->
    counts staged (block barrier) -> records loaded and root recomputed -> culling mask ->
    the 4-point colour walk -> vertex stores issued -> triangle pass -> the record's end."""
    model, cs, N = synth.make_config(config)
    p = gpu.Polygonizer(0)
    p.set_option(gpu.OPT_FINISH_QUAD, 0)
    p.set_model(model)
    lo, hi = _share_range(p, cs, share)
    for _ in range(3):
        p.run(cs, lo, hi)
    p.set_option(gpu.OPT_STAMPS, 1 << 16)
    p.set_option(gpu.OPT_DEBUG, 2048)
    p.run(cs, lo, hi)
    S = p.stamps()
    rec = S["k_finish"].astype(np.int64)
    n = len(rec)
    ph = S["mpu_phases"].astype(np.int64)[:n]
    real = ph[:, 4] != 0
    t0 = rec[:, 0].min()
    print(f"k_finish waves {n}, with a vertex batch {int(real.sum())}; span "
          f"{(rec[:, 1].max() - t0) * TICK_US:.2f} us")
    names = ["entry->staged", "staged->root", "root->cullmask", "walk", "stores", "triangles", "->end"]
    cols = [ph[:, 0], ph[:, 1], ph[:, 2], ph[:, 3], ph[:, 4], ph[:, 5], ph[:, 6], rec[:, 1]]
    for i, nm in enumerate(names):
        a, b = cols[i][real], cols[i + 1][real]
        ok = (a > 0) & (b > 0)
        dt = (b[ok] - a[ok]) * TICK_US
        if len(dt):
            print(f"  {nm:15s} median {np.median(dt):6.2f} us  p90 {np.percentile(dt, 90):6.2f}  max {dt.max():6.2f}")
    life = (rec[real, 1] - rec[real, 0]) * TICK_US
    st = (rec[real, 0] - t0) * TICK_US
    print(f"  life median {np.median(life):.2f} p90 {np.percentile(life, 90):.2f} max {life.max():.2f}; "
          f"start median {np.median(st):.2f} max {st.max():.2f}")
    w7 = ph[:, 7]
    if (w7[real] != 0).any():  # live primitives and vertices per wave (PSGPU_FIN_PHASES builds)
        live = (w7 & 0xFFFF) - (128 - model.ct_prims)
        nv = (w7 >> 16) & 0xFFFF
        walk = (ph[:, 4] - ph[:, 3]) * TICK_US
        lifeall = (rec[:, 1] - rec[:, 0]) * TICK_US
        _live_table("k_finish", live, real, {"walk": walk, "life": lifeall}, {"vertices": nv})
    # the waves that end last: what they spent their time on
    worst = np.argsort(rec[:, 1])[-8:]
    for w in worst:
        if not real[w]:
            continue
        seg = [(cols[i + 1][w] - cols[i][w]) * TICK_US for i in range(len(names))]
        print(f"  late wave {w}: start {(rec[w, 0] - t0) * TICK_US:.2f} end {(rec[w, 1] - t0) * TICK_US:.2f} | "
              + " ".join(f"{x:.2f}" for x in seg))


if __name__ == "__main__":
    if "--finish" in sys.argv:
        finish_phases(share=int(os.environ.get("SHARE", "1")))
        sys.exit(0)
    share = int(os.environ.get("SHARE", "1"))
    if "--precheck" in sys.argv:
        sys.argv.remove("--precheck")
        precheck_phases(share=share)
        sys.exit(0)
    if "--phases" in sys.argv:
        mpu_phases(share=share)
    else:
        main()

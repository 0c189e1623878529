"""Per-wave timeline of several engines (device contexts) taking C3 steps in turn, as bench.py's
throughput regime runs them: the last run of every engine overlaps the others', and every wave
of every kernel records its start, end and hardware slot (PSGPU_OPT_STAMPS).

Reports, per kernel, the summed wave lifetimes (SIMD-time held), the span of each engine's
launch, the delay between an engine's previous kernel ending and this kernel's first wave
starting (waiting for slots other engines hold), and a per-SIMD occupancy census: how much of
the window each SIMD held 0, 1, ... waves and of which kernels.  With one engine it is the
isolated timeline of one polygonization.

Usage (GPU): python tools/engines_timeline.py [--engines 4] [--config C3] [--json out.json]
(--engines 1: one context, its last run alone.)
The environment selects kernel variants (e.g. PSGPU_JIT_FLAGS=-DPSGPU_S2_GROUP=5).
"""
import argparse
import ctypes
import json
import os
import sys

# at least 8 hardware queues, before HIP starts, as bench.py (the box exports 4: with 4, one
# engine's stream shares the null stream's queue and the engines serialise)
os.environ["GPU_MAX_HW_QUEUES"] = str(max(int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4), 8))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

from parsip_amd import gpu, synth  # noqa: E402

TICK_US = 0.01  # s_memrealtime, 100 MHz


def simd_key(hw):
    """XCC, SE, SH, CU, SIMD of a wave from its recorded XCC_ID << 16 | HW_ID[15:0] (HW_ID:
    wave 3:0, SIMD 5:4, pipe 7:6 -- the queue's, not a place --, CU 11:8, SH 12, SE 15:13)."""
    return (hw >> 16) << 10 | ((hw >> 8) & 0xff) << 2 | ((hw >> 4) & 3)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--engines", type=int, default=4)
    ap.add_argument("--config", default="C3")
    ap.add_argument("--warmup", type=int, default=40)
    ap.add_argument("--steps", type=int, default=40, help="queued steps before the recorded ones")
    ap.add_argument("--json")
    ap.add_argument("--share", type=int, default=1, help="time rank --rank's range of a cost split in SHARE parts")
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--tree-split", type=int, default=0, help="PSGPU_OPT_TREE_SPLIT (bench.py: 2 for N > 1 ranks)")
    a = ap.parse_args()
    model, cs, N = synth.make_config(a.config)
    # Three sets of E contexts with stamps on (a context's stamps hold its last run): set A takes
    # the steps in turn, then set T one round, then set B one round, context k of every set on
    # engine stream k, so each stream is one serial chain as an engine's is in the timed loop;
    # T's runs are the steady state's, overlapped by A's last round before them and B's round
    # after them, and every wave around T's window is recorded.
    E = a.engines
    sets = [[gpu.Polygonizer(0) for _ in range(E)] for _ in range(3 if E > 1 else 1)]
    allc = [c for st in sets for c in st]
    hip = ctypes.CDLL("libamdhip64.so")
    streams = []
    for _ in range(E):
        h = ctypes.c_void_p()
        assert hip.hipStreamCreateWithFlags(ctypes.byref(h), 1) == 0  # hipStreamNonBlocking
        streams.append(h.value)
    stream_of = {id(c): streams[i % E] for st in sets for i, c in enumerate(st)}
    for e in allc:
        e.set_option(gpu.OPT_JIT, gpu.JIT_STRUCTURE)
        e.set_option(gpu.OPT_TREE_SPLIT, a.tree_split)
        if E > 1:  # bench.py's grids with several engines
            e.set_option(gpu.OPT_VERTEX_BLOCKS_PER_CU, 8)
            e.set_option(gpu.OPT_FINISH_BLOCKS_PER_CU, 4)
        e.set_model(model)
        e.set_option(gpu.OPT_STAMPS, 1 << 15)
    lo, hi = 0, None
    if a.share > 1:
        b = allc[0].plan_split(cs, a.share)
        lo, hi = int(b[a.rank]), int(b[a.rank + 1])
    for k in range(a.warmup):
        c = allc[k % len(allc)]
        c.polygonize(cs, lo, hi, stream=stream_of[id(c)])
    for e in allc:
        e.finish()
    seq = [sets[0][k % E] for k in range(a.steps)] + (sets[1] + sets[2] if E > 1 else [])
    for e in seq:
        e.polygonize(cs, lo, hi, stream=stream_of[id(e)])
    for e in allc:
        e.finish()
    runs = [e.stamps() for st in sets for e in st]
    tset = sets[1] if E > 1 else sets[0]
    focus = [i for i, e in enumerate(c for st in sets for c in st) if e in tset]
    t_first = min(int(runs[i][k][:, 0].min()) for i in focus for k in gpu.STAMP_KERNELS if len(runs[i][k]))
    t_last = max(int(runs[i][k][:, 1].max()) for i in focus for k in gpu.STAMP_KERNELS if len(runs[i][k]))
    out = {"engines": a.engines, "config": a.config, "share": [a.share, a.rank, lo, hi], "env": {k: v for k, v in os.environ.items() if k.startswith("PSGPU")},
           "window_us": round((t_last - t_first) * TICK_US, 2), "kernels": {}}
    # all waves: (kernel index, engine, start, end, simd)
    rows = []
    for ei, r in enumerate(runs):
        prev_end = None
        for ki, k in enumerate(gpu.STAMP_KERNELS):
            st = r[k].astype(np.int64)
            if not len(st):
                continue
            hw = (st[:, 2] >> 32).astype(np.int64)
            for s, e_, h in zip(st[:, 0], st[:, 1], hw):
                rows.append((ki, ei, int(s), int(e_), int(simd_key(h))))
            if ei not in focus:
                continue
            d = out["kernels"].setdefault(k, {"wave_us_sum": 0.0, "waves": 0, "span_us": [], "start_delay_us": [],
                                             "life_us_p50": [], "life_us_max": []})
            life = (st[:, 1] - st[:, 0]) * TICK_US
            d["wave_us_sum"] += float(life.sum())
            d["waves"] += int(len(st))
            d["span_us"].append(round((int(st[:, 1].max()) - int(st[:, 0].min())) * TICK_US, 2))
            d["start_delay_us"].append(None if prev_end is None else round((int(st[:, 0].min()) - prev_end) * TICK_US, 2))
            d["life_us_p50"].append(round(float(np.percentile(life, 50)), 2))
            d["life_us_max"].append(round(float(life.max()), 2))
            prev_end = int(st[:, 1].max())
    rows = np.array(rows, dtype=np.int64)
    simds = np.unique(rows[:, 4])
    out["simds_seen"] = int(len(simds))
    # occupancy census over set T's window, every recorded wave in it (T's and its neighbours'):
    # per SIMD, at 400 sample times, the waves resident by kernel
    ts = np.linspace(t_first, t_last, 400)
    sidx = {s: i for i, s in enumerate(simds)}
    occ = np.zeros((len(gpu.STAMP_KERNELS), len(simds), len(ts)), np.int16)
    for ki, ei, s, e_, sk in rows:
        i0, i1 = np.searchsorted(ts, s), np.searchsorted(ts, e_)
        occ[ki, sidx[sk], i0:i1] += 1
    tot = occ.sum(0)
    hist = np.bincount(tot.ravel(), minlength=9)[:12]
    out["simd_wave_census"] = {str(i): round(float(c) / tot.size, 4) for i, c in enumerate(hist) if c}
    out["mean_waves_per_simd"] = round(float(tot.mean()), 3)
    out["kernel_share_of_resident_waves"] = {k: round(float(occ[i].sum()) / max(1, float(tot.sum())), 4)
                                             for i, k in enumerate(gpu.STAMP_KERNELS)}
    # while each recorded launch runs (its span): its own resident waves per SIMD vs everyone's
    own = {}
    for ki, k in enumerate(gpu.STAMP_KERNELS):
        sel = rows[rows[:, 0] == ki]
        vals = []
        for ei in focus:
            r = sel[sel[:, 1] == ei]
            if not len(r):
                continue
            i0, i1 = np.searchsorted(ts, r[:, 2].min()), np.searchsorted(ts, r[:, 3].max())
            if i1 <= i0:
                continue
            mine = np.zeros(i1 - i0)
            for s_, e_ in zip(r[:, 2], r[:, 3]):
                j0, j1 = max(np.searchsorted(ts, s_), i0), min(np.searchsorted(ts, e_), i1)
                mine[j0 - i0:j1 - i0] += 1
            vals.append((float(mine.mean()) / len(simds), float(tot[:, i0:i1].mean())))
        own[k] = {"own_waves_per_simd": [round(v[0], 2) for v in vals],
                  "all_waves_per_simd": [round(v[1], 2) for v in vals]}
    out["during_launch"] = own
    # per SIMD, each focus launch: its waves there and its busy span there (first start -> last
    # end): balance across the chip
    per = {}
    for ki, k in enumerate(gpu.STAMP_KERNELS):
        sel = rows[(rows[:, 0] == ki) & np.isin(rows[:, 1], focus)]
        if not len(sel):
            continue
        keys = sel[:, 1] * (1 << 20) + sel[:, 4]
        uk, inv, cnt = np.unique(keys, return_inverse=True, return_counts=True)
        first = np.full(len(uk), np.iinfo(np.int64).max)
        last = np.zeros(len(uk), np.int64)
        np.minimum.at(first, inv, sel[:, 2])
        np.maximum.at(last, inv, sel[:, 3])
        busy = (last - first) * TICK_US
        life = np.zeros(len(uk))
        np.add.at(life, inv, (sel[:, 3] - sel[:, 2]) * TICK_US)
        per[k] = {"waves_per_simd": {str(int(v)): int(c) for v, c in zip(*np.unique(cnt, return_counts=True))},
                  "simd_span_us_p50": round(float(np.percentile(busy, 50)), 2),
                  "simd_span_us_p90": round(float(np.percentile(busy, 90)), 2),
                  "simd_span_us_max": round(float(busy.max()), 2),
                  "simd_wave_us_sum_p50": round(float(np.percentile(life, 50)), 2),
                  "simd_wave_us_sum_max": round(float(life.max()), 2)}
    out["per_simd"] = per
    # idle SIMD-time within each engine's k_* span: how empty the chip is while a kernel runs
    print(json.dumps({k: out[k] for k in ("engines", "window_us", "simds_seen", "mean_waves_per_simd",
                                           "simd_wave_census", "kernel_share_of_resident_waves", "during_launch",
                                           "per_simd")}))
    for k, d in out["kernels"].items():
        d["wave_us_sum"] = round(d["wave_us_sum"], 1)
        print(f"{k:10s} waves {d['waves']:6d} SIMD-us {d['wave_us_sum']:9.1f} span {d['span_us']} "
              f"delay {d['start_delay_us']} life p50 {d['life_us_p50']} max {d['life_us_max']}")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)
    for e in allc:
        e.close()


if __name__ == "__main__":
    main()

"""Summary of tools/waits.sh: per kernel and variant, the wave cycles (quad-cycles per launch),
the parked (WAIT_ANY) and issue-stalled (WAIT_INST_ANY) shares, the memory instructions per
wave and, where the counters exist, how long an instruction of each class stays outstanding
(LEVEL / INSTS, cycles); then the parked cycles the variants remove:
  structure - baked       = waits on the per-primitive scalar parameter loads (lgkmcnt);
  s - s1 (k_mpu)          = waits in the record passes (LDS / table loads, barriers);
  s - s32 (k_finish)      = waits inside the walks (parameters, culling masks);
what stays in s32 is the records' / keys' / offsets' vector loads and stores (vmcnt) and the
block barriers.  Usage: python tools/waits_summary.py gpurun_out/<tag> [> table]"""
import json
import os
import sys

d = sys.argv[1]
V = {}
for v in ("s", "b", "s1", "s32"):
    p = os.path.join(d, v + ".json")
    if os.path.exists(p):
        V[v] = json.load(open(p))["kernels"]
names = sorted({k for kk in V.values() for k in kk if k.startswith("jit_")})
rows = []
print(f"{'kernel':14s} {'var':4s} {'us':>7s} {'waves':>7s} {'wcyc/w':>8s} {'park':>6s} {'stall':>6s} {'active':>6s} "
      f"{'smem/w':>7s} {'lds/w':>6s} {'vmem/w':>7s} {'vm_lat':>7s} {'sm_lat':>7s} {'lds_lat':>7s}")
for k in names:
    for v, ks in V.items():
        e = ks.get(k)
        if not e or not e.get("SQ_WAVES"):
            continue
        w = e["SQ_WAVES"]
        vmem = e.get("SQ_INSTS_VMEM") or (e.get("SQ_INSTS_VMEM_RD", 0) + e.get("SQ_INSTS_VMEM_WR", 0)) or None

        def lat(level, n):
            return round(4 * e[level] / n, 1) if e.get(level) and n else None  # LEVEL counts quad-cycles
        r = {"kernel": k, "variant": v, "us": e.get("median_us_profiled"), "waves": w,
             "wave_quad_cycles": round(e["SQ_WAVE_CYCLES"] / w, 1),
             "parked": e.get("share_wait_any"), "stalled": e.get("share_wait_inst_any"),
             "active": e.get("share_active_inst_any"),
             "parked_quad_cycles_per_wave": round(e.get("SQ_WAIT_ANY", 0) / w, 1),
             "smem_per_wave": round(e.get("SQ_INSTS_SMEM", 0) / w, 1), "lds_per_wave": round(e.get("SQ_INSTS_LDS", 0) / w, 1),
             "vmem_per_wave": round(vmem / w, 1) if vmem else None,
             "vmem_cycles": lat("SQ_INST_LEVEL_VMEM", vmem), "smem_cycles": lat("SQ_INST_LEVEL_SMEM", e.get("SQ_INSTS_SMEM")),
             "lds_cycles": lat("SQ_INST_LEVEL_LDS", e.get("SQ_INSTS_LDS"))}
        rows.append(r)
        f = lambda x, n=6: (f"{x:>{n}}" if x is not None else " " * (n - 1) + "-")  # noqa: E731
        print(f"{k:14s} {v:4s} {f(r['us'], 7)} {w:7.0f} {r['wave_quad_cycles']:8.0f} {f(r['parked'])} {f(r['stalled'])} "
              f"{f(r['active'])} {r['smem_per_wave']:7.1f} {r['lds_per_wave']:6.1f} {f(r['vmem_per_wave'], 7)} "
              f"{f(r['vmem_cycles'], 7)} {f(r['smem_cycles'], 7)} {f(r['lds_cycles'], 7)}")
# parked quad-cycles per launch removed by each variant
print()
attr = {}
for k in names:
    g = {v: V[v][k].get("SQ_WAIT_ANY") for v in V if k in V[v] and V[v][k].get("SQ_WAIT_ANY") is not None}
    if "s" not in g:
        continue
    a = {"parked_total": g["s"]}
    if "b" in g:
        a["scalar_parameter_loads"] = g["s"] - g["b"]
    if "s1" in g and k == "jit_mpu":
        a["record_passes"] = g["s"] - g["s1"]
    if "s32" in g and k in ("jit_finish", "jit_finish_p", "jit_finish_q"):  # bit 5 ablates k_finish's walks only
        a["walks"] = g["s"] - g["s32"]
        a["records_offsets_stores_barriers"] = g["s32"]
    attr[k] = {n: (round(x / g["s"], 3) if n != "parked_total" else round(x)) for n, x in a.items()}
    print(k, json.dumps(attr[k]))
json.dump({"rows": rows, "parked_share_removed": attr}, open(os.path.join(d, "waits.json"), "w"), indent=1)

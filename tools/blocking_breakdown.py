"""Where the blocking contract's time goes (psgpu_polygonize_mpus on C2): the whole call, then
its pieces on the same context -- model upload (set_model), polygonize + finish, the PolyMPUs
export (download + scatter), and a compact-mesh download alone.  Medians of 20 after warm-up.
CONFIG=C3 for another config; PARTS=2 for the same pieces on a group of 2 parts of device 0
(psgpu_group_polygonize_mpus, the blocking drop-in's default)."""
import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from parsip_amd import gpu, soa, synth  # noqa: E402


def med(f, n=20):
    f()
    t = []
    for _ in range(n):
        t0 = time.perf_counter()
        f()
        t.append(time.perf_counter() - t0)
    return round(float(np.median(t)) * 1e3, 4)


def main_group(parts):
    model, cs, _ = synth.make_config(os.environ.get("CONFIG", "C2"))
    g = gpu.Group([0] * parts)
    g.set_option(gpu.GROUP_OPT_BALANCE, gpu.BALANCE_PLAN)
    g.set_option(gpu.OPT_JIT, 1)
    n = gpu.count_mpus(cs, *model.bbox)
    out = np.zeros(max(soa.MAX_MPU_COUNT, n), soa.MPU_DTYPE)
    L = g._L
    ct = ctypes.c_uint32()
    g.set_model(model)  # waits for the generated kernels
    r = {"parts": parts, "whole": med(lambda: g.polygonize_mpus(cs, model, out))}
    pp, mm, oo = model.ptrs()
    r["set_model"] = med(lambda: L.psgpu_group_set_model(g._g, pp, mm, oo))
    r["polygonize+finish"] = med(lambda: g.run(cs))
    r["export_polympus"] = med(lambda: L.psgpu_group_export_polympus(g._g, out.ctypes.data, len(out),
                                                                     ctypes.byref(ct)))
    g.set_option(gpu.OPT_DEBUG, 1 << 22)  # the export's copies without the scatter
    r["export_copies_only"] = med(lambda: L.psgpu_group_export_polympus(g._g, out.ctypes.data, len(out),
                                                                        ctypes.byref(ct)))
    g.set_option(gpu.OPT_DEBUG, 0)
    print(r, flush=True)
    g.close()


def main():
    if int(os.environ.get("PARTS", "0")):
        return main_group(int(os.environ["PARTS"]))
    model, cs, _ = synth.make_config(os.environ.get("CONFIG", "C2"))
    p = gpu.Polygonizer(0)
    p.set_option(gpu.OPT_JIT, 1)
    out = np.zeros(max(soa.MAX_MPU_COUNT, gpu.count_mpus(cs, *model.bbox)), soa.MPU_DTYPE)
    L = p._L
    ct = ctypes.c_uint32()
    p.set_model(model)  # waits for the generated kernels
    r = {"whole": med(lambda: p.polygonize_mpus(cs, model, out))}
    pp, mm, oo = model.ptrs()
    r["set_model"] = med(lambda: L.psgpu_set_model(p._ctx, pp, mm, oo))
    r["polygonize+finish"] = med(lambda: p.run(cs))
    r["export_polympus"] = med(lambda: L.psgpu_export_polympus(p._ctx, out.ctypes.data, len(out), ctypes.byref(ct)))
    p.set_option(gpu.OPT_DEBUG, 1 << 22)  # the export's copies without the scatter
    r["export_copies_only"] = med(lambda: L.psgpu_export_polympus(p._ctx, out.ctypes.data, len(out), ctypes.byref(ct)))
    p.set_option(gpu.OPT_DEBUG, 0)
    small = np.zeros(ct.value, soa.MPU_DTYPE)
    r["export_into_ctMPUs_buffer"] = med(lambda: L.psgpu_export_polympus(p._ctx, small.ctypes.data, len(small),
                                                                         ctypes.byref(ct)))
    print(r, flush=True)
    p.close()


if __name__ == "__main__":
    main()

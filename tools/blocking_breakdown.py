"""Where the blocking contract's time goes (psgpu_polygonize_mpus on C2): the whole call, then
its pieces on the same context -- model upload (set_model), polygonize + finish, the PolyMPUs
export (download + scatter), and a compact-mesh download alone.  Medians of 20 after warm-up."""
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


def main():
    model, cs, _ = synth.make_config(os.environ.get("CONFIG", "C2"))
    p = gpu.Polygonizer(0)
    out = np.zeros(soa.MAX_MPU_COUNT, soa.MPU_DTYPE)
    L = p._L
    ct = ctypes.c_uint32()
    r = {"whole": med(lambda: p.polygonize_mpus(cs, model, out))}
    pp, mm, oo = model.ptrs()
    r["set_model"] = med(lambda: L.psgpu_set_model(p._ctx, pp, mm, oo))
    r["polygonize+finish"] = med(lambda: p.run(cs))
    r["export_polympus"] = med(lambda: L.psgpu_export_polympus(p._ctx, out.ctypes.data, len(out), ctypes.byref(ct)))
    r["download_mesh"] = med(lambda: p.download())
    small = np.zeros(ct.value, soa.MPU_DTYPE)
    r["export_into_ctMPUs_buffer"] = med(lambda: L.psgpu_export_polympus(p._ctx, small.ctypes.data, len(small),
                                                                         ctypes.byref(ct)))
    print(r, flush=True)
    p.close()


if __name__ == "__main__":
    main()

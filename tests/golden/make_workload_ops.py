"""Generate tests/golden/workload_ops.json: the reference algorithm's fp32 operation count
per kernel of one polygonization, for bench.py's roofline `achieved` figure.

The oracle (oracle/psoracle.c) counts, per phase, what the reference executes on the
benchmark inputs: primitive evaluations by type (after its depth>3 op-box pruning),
matrices applied, box tests, op evaluations by type and colour-pass steps.  Each count is
priced with parsip_amd/costmodel.py (ops per lane-evaluation, contraction off).  Phases
map to kernels: S1 -> k_precheck, S2 -> k_mpu, root + normal samples -> k_vertex,
fieldValueAndColor -> k_finish.

Usage: python tests/golden/make_workload_ops.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]

import psoracle  # noqa: E402

from parsip_amd import costmodel, synth  # noqa: E402

COLOUR_STEP = 13  # weights (<= 4) + 3 x (2 mul + 1 add)


def phase_ops(row) -> int:
    ops = 0
    for t in range(16):
        ops += int(row[t]) * costmodel.PRIM_OPS.get(t, costmodel.WYVILL)
    ops += int(row[16]) * 18 + int(row[17]) * costmodel.BOX_TEST + int(row[18]) * COLOUR_STEP
    for t in range(32):
        ops += int(row[32 + t]) * costmodel.OP_OPS.get(t, 0)
    return ops


out = {"generator": "tests/golden/make_workload_ops.py (oracle work counters x parsip_amd/costmodel.py)",
       "note": "fp32 operations the reference algorithm executes per polygonization, by kernel"}
for name in ("C2", "C3", "C5"):
    model, cs, n = synth.make_config(name)
    om = psoracle.polygonize(model, cs, threads=os.cpu_count() or 1, keep=False, count=True)
    c = psoracle.work_counts()
    ph = {p: phase_ops(c[i]) for i, p in enumerate(psoracle.PHASES)}
    prim_evals = {p: int(c[i][:16].sum()) for i, p in enumerate(psoracle.PHASES)}
    out[name] = {"k_precheck": ph["s1"], "k_mpu": ph["s2"], "k_vertex": ph["roots"] + ph["normals"],
                 "k_finish": ph["colour"], "prim_evals": prim_evals,
                 "vertices": int(om.stats[:, 2].sum()), "passed_s1": int(om.stats[:, 0].sum())}
    print(name, out[name])
with open(os.path.join(HERE, "workload_ops.json"), "w") as f:
    json.dump(out, f, indent=1)

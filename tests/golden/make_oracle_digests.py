"""Generate tests/golden/oracle_digests.json: SHA-256 digests of the oracle's full output
(per-MPU stats, positions, normals, colours, MPU-local triangles) for C1, C2 and C3.

The oracle itself is pinned by tests/golden/reference_probe.json (counts recorded from the
reference) and tritable.json; these digests freeze its bits so the GPU tests can check the
full-size meshes without re-running the oracle, and so any oracle change is noticed.
NaNs are canonicalised before hashing (x86 and CDNA default-NaN payloads differ).

Usage: python tests/golden/make_oracle_digests.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]

import psoracle  # noqa: E402
from parity_util import mesh_digests  # noqa: E402

from parsip_amd import synth  # noqa: E402

out = {"generator": "oracle/psoracle.c (IEEE build), parsip_amd.synth.make_config(name) defaults"}
for name in ("C1", "C2", "C3"):
    model, cs, n = synth.make_config(name)
    om = psoracle.polygonize(model, cs, threads=os.cpu_count() or 1)
    out[name] = mesh_digests(om.stats[:, :4], om.pos, om.nrm, om.col, om.tris)
    print(name, out[name]["vertices"], out[name]["triangles"])
with open(os.path.join(HERE, "oracle_digests.json"), "w") as f:
    json.dump(out, f, indent=1)

"""Generate tests/golden/tritable.json: digests of the reference's marching-cubes table.

Reads (as text) Parsip100/PS_SimdPoly/include/_CellConfigTable.h from the read-only
reference checkout, parses g_triTableCache[256][16], corner1/corner2/edgeaxis, and stores
only SHA-256 digests of their little-endian int32 bytes plus per-config triangle counts.
No reference source is copied; the library and the oracle generate their tables
algorithmically and the tests compare digests.

Usage: python tests/golden/make_tritable_digest.py [/root/reference]
"""
import hashlib
import json
import os
import re
import sys

import numpy as np

ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
path = os.path.join(ref, "Parsip100/PS_SimdPoly/include/_CellConfigTable.h")
txt = open(path).read()


def int_array(name, n):
    m = re.search(name + r"\[\d+\]\s*=\s*\{([^}]*)\}", txt)
    sym = {k: v for v, k in enumerate(["LBN", "LBF", "LTN", "LTF", "RBN", "RBF", "RTN", "RTF"])}
    sym.update({"AAX": 0, "AAY": 1, "AAZ": 2})
    vals = [sym[t.strip()] if t.strip() in sym else int(t) for t in m.group(1).split(",")]
    assert len(vals) == n
    return np.array(vals, np.int32)


body = txt[txt.index("g_triTableCache"):]
rows = re.findall(r"\{([-0-9, ]+)\}", body)[:256]
table = np.array([[int(x) for x in r.split(",")] for r in rows], np.int32)
assert table.shape == (256, 16)
out = {
    "source": "Parsip100/PS_SimdPoly/include/_CellConfigTable.h (g_triTableCache, corner1, corner2, edgeaxis)",
    "tritable_sha256": hashlib.sha256(table.astype("<i4").tobytes()).hexdigest(),
    "corner1_sha256": hashlib.sha256(int_array("corner1", 12).astype("<i4").tobytes()).hexdigest(),
    "corner2_sha256": hashlib.sha256(int_array("corner2", 12).astype("<i4").tobytes()).hexdigest(),
    "edgeaxis_sha256": hashlib.sha256(int_array("edgeaxis", 12).astype("<i4").tobytes()).hexdigest(),
    "triangles_per_config": [int((r >= 0).sum() // 3) for r in table],
}
dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tritable.json")
with open(dst, "w") as f:
    json.dump(out, f, indent=1)
print(dst, out["tritable_sha256"])

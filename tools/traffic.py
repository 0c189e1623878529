"""Per-kernel HBM traffic per launch from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE)
and the kernel-trace stats, following MI355X_MICROARCH.md "HBM": FETCH_SIZE / WRITE_SIZE
are KiB; FETCH_SIZE is doubled on gfx950 (it tallies 128-B read requests at 64 B).
Usage: python tools/traffic.py gpurun_out/<tag> [JIT]  -> JSON on stdout (JIT: the bench's --jit of
the profiled command, recorded as "jit" so bench.py pairs the file with the tier it timed)."""
import collections
import csv
import glob
import json
import os
import sys

d = sys.argv[1]


def pmc(sub, counter):
    paths = glob.glob(os.path.join(d, sub, "**", "*counter_collection.csv"), recursive=True)
    acc = collections.defaultdict(list)
    for p in paths:
        for r in csv.DictReader(open(p)):
            if r["Counter_Name"] == counter:
                acc[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def stats():
    paths = glob.glob(os.path.join(d, "kt", "**", "*kernel_stats.csv"), recursive=True)
    out = {}
    for p in paths:
        for r in csv.DictReader(open(p)):
            out[r["Name"].split("(")[0]] = {"calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3,
                                            "pct": float(r["Percentage"])}
    return out


fetch, write = pmc("fetch", "FETCH_SIZE"), pmc("write", "WRITE_SIZE")
res = {"note": "bytes per launch; read = 2 x FETCH_SIZE (gfx950 correction), write = WRITE_SIZE; KiB -> B",
       "kernels": {}}
if len(sys.argv) > 2:
    res["jit"] = int(sys.argv[2])
st = stats()
for k in sorted(set(fetch) | set(write) | set(st)):
    if "rocclr" in k or "__amd" in k:
        continue
    e = {}
    if k in fetch:
        e["read_bytes"] = 2 * fetch[k] * 1024
    if k in write:
        e["write_bytes"] = write[k] * 1024
    if "read_bytes" in e and "write_bytes" in e:
        e["traffic_bytes"] = e["read_bytes"] + e["write_bytes"]
    if k in st:
        e.update(st[k])
    res["kernels"][k] = e
print(json.dumps(res, indent=1))

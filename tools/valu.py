"""Per-kernel VALU instruction counts per launch from a rocprofv3 PMC pass
(--pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES) -> JSON on stdout (profiles/<tag>_valu.json).
Usage: python tools/valu.py gpurun_out/<tag>/valu"""
import collections
import csv
import glob
import json
import os
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(list))
for p in glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(p)):
        acc[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {"note": "per launch, averaged over the profiled launches; VALU issue utilisation = "
               "SQ_INSTS_VALU x 2 cycles (wave64 on SIMD-32) / (kernel time x 2.4 GHz x 1024 SIMDs)", "kernels": {}}
for k, d in acc.items():
    if "rocclr" in k or "__amd" in k:
        continue
    out["kernels"][k] = {c: sum(v) / len(v) for c, v in d.items()}
print(json.dumps(out, indent=1))
